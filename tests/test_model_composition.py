"""Model composition over closed forms (svgdcpp_amd.api.Model), following the
reference's tests/test_model.cpp:186-315: + - * / of function models, the
Evaluate* family (value, log, gradient, Hessian and their log forms), the
dimension-mismatch and unset-function errors, and parameter routing through a
composition.  The expected values are the closed forms the reference's test
writes out; derivatives of compositions are checked by central differences."""
import math

import numpy as np
import pytest

from svgdcpp_amd import api


def linear_fun(x, p):  # test_model.cpp linear_fun: sum(a .* x)
    return float(np.sum(p[0].reshape(-1) * x))


def linear_grad(x, p):
    return p[0].reshape(-1).copy()


def linear_hess(x, p):
    return np.zeros((x.size, x.size))


def squared_fun(x, p):  # x^T B x
    return float(x @ p[1] @ x)


def squared_grad(x, p):
    return (p[1] + p[1].T) @ x


def squared_hess(x, p):
    return p[1] + p[1].T


def sum_fun(x, p):  # 2 sum(x) (test_model.cpp:199-205)
    return 2.0 * float(np.sum(x))


def sum_grad(x, p):
    return np.full(x.size, 2.0)


def sum_hess(x, p):
    return np.zeros((x.size, x.size))


PARAMS = [np.array([1.5, 0.7]), np.array([[2.0, 0.3], [0.1, 1.2]])]
X_LOW = np.array([0.9, 1.4])
X_HIGH = np.array([0.3, 1.1, 0.6, 0.2, 0.8])


def _model(dim, f, g, h, params=None):
    m = api.Model(dim)
    m.UpdateModel(f, g, h)
    if params is not None:
        m.UpdateParameters(params)
    m.Initialize()
    return m


def _fd_grad(f, x, eps=1e-6):
    g = np.empty_like(x)
    for k in range(x.size):
        e = np.zeros_like(x)
        e[k] = eps
        g[k] = (f(x + e) - f(x - e)) / (2 * eps)
    return g


def _fd_hess(gf, x, eps=1e-6):
    H = np.empty((x.size, x.size))
    for k in range(x.size):
        e = np.zeros_like(x)
        e[k] = eps
        H[:, k] = (gf(x + e) - gf(x - e)) / (2 * eps)
    return H


def test_composition_operators():  # test_model.cpp:186-234
    low = _model(2, linear_fun, linear_grad, linear_hess, PARAMS)
    high = _model(5, sum_fun, sum_grad, sum_hess)
    with pytest.raises(api.DimensionMismatchException):
        low + high
    with pytest.raises(api.DimensionMismatchException):
        low * high
    low2 = _model(2, squared_fun, squared_grad, squared_hess, PARAMS)
    high2 = _model(5, sum_fun, sum_grad, sum_hess)
    lin = float(np.sum(PARAMS[0] * X_LOW))
    sq = float(X_LOW @ PARAMS[1] @ X_LOW)
    assert (low + low).EvaluateModel(X_LOW) == pytest.approx(2 * lin)
    assert (low + low2).EvaluateModel(X_LOW) == pytest.approx(lin + sq)
    assert (low2 - low).EvaluateModel(X_LOW) == pytest.approx(sq - lin)
    assert (high * high).EvaluateModel(X_HIGH) == pytest.approx(4 * X_HIGH.sum() ** 2)
    assert (high / high2).EvaluateModel(X_HIGH) == pytest.approx(1.0)


def test_unset_function_refused():
    with pytest.raises(api.UnsetException):
        api.Model(2) + _model(2, linear_fun, linear_grad, linear_hess, PARAMS)


@pytest.mark.parametrize("op", ["+", "-", "*", "/"])
def test_composed_derivatives(op):  # the Evaluate* family on compositions (:246-315)
    a = _model(2, squared_fun, squared_grad, squared_hess, PARAMS)
    b = _model(2, linear_fun, linear_grad, linear_hess, PARAMS)
    m = {"+": a + b, "-": a - b, "*": a * b, "/": a / b}[op]
    x = X_LOW
    f = m.EvaluateModel
    np.testing.assert_allclose(m.EvaluateModelGrad(x), _fd_grad(f, x), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(m.EvaluateModelHessian(x), _fd_hess(m.EvaluateModelGrad, x),
                               rtol=1e-5, atol=1e-6)
    assert m.EvaluateLogModel(x) == pytest.approx(math.log(f(x)))
    np.testing.assert_allclose(m.EvaluateLogModelGrad(x), _fd_grad(m.EvaluateLogModel, x), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(m.EvaluateLogModelHessian(x), _fd_hess(m.EvaluateLogModelGrad, x),
                               rtol=1e-5, atol=1e-6)


def test_evaluate_family_closed_forms():  # test_model.cpp:269-315
    low = _model(2, linear_fun, linear_grad, linear_hess, PARAMS)
    sq = _model(2, squared_fun, squared_grad, squared_hess, PARAMS)
    x = X_LOW
    lin, g = float(np.sum(PARAMS[0] * x)), PARAMS[0]
    assert low.EvaluateLogModel(x) == pytest.approx(math.log(lin))
    np.testing.assert_allclose(low.EvaluateLogModelGrad(x), g / lin)
    np.testing.assert_allclose(low.EvaluateLogModelHessian(x), -np.outer(g, g) / lin ** 2)
    B = PARAMS[1]
    v, gs = float(x @ B @ x), (B + B.T) @ x
    np.testing.assert_allclose(sq.EvaluateLogModelHessian(x), (B + B.T) / v - np.outer(gs, gs) / v ** 2)


def test_parameters_route_through_composition():  # Model.hpp:70-74, 377-406
    a = _model(2, linear_fun, linear_grad, linear_hess, PARAMS)
    b = _model(2, squared_fun, squared_grad, squared_hess, PARAMS)
    m = a * b
    assert len(m.GetParameters()) == 4
    newp = [np.array([0.2, 3.0]), np.eye(2), np.array([1.0, 1.0]), np.array([[1.0, 0.5], [0.5, 2.0]])]
    m.UpdateParameters(newp)
    x = X_LOW
    assert m.EvaluateModel(x) == pytest.approx(float(np.sum(newp[0] * x)) * float(x @ newp[3] @ x))
    with pytest.raises(api.DimensionMismatchException):
        m.UpdateParameters(newp[:3])
    # the operands are copies (Model.hpp:70-81; tests/cpp/test_api.cpp): the
    # update leaves a and b, and other compositions of them, untouched
    assert a.EvaluateModel(x) == pytest.approx(float(np.sum(PARAMS[0].reshape(-1) * x)))
    assert b.EvaluateModel(x) == pytest.approx(float(x @ PARAMS[1] @ x))
    m2 = a + b
    c2 = m2 * a  # a composition of a composition
    m2.UpdateParameters(newp)
    assert a.GetParameters()[0].tolist() == PARAMS[0].tolist()
    assert c2.EvaluateModel(x) == pytest.approx((float(np.sum(PARAMS[0].reshape(-1) * x)) + float(x @ PARAMS[1] @ x))
                                                * float(np.sum(PARAMS[0].reshape(-1) * x)))
    # a copy of a composition keeps its parameters when the original's change
    m3 = a * b
    m3b = api._clone_model(m3)
    m3.UpdateParameters(newp)
    assert m3b.EvaluateModel(x) == pytest.approx(a.EvaluateModel(x) * b.EvaluateModel(x))


def test_gaussian_operands():
    """Gaussian + Gaussian stays the batched Gaussian form; Gaussian times a
    function model composes, and its log-gradient is the sum of the factors'."""
    g1 = api.MultivariateNormal([0.0, 1.0], [[1.0, 0.2], [0.2, 0.8]])
    g2 = api.MultivariateNormal([1.0, -1.0], [[0.5, 0.0], [0.0, 2.0]])
    s = g1 + g2
    assert isinstance(s, api.GaussianSum)
    x = np.array([0.4, -0.3])
    p = g1.EvaluateModel(x) + g2.EvaluateModel(x)
    assert s.EvaluateModel(x) == pytest.approx(p)
    np.testing.assert_allclose(g1.EvaluateModelGrad(x), _fd_grad(g1.EvaluateModel, x), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(g1.EvaluateModelHessian(x), _fd_hess(g1.EvaluateModelGrad, x), rtol=1e-5, atol=1e-8)
    sq = _model(2, squared_fun, squared_grad, squared_hess, PARAMS)
    m = g1 * sq
    assert not isinstance(m, api.GaussianSum)
    np.testing.assert_allclose(m.EvaluateLogModelGrad(x), g1.EvaluateLogModelGrad(x) + sq.EvaluateLogModelGrad(x),
                               rtol=1e-10)
    X = np.stack([x, x + 0.1])
    np.testing.assert_allclose(m.log_model_grad(X)[1], m.EvaluateLogModelGrad(x + 0.1), rtol=1e-12)
    assert len(s.GetParameters()) == 4
    s.UpdateParameters(g2.GetParameters() + g1.GetParameters())
    assert s.EvaluateModel(x) == pytest.approx(p)
    # a Gaussian operand of a composition is copied (its own C++ host model)
    m.UpdateParameters([np.array([3.0, 3.0]), np.eye(2)] + sq.GetParameters())
    np.testing.assert_allclose(g1.log_model_grad(x[None])[0],
                               -np.linalg.solve([[1.0, 0.2], [0.2, 0.8]], x - np.array([0.0, 1.0])), rtol=1e-12)
    np.testing.assert_allclose(m.EvaluateLogModelGrad(x), -(x - 3.0) + sq.EvaluateLogModelGrad(x), rtol=1e-10)
