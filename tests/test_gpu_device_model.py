"""Device-side grad log p for the built-in Gaussian-sum models (SURVEY §8(f)
rank 1; MultivariateNormal.hpp:56-61, Model::operator+ Model.hpp:55-92).

The device kernel evaluates the same closed form in the same operation order
as the C++ host model, so the gradients agree to fp64 rounding (tolerance
1e-13 relative + 1e-14 absolute), and a fully device-resident step
(svgd_step(ctx, NULL)) follows the host-gradient step to 1e-12."""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _model(oracle, d, k, seed):
    mus = oracle.splitmix((k, d), 3.0, seed)
    rng = np.random.default_rng(seed)
    covs = []
    for _ in range(k):
        A = rng.standard_normal((d, d)) * 0.3
        covs.append(A @ A.T + np.eye(d) * (1.0 + rng.random()))
    return S.GaussianSum(list(mus), covs)


@pytest.mark.parametrize("d,k", [(1, 1), (2, 1), (8, 4), (9, 3), (16, 2), (32, 2)])
def test_device_gradient_matches_host_model(oracle, d, k):
    n = 1000
    X = oracle.splitmix((n, d), 4.0, 3)
    model = _model(oracle, d, k, 17 + d)
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_device_model(model)
    Gd = c.device_logp_grad()
    Gh = model.log_model_grad(X)
    np.testing.assert_allclose(Gd, Gh, rtol=1e-13, atol=1e-14)
    # and against the oracle's independent restatement (log-sum-exp)
    Go = oracle.logp_grad_gmm(X, np.stack(model.means_), np.stack(model.covs_))
    np.testing.assert_allclose(Gd, Go, rtol=1e-11, atol=1e-12)


def test_device_step_follows_host_gradient_step(oracle):
    n, d, steps = 2500, 8, 5
    X0 = oracle.splitmix((n, d), 3.0, 9)
    model = _model(oracle, d, 4, 5)
    runs = []
    for device in (False, True):
        c = S.Context(d, n)
        c.set_particles(X0)
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
        if device:
            c.set_device_model(model)
        for _ in range(steps):
            c.step_device() if device else c.step_with_model(model)
        runs.append((c.get_particles(), c.last_scale()[0]))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=0, atol=1e-12)
    assert runs[1][1] == pytest.approx(runs[0][1], rel=1e-13)


def test_device_step_without_model_is_an_argument_error(oracle):
    c = S.Context(2, 10)
    c.set_particles(oracle.splitmix((10, 2), 1.0, 1))
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    with pytest.raises(ValueError):
        c.step_device()
    with pytest.raises(S.DimensionMismatchException):
        c.set_device_model(_model(oracle, 3, 1, 2))
