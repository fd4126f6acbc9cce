"""svgd_step_host_model: the X_t copy, the host gradient and the G upload
pipelined in row chunks (SVGD.hpp:373-400 with Model::EvaluateLogModelGrad,
Model.hpp:335-338).  GPU only.

The pipelined step must give the same trajectory, bit for bit, as the split
begin / gradient / finish calls (the same kernels on the same G), and match
the oracle's SVGD::Step.
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _ctx(X, dtype=C.SVGD_F64):
    n, d = X.shape
    c = S.Context(d, n, dtype=dtype)
    c.set_particles(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    return c


@pytest.mark.parametrize("n,d,k,dtype", [(1500, 3, 2, C.SVGD_F64), (9000, 8, 4, C.SVGD_F64),
                                         (20000, 2, 1, C.SVGD_F64), (5000, 64, 1, C.SVGD_F32)])
def test_pipelined_step_matches_split_step(oracle, n, d, k, dtype):
    X = oracle.splitmix((n, d), 3.0, n + d + k)
    mus = oracle.splitmix((k, d), 2.0, 11)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    a, b = _ctx(X, dtype), _ctx(X, dtype)
    for step in range(4):
        a.step_with_model(model, pipelined=True)
        b.step_with_model(model, pipelined=False)
        assert np.array_equal(a.get_particles(), b.get_particles()), step
        assert a.last_scale()[:2] == b.last_scale()[:2], step
    a.close()
    b.close()


def test_pipelined_step_matches_oracle(oracle):
    n, d = 6000, 8
    X = oracle.splitmix((n, d), 3.0, 21)
    mus = oracle.splitmix((4, d), 3.0, 22)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(4)])
    model = S.GaussianSum(list(mus), list(covs))
    c = _ctx(X)
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    Xr = X.copy()
    for _ in range(3):
        a_ref, _ = oracle.median_scale(Xr)
        G = oracle.logp_grad_gmm(Xr, mus, covs)
        c.step_with_model(model)
        a_dev = c.last_scale()[0]
        assert a_dev == pytest.approx(a_ref, rel=1e-12)
        oracle.apply_update(Xr, opt.step(oracle.phi(Xr, G, a_dev)))
        assert np.max(np.abs(c.get_particles() - Xr)) <= 1e-9
    c.close()


def test_pipelined_step_rejects_bad_model():
    X = np.zeros((100, 3))
    c = _ctx(X)
    other = S.GaussianSum([np.zeros(4)], [np.eye(4)])
    with pytest.raises(ValueError):
        c.step_with_model(other)
    c.close()
