"""The fp32 accuracy of the F32 path's bf16 emulation, pinned on the GPU.  GPU only.

For 16 < d <= 64 the F32 path forms every fp32 product on the bf16 matrix
cores: k_phi_b3 (phi_hat) splits each fp32 operand into three bf16 parts and
sums six part products; k_pair_tcol3 (the median keys, also every debug /
sample key pass) defines the pair key by the same six-part Gram
(svgd_device.h).  The CPU emulation proves a 2^-22 relative
bound per product (tests/test_b3_split.py); these tests check that the
shipped kernels deliver fp32 accuracy, not the coarser bf16x3 one, by
comparing their error against the fp64 oracle with the error of real fp32
arithmetic on the same inputs:

  * phi_hat: err(k_phi_b3) <= max(2 err(k_phi_f32s), 2e-6 max|phi_hat|), both
    against the oracle's fp64 phi_hat (SVGD.hpp:407-454) from identical
    (X, G, a), a the median heuristic's scale (GaussianRBFKernel.hpp:168-188);
    k_phi_f32s is the fp32-MFMA kernel (v_mfma_f32_16x16x4f32);
  * keys: max over all pairs of |key - D^2| / (|xc_i|^2 + |xc_j|^2), the
    device's six-part keys (svgd_debug_pair_keys) against fp32 keys from an
    fp32 Gram (numpy sgemm on the same fp32 coordinates): <= 2x + 2^-22;
  * cfg5's full size (N = 65536, d = 64): phi_hat on 1024 sampled rows, the
    same bar.
The observed errors are printed (pytest -s) and the cfg5 bench line records
its own (cpu_baseline.accuracy).
"""
import numpy as np
import pytest

import bench
import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _phi(monkeypatch, X, G, a, b3):
    n, d = X.shape
    monkeypatch.setenv("SVGD_PHI_B3", "1" if b3 else "0")
    c = S.Context(d, n, dtype=C.SVGD_F32)
    c.set_particles(X)
    name = c.phi_kernel_name()
    assert name.startswith("k_phi_b3" if b3 else "k_phi_f32s"), name
    ph = c.phi(G, a)
    c.close()
    return ph


@pytest.mark.parametrize("n,d", [(2049, 32), (3001, 33), (1000, 64), (4096, 64), (1500, 48)])
def test_b3_phi_error_within_fp32(oracle, monkeypatch, n, d):
    X = oracle.splitmix((n, d), 3.0, 900 + n + d)
    mus = oracle.splitmix((1, d), 0.5, 901 + d)
    G = oracle.logp_grad_gmm(X, mus, np.eye(d)[None])
    a, _ = oracle.median_scale(X)
    ref = oracle.phi(X, G, a)
    scale = np.max(np.abs(ref))
    e_b3 = np.max(np.abs(_phi(monkeypatch, X, G, a, True) - ref))
    e_f32 = np.max(np.abs(_phi(monkeypatch, X, G, a, False) - ref))
    print(f"n={n} d={d}: b3 {e_b3 / scale:.3e} f32s {e_f32 / scale:.3e} (x max|phi|)")
    assert e_b3 <= max(2.0 * e_f32, 2e-6 * scale), (e_b3 / scale, e_f32 / scale)


@pytest.mark.parametrize("n,d", [(1500, 32), (1200, 64), (999, 40)])
def test_b3_keys_error_within_fp32(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 950 + n + d)
    c = S.Context(d, n, dtype=C.SVGD_F32)
    c.set_particles(X)
    keys = np.empty(n * (n - 1) // 2)
    c.check(c.lib.svgd_debug_pair_keys(c.h, C.dptr(keys), keys.size))
    c.close()
    xc = X - X.mean(axis=0)
    nrm = (xc * xc).sum(axis=1)
    iu = np.triu_indices(n, 1)
    exact = ((xc[iu[0]] - xc[iu[1]]) ** 2).sum(axis=1)
    den = nrm[iu[0]] + nrm[iu[1]]
    # fp32-direct keys: fp32 coordinates and norms, an fp32 Gram
    x32 = xc.astype(np.float32)
    n32 = nrm.astype(np.float32)
    gram = x32 @ x32.T
    k32 = np.maximum(n32[iu[0]] + n32[iu[1]] - np.float32(2.0) * gram[iu], np.float32(0.0)).astype(np.float64)
    e_dev = np.max(np.abs(keys - exact) / den)
    e_32 = np.max(np.abs(k32 - exact) / den)
    print(f"n={n} d={d}: keys b3 {e_dev:.3e} fp32 {e_32:.3e} (x (|xc_i|^2 + |xc_j|^2))")
    assert e_dev <= 2.0 * e_32 + 2.0 ** -22, (e_dev, e_32)


def test_b3_phi_cfg5_fullsize_sampled_rows(oracle, monkeypatch):
    n, d = 65536, 64
    X, mus, covs = bench.config_workload("cfg5", n, d, 1)
    model = S.GaussianSum(list(mus), list(covs))
    G = model.log_model_grad(X)
    monkeypatch.setenv("SVGD_PHI_B3", "1")
    c = S.Context(d, n, dtype=C.SVGD_F32)
    c.set_particles(X)
    a, _ = c.median_scale()
    ph = {True: c.phi(G, a)}
    c.close()
    ph[False] = _phi(monkeypatch, X, G, a, False)
    err = {True: 0.0, False: 0.0}
    scale = 0.0
    for r0, r1 in bench.accuracy_rows(n):
        ref = oracle.phi(X, G, a, rows=(r0, r1))
        scale = max(scale, np.max(np.abs(ref)))
        for k in err:
            err[k] = max(err[k], np.max(np.abs(ph[k][r0:r1] - ref)))
    print(f"cfg5 rows: b3 {err[True] / scale:.3e} f32s {err[False] / scale:.3e} (x max|phi|)")
    assert err[True] <= max(2.0 * err[False], 2e-6 * scale), (err[True] / scale, err[False] / scale)
