"""The bracket collect pass on the matrix cores (k_pair_mcol).  GPU only.

k_pair_mcol classifies every pair from an fp32 MFMA Gram product against
per-row thresholds widened by a proven fp32 error bound, and forms the exact
fp64 key (k_pair_rows' arithmetic) only for the undecided band.  Its outputs
must make the median selection BIT-IDENTICAL to the all-fp64 collect pass
(SVGD_COLLECT_FP64=1, k_pair_rows MODE 0) and to the exact order statistics of
the device's own keys (svgd_debug_pair_keys), including diagonal tiles, ragged
n, every d <= 16, and the pathological inputs whose band outgrows the staging
area (ties, huge or tiny coordinates: the region is reported overflowed and
the exact streamed fallback selects).  GaussianRBFKernel.hpp:164-188, 222-254.

The sample (2^16 pairs, 3 sigma) keeps the bracket under the 2 % band share
above which the library takes k_pair_rows' collect instead.

For d <= 8 the Gram is split bf16 by default (one v_mfma_f32_16x16x32_bf16 per
16 x 16 block, a wider proven margin); SVGD_MCOL_BF16=0 selects the f32 Gram.
Both are checked against the same fp64 collect and exact statistics.
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _median(X, monkeypatch, fp64, sample=1 << 16, bf16=True):
    monkeypatch.setenv("SVGD_COLLECT_FP64", "1" if fp64 else "0")
    monkeypatch.setenv("SVGD_MCOL_BF16", "1" if bf16 else "0")
    n, d = X.shape
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_median_tuning(direct_max_pairs=0, sample_size=sample)  # force the bracket path
    a, med = c.median_scale()
    out = (a, med, c.last_scale()[2], c.last_median_keys())
    return c, out


def _exact_median(c, n):
    """Exact order statistics of the device's own keys (all n(n-1)/2 pairs)."""
    keys = np.empty(n * (n - 1) // 2)
    c.check(c.lib.svgd_debug_pair_keys(c.h, C.dptr(keys), keys.size))
    u = np.sort(keys)
    tot = n * n

    def at(k):
        return 0.0 if k < n else np.sqrt(u[(k - n) // 2])
    return (at(tot // 2 - 1) + at(tot // 2)) / 2 if tot % 2 == 0 else at(tot // 2)


@pytest.mark.parametrize("bf16", [True, False], ids=["bf16", "f32"])
@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 8, 12, 16])
@pytest.mark.parametrize("n", [300, 1000, 2049, 4097])
def test_mcol_matches_fp64_collect_and_exact(oracle, monkeypatch, n, d, bf16):
    if not bf16 and d > 8:
        pytest.skip("d > 8 always takes the f32 Gram")
    X = oracle.splitmix((n, d), 3.0, 7 * n + d)
    c, got = _median(X, monkeypatch, fp64=False, bf16=bf16)
    assert got[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET), got
    exp = _exact_median(c, n)
    c.close()
    f, ref = _median(X, monkeypatch, fp64=True)
    f.close()
    assert got[:2] == ref[:2] and got[3] == ref[3]  # same keys, bit for bit
    assert got[1] == exp


@pytest.mark.parametrize("bf16", [True, False], ids=["bf16", "f32"])
@pytest.mark.parametrize("kind", ["ties", "huge", "tiny", "outlier"])
def test_mcol_pathological_inputs_exact(oracle, monkeypatch, kind, bf16):
    """Bands the fp32 classification cannot narrow: the result is still exact."""
    n, d = 1500, 8
    X = oracle.splitmix((n, d), 1.0, 99)
    if kind == "ties":
        X = np.repeat(X[:6], n // 6, axis=0)  # six distinct points
    elif kind == "huge":
        X = X * 1e22  # |x|^2 > 2^40: no fp32 classification at all
    elif kind == "tiny":
        X = X * 1e-25  # fp32 products underflow: everything undecided
    else:
        X[17] = 1e6  # one far particle widens every threshold
    n = X.shape[0]
    c, got = _median(X, monkeypatch, fp64=False, bf16=bf16)
    exp = _exact_median(c, n)
    c.close()
    f, ref = _median(X, monkeypatch, fp64=True)
    f.close()
    assert got[1] == exp
    assert got[:2] == ref[:2]


@pytest.mark.parametrize("n,d", [(20011, 8), (16384, 2)])
def test_mcol_large_matches_fp64_collect(oracle, monkeypatch, n, d):
    """Default sample sizes (no tuning) at sizes where the bracket path is the default."""
    X = oracle.splitmix((n, d), 3.0, n + d)
    res = []
    for fp64, bf16 in ((False, True), (False, False), (True, True)):
        monkeypatch.setenv("SVGD_COLLECT_FP64", "1" if fp64 else "0")
        monkeypatch.setenv("SVGD_MCOL_BF16", "1" if bf16 else "0")
        c = S.Context(d, n)
        c.set_particles(X)
        a, med = c.median_scale()
        res.append((a, med, c.last_median_keys()))
        assert c.last_scale()[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)
        c.close()
    assert res[0] == res[2] and res[1] == res[2]


# ---------------------------------------------------------------- fp32 tiles --
# k_pair_tcol: the fp32 tile path's collect (SVGD_F32, any d) on the matrix
# cores with k_pair_tiles<float>'s own key arithmetic.  Its median must be
# BIT-IDENTICAL to k_pair_tiles MODE 0 (SVGD_COLLECT_FP64=1) and to the exact
# order statistics of the device's own fp32 keys.

def _median32(X, monkeypatch, ref, sample=0, direct=None):
    monkeypatch.setenv("SVGD_COLLECT_FP64", "1" if ref else "0")
    n, d = X.shape
    c = S.Context(d, n, dtype=C.SVGD_F32)
    c.set_particles(X)
    kw = {"direct_max_pairs": 0} if direct is None else {"direct_max_pairs": direct}
    if sample:
        kw["sample_size"] = sample
    c.set_median_tuning(**kw)
    a, med = c.median_scale()
    return c, (a, med, c.last_scale()[2], c.last_median_keys())


@pytest.mark.parametrize("d", [2, 7, 16, 20, 33, 64])
@pytest.mark.parametrize("n", [300, 1000, 4097])
def test_tcol_matches_tile_collect_and_exact(oracle, monkeypatch, n, d):
    X = oracle.splitmix((n, d), 3.0, 11 * n + d)
    c, got = _median32(X, monkeypatch, ref=False)
    exp = _exact_median(c, n)
    c.close()
    f, ref = _median32(X, monkeypatch, ref=True)
    f.close()
    assert got == ref  # same keys and counts: the same path, bit for bit
    assert got[1] == exp


@pytest.mark.parametrize("kind", ["ties", "zeros", "outlier", "direct"])
def test_tcol_edge_inputs_exact(oracle, monkeypatch, kind):
    """Ties (a wide band of equal keys), all-zero distances (lo key 0), one far
    particle, and the direct path (every pair a candidate: bracket [0, inf))."""
    n, d = 1500, 64
    X = oracle.splitmix((n, d), 1.0, 5)
    direct = None
    if kind == "ties":
        X = np.repeat(X[:6], n // 6, axis=0)
    elif kind == "zeros":
        X = np.zeros((n, d))
        X[:10] = 1.0
    elif kind == "outlier":
        X[17] = 1e6
    else:
        direct = 1 << 40
    n = X.shape[0]
    c, got = _median32(X, monkeypatch, ref=False, direct=direct)
    exp = _exact_median(c, n)
    c.close()
    f, ref = _median32(X, monkeypatch, ref=True, direct=direct)
    f.close()
    assert got[1] == exp
    assert got[:2] == ref[:2]


def test_tcol_full_size_matches_tile_collect(oracle, monkeypatch):
    """cfg5's shape (N = 65536, d = 64, fp32) with the default tuning."""
    n, d = 65536, 64
    X = oracle.splitmix((n, d), 3.0, 64)
    res = []
    for ref in (False, True):
        monkeypatch.setenv("SVGD_COLLECT_FP64", "1" if ref else "0")
        c = S.Context(d, n, dtype=C.SVGD_F32)
        c.set_particles(X)
        res.append(c.median_scale() + (c.last_median_keys(),))
        assert c.last_scale()[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)
        c.close()
    assert res[0] == res[1]
