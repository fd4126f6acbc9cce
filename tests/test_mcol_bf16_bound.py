"""The error bound behind k_pair_mcol's split-bf16 Gram (svgd_collect.hip,
MCOL_DELTA_BF).  CPU only (numpy emulation of the arithmetic).

Each fp32 coordinate is split x = hi + lo + r with hi = bf16_rn(x) and
lo = bf16_rn(x - hi) (|x - hi - lo| <= 2^-17 |x|); the MFMA sums the four
bf16 products hi.hi, lo.hi, hi.lo, lo.lo (exact in fp32) and h_j in fp32.
The classification margin 2^-15 max|xc|^2 must cover |ef - e| for
e = h_j + xc_i.xc_j (proven bound 1.84e-5 max|xc|^2): checked here on
random, clustered and cancelling data, with every fp32 addition rounded (the
worst order the hardware could use is not known, so sequential rounding in
two orders is emulated) and with truncation instead of rounding.
"""
import numpy as np
import pytest


def bf16_rn(x32):
    """fp32 -> bf16 (round to nearest even), returned as fp32 values."""
    u = x32.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return r.astype(np.uint32).view(np.float32)


def split(x32):
    hi = bf16_rn(x32)
    lo = bf16_rn((x32 - hi).astype(np.float32))
    return hi, lo


def f32_sum(terms, trunc=False):
    """Sequential fp32 sum (each addition rounded, or truncated toward 0)."""
    acc = np.zeros(terms.shape[1:], dtype=np.float32)
    for t in terms:
        exact = acc.astype(np.float64) + t.astype(np.float64)
        s = exact.astype(np.float32)
        if trunc:
            over = np.abs(s.astype(np.float64)) > np.abs(exact)
            s = np.where(over, np.nextafter(s, np.float32(0)), s)
        acc = s
    return acc


@pytest.mark.parametrize("kind", ["gauss", "cluster", "cancel", "wide"])
@pytest.mark.parametrize("d", [1, 2, 5, 8])
def test_split_bf16_gram_within_margin(kind, d):
    rng = np.random.default_rng(1000 * d + len(kind))
    n = 4000
    if kind == "gauss":
        X = rng.normal(size=(n, d))
    elif kind == "cluster":
        X = rng.normal(size=(n, d)) * 1e-3 + 5.0
    elif kind == "cancel":
        X = rng.normal(size=(n, d))
        X[n // 2:] = -X[: n // 2] + rng.normal(size=(n // 2, d)) * 1e-6
    else:
        X = rng.normal(size=(n, d)) * np.exp(rng.uniform(-8, 8, size=(n, 1)))
    X -= X.mean(axis=0)
    nmax = float(np.max(np.sum(X * X, axis=1)))
    delta = 2.0 ** -15 * nmax

    i = rng.integers(0, n, 20000)
    j = rng.integers(0, n, 20000)
    xi, xj = X[i], X[j]
    e = -0.5 * np.sum(xj * xj, axis=1) + np.sum(xi * xj, axis=1)  # fp64 reference

    xi32, xj32 = xi.astype(np.float32), xj.astype(np.float32)
    hj = (-0.5 * np.sum(xj * xj, axis=1)).astype(np.float32)
    hi_i, lo_i = split(xi32)
    hi_j, lo_j = split(xj32)
    # the split itself: |x - hi - lo| <= 2^-17 |x|
    for x, h, l in ((xi32, hi_i, lo_i), (xj32, hi_j, lo_j)):
        r = x.astype(np.float64) - h.astype(np.float64) - l.astype(np.float64)
        assert np.all(np.abs(r) <= 2.0 ** -17 * np.abs(x.astype(np.float64)) + 1e-300)
    prods = np.concatenate([hi_i * hi_j, lo_i * hi_j, hi_i * lo_j, lo_i * lo_j], axis=1).astype(np.float64)
    # bf16 x bf16 products are exact in fp32
    assert np.all(prods.astype(np.float32).astype(np.float64) == prods)
    for order in (1, -1):
        for trunc in (False, True):
            terms = np.concatenate([hj[None, :], prods.T[::order].astype(np.float32)], axis=0)
            ef = f32_sum(terms, trunc=trunc).astype(np.float64)
            err = np.max(np.abs(ef - e))
            assert err <= 1.84e-5 * nmax + 1e-300, (kind, d, err / nmax)
            assert err < delta


def split3_exact(q32):
    """fp32 -> three bf16 parts summing to it exactly (mcol_fold_row)."""
    p0 = bf16_rn(q32)
    r = (q32 - p0).astype(np.float32)
    p1 = bf16_rn(r)
    p2 = bf16_rn((r - p1).astype(np.float32))
    return p0, p1, p2


@pytest.mark.parametrize("kind", ["gauss", "cluster", "cancel", "wide"])
@pytest.mark.parametrize("d", [1, 2, 5, 8])
def test_folded_centre_form_within_margin(kind, d):
    """The folded form (svgd_collect.hip mcol_fold_row): v = fl32(h_j - TM) +
    hi.hi + lo.hi + hi.lo (no lo.lo) + the three bf16 parts of fl32(-|x_i|^2/2)
    approximates x = h_j + x_i.x_j - |x_i|^2/2 - TM within the proven 3.62e-5
    max|xc|^2 < MCOL_DELTA_FOLD = 2^-14 max|xc|^2."""
    rng = np.random.default_rng(7000 * d + len(kind))
    n = 4000
    if kind == "gauss":
        X = rng.normal(size=(n, d))
    elif kind == "cluster":
        X = rng.normal(size=(n, d)) * 1e-3 + 5.0
    elif kind == "cancel":
        X = rng.normal(size=(n, d))
        X[n // 2:] = -X[: n // 2] + rng.normal(size=(n // 2, d)) * 1e-6
    else:
        X = rng.normal(size=(n, d)) * np.exp(rng.uniform(-8, 8, size=(n, 1)))
    X -= X.mean(axis=0)
    nrm = np.sum(X * X, axis=1)
    nmax = float(nrm.max())
    i = rng.integers(0, n, 20000)
    j = rng.integers(0, n, 20000)
    xi, xj = X[i], X[j]
    d2 = np.sum((xi - xj) ** 2, axis=1)
    for med in (np.median(d2), 0.0, 4 * nmax):  # centred, and the clamp's extremes
        TM = float(np.clip(-0.5 * med, -nmax, nmax))
        TMf = np.float32(TM)
        x = -0.5 * nrm[j] + np.sum(xi * xj, axis=1) - 0.5 * nrm[i] - float(TMf)  # exact (fp64)
        hj = (-0.5 * nrm[j]).astype(np.float32)
        C = (hj - TMf).astype(np.float32)
        xi32, xj32 = xi.astype(np.float32), xj.astype(np.float32)
        hi_i, lo_i = split(xi32)
        hi_j, lo_j = split(xj32)
        prods = np.concatenate([hi_i * hi_j, lo_i * hi_j, hi_i * lo_j], axis=1).astype(np.float64)
        q = (-0.5 * nrm[i]).astype(np.float32)
        p0, p1, p2 = split3_exact(q)
        assert np.all(p0.astype(np.float64) + p1 + p2 == q.astype(np.float64))
        rows = np.concatenate([prods, np.stack([p0, p1, p2], axis=1).astype(np.float64)], axis=1)
        assert np.all(rows.astype(np.float32).astype(np.float64) == rows)
        for order in (1, -1):
            for trunc in (False, True):
                terms = np.concatenate([C[None, :], rows.T[::order].astype(np.float32)], axis=0)
                v = f32_sum(terms, trunc=trunc).astype(np.float64)
                err = np.max(np.abs(v - x))
                assert err <= 3.62e-5 * nmax + 1e-300, (kind, d, med, err / nmax)
                assert err < 2.0 ** -14 * nmax
