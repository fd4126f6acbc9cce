"""The three-part bf16 split of the F32 tile phi on the matrix cores
(k_phi_b3, svgd_kernels.hip): numpy emulation of v_cvt_pk_bf16_f32 (round to
nearest even) on fp32 data.

* every fp32 x with |x| >= 2^-100 splits exactly: x = h + m + l, each part
  a bf16 value, |m| <= 2^-8 |x|, |l| <= 2^-16 |x| (below that the parts
  reach the subnormal range and the split is exact to 2^-133 absolute);
* a dot product formed from the six part products hh, hm, mh, hl, lh, mm
  (exact in fp32, as the MFMA forms them) differs from the exact dot of the
  fp32 inputs by <= 2^-22 * sum |a_k b_k| before the fp32 accumulation, i.e.
  the dropped products cost no more than the fp32 MFMA's own rounding."""
import numpy as np


def bf16_rn(x):
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    x = np.asarray(x, dtype=np.float32)
    h = bf16_rn(x)
    r1 = (x - h).astype(np.float32)
    m = bf16_rn(r1)
    r2 = (r1 - m).astype(np.float32)
    low = bf16_rn(r2)
    return h, m, low


def test_split_is_exact():
    rng = np.random.default_rng(1)
    for scale in (1e-30, 1e-3, 1.0, 7.0, 1e4, 1e30):
        x = (rng.standard_normal(200000) * scale).astype(np.float32)
        x = x[np.abs(x) >= 2.0 ** -100]
        h, m, low = split3(x)
        for p in (h, m, low):
            assert np.array_equal(bf16_rn(p), p)  # each part is a bf16 value
        s = h.astype(np.float64) + m.astype(np.float64) + low.astype(np.float64)
        assert np.array_equal(s, x.astype(np.float64))
        ax = np.abs(x.astype(np.float64))
        assert np.all(np.abs(m) <= 2.0 ** -8 * ax)
        assert np.all(np.abs(low) <= 2.0 ** -16 * ax)


def test_six_products_bound():
    rng = np.random.default_rng(2)
    for d in (17, 32, 64):
        a = rng.standard_normal((2000, d)).astype(np.float32) * 3
        b = rng.standard_normal((2000, d)).astype(np.float32) * 3
        ah, am, al = (p.astype(np.float64) for p in split3(a))
        bh, bm, bl = (p.astype(np.float64) for p in split3(b))
        six = (ah * bh + ah * bm + am * bh + ah * bl + al * bh + am * bm).sum(-1)
        exact = (a.astype(np.float64) * b.astype(np.float64)).sum(-1)
        mag = np.abs(a.astype(np.float64) * b.astype(np.float64)).sum(-1)
        assert np.all(np.abs(six - exact) <= 2.0 ** -22 * mag)


def split3_trunc(x):
    """The kernel's split of P (b3_trunc_pair): each part the top 16 bits of
    the remaining residual (truncation), residuals exact in fp32."""
    x = np.asarray(x, dtype=np.float32)
    mask = np.uint32(0xFFFF0000)
    h = (x.view(np.uint32) & mask).view(np.float32)
    r1 = (x - h).astype(np.float32)
    m = (r1.view(np.uint32) & mask).view(np.float32)
    r2 = (r1 - m).astype(np.float32)
    low = (r2.view(np.uint32) & mask).view(np.float32)
    return h, m, low


def test_truncating_split_is_exact_and_mixed_bound():
    rng = np.random.default_rng(3)
    for scale in (1e-20, 1e-3, 1.0, 1e4):
        x = (rng.random(200000) * scale).astype(np.float32)  # P in (0, scale)
        x = x[x >= 2.0 ** -100]
        h, m, low = split3_trunc(x)
        assert np.array_equal(h.astype(np.float64) + m + low, x.astype(np.float64))
        ax = x.astype(np.float64)
        assert np.all(np.abs(m) < 2.0 ** -7 * ax) and np.all(np.abs(low) < 2.0 ** -15 * ax)
    # P (truncated parts) against V (round-to-nearest parts): six products
    p = rng.random((2000, 32)).astype(np.float32)
    v = (rng.standard_normal((2000, 32)) * 5).astype(np.float32)
    ph, pm, pl = (q.astype(np.float64) for q in split3_trunc(p))
    vh, vm, vl = (q.astype(np.float64) for q in split3(v))
    six = (ph * vh + ph * vm + pm * vh + ph * vl + pl * vh + pm * vm).sum(-1)
    exact = (p.astype(np.float64) * v.astype(np.float64)).sum(-1)
    mag = np.abs(p.astype(np.float64) * v.astype(np.float64)).sum(-1)
    assert np.all(np.abs(six - exact) <= 2.0 ** -22 * mag)
