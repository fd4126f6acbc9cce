"""C-ABI library checks that need no GPU: it loads, exports every function
declared in include/svgdcpp_amd/svgd_capi.h, and its host-only helpers
(work partition plan, median rank mapping, host models) are correct."""
import ctypes
import re

import numpy as np
import pytest

from svgdcpp_amd import _capi as C


def _declared_functions():
    src = open(C.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(svgd_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(C.LIB_PATH)
    declared = _declared_functions()
    assert len(declared) >= 30
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    # and the Python binding covers exactly the declared set
    assert sorted(C.SIGNATURES) == declared


def test_binding_loads():
    assert C.lib() is not None


def _rows(n, world, rank):
    r0, r1 = ctypes.c_int64(), ctypes.c_int64()
    C.lib().svgd_plan_rows(n, world, rank, ctypes.byref(r0), ctypes.byref(r1))
    return r0.value, r1.value


@pytest.mark.parametrize("n", [1, 5, 64, 65, 1000, 65536, 262144])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_plan_rows_partition(n, world):
    spans = [_rows(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a0 <= a1
    chunk = -(-n // world)
    assert all(r1 - r0 <= chunk for r0, r1 in spans)


def _tiles(n, world, rank, block=64):
    lib = C.lib()
    T = lib.svgd_plan_pair_tiles(n, block, world, rank)
    out = []
    I, J = ctypes.c_int64(), ctypes.c_int64()
    for t in range(T):
        lib.svgd_plan_pair_tile(n, block, world, rank, t, ctypes.byref(I), ctypes.byref(J))
        out.append((I.value, J.value))
    return out


@pytest.mark.parametrize("n", [1, 63, 64, 65, 128, 129, 300, 640, 1000, 3000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("block", [64, 256])
def test_plan_pair_tiles_cover_each_pair_once(n, world, block):
    """Every unordered particle pair i<j is in exactly one tile of one rank."""
    nb = -(-n // block)
    seen = np.zeros((nb, nb), dtype=int)
    counts = []
    for r in range(world):
        t = _tiles(n, world, r, block)
        counts.append(len(t))
        for I, J in t:
            if I == J:
                seen[I, I] += 1
            else:
                seen[min(I, J), max(I, J)] += 1
    assert np.all(seen[np.triu_indices(nb)] == 1)
    assert max(counts) - min(counts) <= 1  # balanced


def test_plan_median_ranks_matches_full_list():
    lib = C.lib()
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    for n in range(1, 60):
        navg = lib.svgd_plan_median_ranks(n, ctypes.byref(lo), ctypes.byref(hi))
        tot = n * n
        ks = [tot // 2 - 1, tot // 2] if tot % 2 == 0 else [tot // 2]
        assert navg == len(ks)
        exp = [(-1 if k < n else (k - n) // 2) for k in ks]
        got = [lo.value, hi.value][: len(ks)]
        assert got == exp


def test_host_model_matches_oracle(oracle):
    d, k = 5, 3
    mus = oracle.splitmix((k, d), 3.0, 1)
    A = oracle.splitmix((k, d, d), 1.0, 2)
    covs = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
    X = oracle.splitmix((257, d), 4.0, 3)
    h = ctypes.c_void_p()
    assert C.lib().svgd_model_create(ctypes.byref(h), d, k, C.dptr(np.ascontiguousarray(mus)),
                                     C.dptr(np.ascontiguousarray(covs))) == 0
    G = np.empty_like(X)
    C.lib().svgd_model_logp_grad(h, C.dptr(X), X.shape[0], C.dptr(G))
    C.lib().svgd_model_destroy(h)
    np.testing.assert_allclose(G, oracle.logp_grad_gmm(X, mus, covs), rtol=1e-11, atol=1e-12)


def test_python_api_host_side(oracle):
    """Host-only parts of the Python mirror: argument checks and models."""
    import svgdcpp_amd as S
    with pytest.raises(ValueError, match=r"^SVGDCpp: \[Argument Error\]"):
        S.RMSProp(2, 3, 0.1, 1.5)
    with pytest.raises(S.DimensionMismatchException, match=r"^SVGDCpp: \[Dimension Error\]"):
        S.MultivariateNormal([0.0, 1.0], np.eye(3))
    m = S.MultivariateNormal([0.0, 1.0], [[2.0, 0.3], [0.3, 1.0]]) + \
        S.MultivariateNormal([1.0, -1.0], [[1.0, 0.0], [0.0, 1.0]])
    X = oracle.splitmix((9, 2), 2.0, 4)
    ref = oracle.logp_grad_gmm(X, np.array([[0.0, 1.0], [1.0, -1.0]]),
                               np.array([[[2.0, 0.3], [0.3, 1.0]], [[1.0, 0.0], [0.0, 1.0]]]))
    np.testing.assert_allclose(m.log_model_grad(X), ref, rtol=1e-12, atol=1e-14)


def test_exp2_table_and_coefficients_match_generator():
    """The kernel's 2^(i/256) table and Taylor coefficients (exp2_256) are the
    correctly rounded values tools/make_exp_table.py derives at 60 digits."""
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("mk", os.path.join(root, "tools", "make_exp_table.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    src = open(os.path.join(root, "svgdcpp_amd", "csrc", "svgd_kernels.hip")).read()
    body = src[src.index("EXP2_TAB256[256] = {"):]
    body = body[body.index("{") + 1:body.index("}")]
    vals = [float.fromhex(v.strip()) for v in body.replace("\n", " ").split(",") if v.strip()]
    assert vals == mk.table()
    fn = src[src.index("double exp2_256_poly("):]
    fn = fn[:fn.index("return")]
    lits = [float.fromhex(t) for t in re.findall(r"0x1\.[0-9a-f]+p[-+]\d+", fn)]
    c = mk.coeffs()
    assert lits == [c[4], c[3], c[2], c[1]]


def test_exp2_4096_table_and_coefficients_match_generator():
    """The row-stream phi kernel's 2^(i/4096) table (svgd_exp_table.h) and its
    levelled degree-2 coefficients are what tools/make_exp_table.py derives, and
    the form's relative error stays <= 2.6e-14 on |f| <= 1/2 (checked at 60
    digits)."""
    import importlib.util
    import os
    from decimal import Decimal, getcontext

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("mk", os.path.join(root, "tools", "make_exp_table.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    hdr = open(os.path.join(root, "svgdcpp_amd", "csrc", "svgd_exp_table.h")).read()
    assert hdr == mk.header_text()
    src = open(os.path.join(root, "svgdcpp_amd", "csrc", "svgd_kernels.hip")).read()
    fn = src[src.index("double exp2_4096_poly("):]
    fn = fn[:fn.index("}")]
    lits = [float.fromhex(t) for t in re.findall(r"0x1\.[0-9a-f]+p[-+]\d+", fn)]
    c1, c2 = mk.coeffs4096()
    assert lits == [c2, c1]
    getcontext().prec = 60
    k = Decimal(2).ln() / 4096
    worst = max(abs((1 + Decimal(c1) * f + Decimal(c2) * f * f) / (k * f).exp() - 1)
                for f in (Decimal(i) / 1000 for i in range(-500, 501)))
    assert worst <= Decimal("2.6e-14")


def test_host_model_hessian_sum_matches_oracle(oracle):
    import svgdcpp_amd as S

    rng = np.random.default_rng(4)
    d, k, n = 5, 3, 400
    mus = rng.standard_normal((k, d))
    covs = []
    for _ in range(k):
        A = rng.standard_normal((d, d)) * 0.3
        covs.append(A @ A.T + np.eye(d))
    X = rng.standard_normal((n, d)) * 2
    m = S.GaussianSum(list(mus), covs)
    np.testing.assert_allclose(m.neg_hess_sum(X), oracle.neg_hess_sum_gmm(X, mus, np.stack(covs)),
                               rtol=1e-11, atol=1e-11)


def test_plan_bucket_select():
    """Bucket of each median rank from an ascending bucket histogram (the
    all-reduced key-range counts of the collect pass)."""
    lib = C.lib()
    rng = np.random.default_rng(7)
    for trial in range(50):
        nb = int(rng.integers(1, 64))
        counts = rng.integers(0, 5, nb).astype(np.uint64)
        tot = int(counts.sum())
        if tot == 0:
            continue
        cum = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        nsel = int(rng.integers(1, 3))
        r = np.sort(rng.integers(0, tot, nsel)).astype(np.int64)
        bsel = (ctypes.c_int * 2)()
        rin = (ctypes.c_int64 * 2)()
        tot_sel = ctypes.c_int64()
        rc = lib.svgd_plan_bucket_select(counts.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nb, nsel,
                                         r.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), bsel, rin,
                                         ctypes.byref(tot_sel))
        assert rc == 0
        exp_b = [int(np.searchsorted(cum, x, side="right") - 1) for x in r]
        for s in range(nsel):
            assert bsel[s] == exp_b[s]
            assert rin[s] == r[s] - cum[exp_b[s]]
        bs = sorted(set(exp_b))
        assert tot_sel.value == sum(int(counts[b]) for b in bs)
    # a rank past the candidates is refused
    counts = np.array([1, 2, 0], dtype=np.uint64)
    r = np.array([3], dtype=np.int64)
    bsel = (ctypes.c_int * 2)()
    rin = (ctypes.c_int64 * 2)()
    t = ctypes.c_int64()
    assert lib.svgd_plan_bucket_select(counts.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 3, 1,
                                       r.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), bsel, rin,
                                       ctypes.byref(t)) == -1


def _tile(lib, n, block, t):
    I, J = ctypes.c_int64(), ctypes.c_int64()
    lib.svgd_plan_pair_tile(n, block, 1, 0, t, ctypes.byref(I), ctypes.byref(J))
    return I.value, J.value


@pytest.mark.parametrize("n,block,world,grid", [(65536, 1536, 1, 256), (65536, 1536, 2, 256),
                                               (65536, 1536, 4, 256), (65536, 1536, 8, 256),
                                               (262144, 1536, 8, 256), (16384, 4096, 1, 256),
                                               (6007, 1536, 3, 5), (3001, 2048, 2, 7), (1537, 1536, 1, 4)])
def test_plan_sym_units(n, block, world, grid):
    """The symmetric phi pass's unit plan (svgd_plan_sym_units, used by the
    context for k_phi_sym / k_sym_finish): the units are the plan's (tile,
    sub-tile) pairs without the padding-only sub-tiles of the last column
    block (svgd_plan_sym_total / svgd_plan_sym_unit); the ranks' unit ranges
    partition them once; each work-group's contiguous run is
    non-empty; blkg holds exactly the work-groups whose runs visit a row
    block (a contiguous range); rbase numbers each row block's records
    contiguously in work-group order; Ia..Ib span the rank's row blocks; and
    the finish's column-partial index (column block J, slot (J - I) mod nb)
    is one-to-one over the off-diagonal tiles."""
    lib = C.lib()
    nsub = block // 64
    nb = (n + block - 1) // block
    T = nb * (nb + 1) // 2
    tiles = [_tile(lib, n, block, t) for t in range(T)]
    # the units: every (tile, sub-tile) in plan order except the last column
    # block's sub-tiles that hold only padding columns
    U = lib.svgd_plan_sym_total(n, block, nsub)
    unit_tile = []
    for u in range(U):
        t, q = ctypes.c_int64(), ctypes.c_int64()
        assert lib.svgd_plan_sym_unit(n, block, nsub, u, ctypes.byref(t), ctypes.byref(q)) == 0
        unit_tile.append((t.value, q.value))
    expect = [(t, q) for t in range(T) for q in range(nsub) if tiles[t][1] * block + 64 * q < n]
    assert unit_tile == expect
    t, q = ctypes.c_int64(), ctypes.c_int64()
    assert lib.svgd_plan_sym_unit(n, block, nsub, U, ctypes.byref(t), ctypes.byref(q)) == -1
    slots = {}
    for t, (I, J) in enumerate(tiles):
        if I != J:
            key = (J, (J - I) % nb)
            assert key not in slots, (key, t, slots.get(key))
            slots[key] = t
    assert len(slots) == T - nb
    cover = []
    for r in range(world):
        u0, u1, Ia, Ib = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        blkg = (ctypes.c_int * (2 * nb))()
        rbase = (ctypes.c_int * nb)()
        g = min(grid, max(1, U * (r + 1) // world - U * r // world))
        nrec = lib.svgd_plan_sym_units(n, block, nsub, world, r, g, ctypes.byref(u0), ctypes.byref(u1), blkg,
                                       rbase, ctypes.byref(Ia), ctypes.byref(Ib))
        u0, u1 = u0.value, u1.value
        cover.append((u0, u1))
        V = u1 - u0
        visits = {}
        for wg in range(g):
            a, b = u0 + V * wg // g, u0 + V * (wg + 1) // g
            assert b > a
            for P in {tiles[unit_tile[u][0]][0] for u in range(a, b)}:
                visits.setdefault(P, []).append(wg)
        expect_rec = 0
        for P in range(nb):
            lo, hi = blkg[2 * P], blkg[2 * P + 1]
            got = list(range(lo, hi + 1)) if hi >= lo else []
            assert got == sorted(visits.get(P, [])), (r, P, got, visits.get(P))
            assert rbase[P] == expect_rec
            expect_rec += len(got)
        assert nrec == expect_rec
        rows = {tiles[unit_tile[u][0]][0] for u in range(u0, u1)}
        assert rows == set(range(Ia.value, Ib.value + 1))
    assert cover[0][0] == 0 and cover[-1][1] == U
    assert all(a[1] == b[0] for a, b in zip(cover, cover[1:]))
