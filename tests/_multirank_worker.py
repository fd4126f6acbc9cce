"""Rank body of tests/test_multirank_cpu.py (gloo, one process per rank).

Re-enacts, step after step, the sharded step protocol the library runs over
RCCL (svgd_capi.cpp scale_begin / median_begin / collect_counts /
median_finish(_spec) / upload_g_finish / run_phi_opt), with the
library's own host planners (libsvgdcpp_amd.so) and numpy + the oracle as the
arithmetic.  Per step:

  1. rows [row0, row1) = svgd_plan_rows; G for own rows;
  2. median (GaussianRBFKernel.hpp:164-188, 222-254), exact:
     a. bracket, decided before the collect (trk_plan):
        - tracked (the shipped default on speculative steps): the last
          selected medians extrapolated quadratically, half-width 4x the
          largest recent prediction error (trk_predict / trk_record); no
          sample, no collective;
        - else sampled: protocol "shipped" -- EVERY rank draws the whole
          sample (<= 2^20 pairs of one counter-based sequence) and runs the
          two 11-bit radix passes locally: the same bracket everywhere with
          no collective; protocol "shard" (SVGD_SAMPLE_SHARD=1, round 2's) --
          rank r draws pairs [S r/P, S (r+1)/P) and each radix pass
          all-reduces its histograms;
     b. collect over this rank's svgd_plan_pair_tiles tiles: keys below lo
        counted, keys in [lo, hi) kept and histogrammed in NBK buckets; ONE
        all-reduce of [below, candidates, NBK bucket counts] (comm);
     c. bracket hit: svgd_plan_bucket_select names the bucket(s), ONE
        all-gather of the compacted keys (comm), every rank selects the same
        keys; a tracked bracket that misses = a failed device plan: the step
        is redone with a sampled bracket; a sampled one that misses -> the
        streamed radix select over every key (one all-reduce per digit);
  3. the G all-gather on the G communicator (a second gloo group standing
     for the ncclCommSplit one, or the main group when gcomm is off), issued
     where upload_g_finish issues it: after every comm call of the median's
     first phase -- so on speculative steps after the keys all-gather, on
     synchronous ones before it (the cross-communicator issue order of
     svgd_ctx);
  4. phi_hat, Adam and clamp for own rows; the X all-gather (comm).

Every collective is logged as (group, op); the test checks the sequence.
"""
import ctypes
import os
import struct
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

RADIX = 11
NBK = 2048  # svgd_kernels.h
CAPG = 262144  # svgd_kernels.h: the selected buckets' key cap of the bucket path
CAPR_MIN = 4096  # svgd_kernels.h: the speculative cap's floor (plan_step: adaptive)


def spec_cap(last_tot):
    """svgd_capi.cpp plan_step: twice the last total, a power of two in [CAPR_MIN, CAPG]."""
    cap = CAPR_MIN
    while cap < 2 * last_tot and cap < CAPG:
        cap <<= 1
    return min(cap, CAPG)
M64 = (1 << 64) - 1
# svgd_capi.cpp tracked-bracket constants (trk_min_w, trk_err_mult)
TRK_MIN_W = 2e-5
TRK_ERR_MULT = 4.0


def _key(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _val(k):
    return struct.unpack("<d", struct.pack("<Q", int(k)))[0]


def _sqdist_keys(X, I, J, block):
    """u64 keys (bit patterns of D^2) of the unordered pairs of tile (I, J)."""
    n = X.shape[0]
    r0, r1 = I * block, min(n, (I + 1) * block)
    c0, c1 = J * block, min(n, (J + 1) * block)
    diff = X[r0:r1, None, :] - X[None, c0:c1, :]
    D2 = np.einsum("ijk,ijk->ij", diff, diff)
    if I == J:
        D2 = D2[np.triu_indices(r1 - r0, k=1)]
    return D2.ravel().astype(np.float64).view(np.uint64)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _sample_keys(X, g0, g1):
    """Keys of sample slots [g0, g1) of the counter-based pair sequence
    (k_sample_keys_f32: pair (i, j != i) from mix64(2 g + 1))."""
    n = X.shape[0]
    g = np.arange(g0, g1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _mix64(g * np.uint64(2) + np.uint64(1))
    i = ((h >> np.uint64(32)) * np.uint64(n)) >> np.uint64(32)
    j = i + np.uint64(1) + (((h & np.uint64(0xFFFFFFFF)) * np.uint64(n - 1)) >> np.uint64(32))
    j = np.where(j >= n, j - np.uint64(n), j)
    diff = X[i.astype(np.int64)] - X[j.astype(np.int64)]
    return np.einsum("ij,ij->i", diff, diff).view(np.uint64)


def sample_size(M, world):
    """svgd_capi.cpp sample_size(): automatic S, every rank draws all of it at P > 1."""
    S = min(max(M // 256, 1 << 18), 1 << 22)
    if world > 1:
        S = min(S, 1 << 20)
    return min(S, M)


class Comms:
    """The main communicator and the G one; every call logged as (group, op)."""

    def __init__(self, dist, torch, gcomm):
        self.dist, self.torch = dist, torch
        self.g = dist.new_group() if gcomm else None
        self.log = []

    def allreduce(self, arr):
        t = self.torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
        self.dist.all_reduce(t)
        self.log.append(("comm", "allreduce"))
        return t.numpy()

    def allgather(self, arr, group="comm", what="allgather"):
        t = self.torch.from_numpy(np.ascontiguousarray(arr))
        parts = [self.torch.zeros_like(t) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(parts, t, group=self.g if group == "gcomm" and self.g is not None else None)
        self.log.append(("gcomm" if group == "gcomm" and self.g is not None else "comm", what))
        return [p.numpy() for p in parts]


def _radix_select(reduce, keys, ranks, passes):
    """Dual radix select from bit 63 down, `passes` digits of RADIX bits;
    `reduce` combines the histograms (an all-reduce, or the identity when
    every rank holds the whole key set).  Returns the resolved prefixes and
    the bit below them."""
    prefix = [0, 0]
    rank = list(ranks)
    hi_bit = 63
    for _ in range(passes):
        lo_bit = max(0, hi_bit - RADIX)
        width = hi_bit - lo_bit
        hists = []
        for s in range(2):
            sel = keys[(keys >> np.uint64(hi_bit)) == np.uint64(prefix[s] >> hi_bit)]
            digit = ((sel >> np.uint64(lo_bit)) & np.uint64((1 << width) - 1)).astype(np.int64)
            hists.append(np.bincount(digit, minlength=1 << RADIX))
        h = reduce(np.concatenate(hists))
        for s in range(2):
            cum = np.cumsum(h[s * (1 << RADIX):(s + 1) * (1 << RADIX)])
            b = int(np.searchsorted(cum, rank[s], side="right"))
            rank[s] -= int(cum[b - 1]) if b > 0 else 0
            prefix[s] |= b << lo_bit
        hi_bit = lo_bit
        if hi_bit == 0:
            break
    return prefix, hi_bit


class Tracker:
    """svgd_capi.cpp trk_record / trk_extrapolate / trk_predict."""

    def __init__(self):
        self.m = [0.0, 0.0, 0.0]
        self.n = 0
        self.err = [0.0, 0.0, 0.0]
        self.nerr = 0
        self.dens = 0.0
        self.pred = -1.0

    def extrapolate(self):
        m = self.m
        p = 3.0 * m[0] - 3.0 * m[1] + m[2] if self.n >= 3 else 2.0 * m[0] - m[1]
        return p if p > 0.0 else m[0]

    def record(self, m_sel, lo_key, hi_key, cand):
        if not (m_sel > 0.0) or not np.isfinite(m_sel):
            self.n = 0
            return
        if self.n >= 2:
            p = self.pred if self.pred >= 0 else self.extrapolate()
            self.err = [abs(m_sel - p) / m_sel] + self.err[:2]
            self.nerr = min(self.nerr + 1, 3)
        lo = _val(lo_key)
        hi = np.inf if hi_key >= 0x7FF0000000000000 else _val(hi_key)
        self.dens = cand / (hi - lo) if np.isfinite(hi) and hi > lo else 0.0
        self.m = [m_sel] + self.m[:2]
        self.n = min(self.n + 1, 3)

    def predict(self, Mq, band_samp):
        self.pred = -1.0
        if self.n < 2 or not self.dens > 0.0:
            return None
        m1, m2 = self.m[0], self.m[1]
        pred = self.extrapolate()
        e = abs(m1 - m2) / m1 if self.nerr == 0 else 0.0
        for k in range(self.nerr):
            e = max(e, self.err[k])
        w = max(TRK_ERR_MULT * e, TRK_MIN_W)
        if not w < 0.05:
            return None
        lo, hi = pred * (1.0 - w), pred * (1.0 + w)
        band = self.dens * (hi - lo) / Mq
        if not band <= band_samp:
            return None
        self.pred = pred
        return _key(lo), _key(hi) + 1


def _bucket_of(keys, lo, binv):
    t = (keys - np.uint64(lo)).astype(np.float64) * binv
    return np.where(t < NBK - 1, np.where(t > 0, t, 0).astype(np.int64), NBK - 1)


def _median(cm, lib, X, keys, protocol, sigma, shift, trk, spec, on_g, cap=CAPG):
    """One step's exact median; on_g() issues the G all-gather where
    upload_g_finish would.  Returns (med, path, bracket kind, selected D^2
    of the lower order statistic, fast, bracket record for the tracker)."""
    n = X.shape[0]
    world, rank = cm.dist.get_world_size(), cm.dist.get_rank()
    M = n * (n - 1) // 2
    lo_r, hi_r = ctypes.c_int64(), ctypes.c_int64()
    navg = lib.svgd_plan_median_ranks(n, ctypes.byref(lo_r), ctypes.byref(hi_r))
    sel = sorted({r for r in (lo_r.value, hi_r.value) if r >= 0})
    r0, r1 = sel[0], sel[-1]
    S = sample_size(M, world)
    sig = np.sqrt(S * 0.25) + 1.0
    band_samp = (2.0 * sigma * sig + 3.0) / S
    # a. bracket: tracked (speculative steps only), else sampled
    br = trk.predict(float(M), band_samp) if (spec and protocol == "shipped" and not shift) else None
    kind = "tracked" if br is not None else "sampled"
    if br is not None:
        lo, hi = br
    else:
        if protocol == "shipped":  # every rank draws the whole sample: no collective
            g0, g1 = 0, S
            reduce = lambda h: h  # noqa: E731
        else:  # round 2's sharded sample: histograms all-reduced per pass
            g0, g1 = S * rank // world, S * (rank + 1) // world
            reduce = cm.allreduce
        skeys = _sample_keys(X, g0, g1)
        qlo, qhi = r0 / M, r1 / M
        slo = max(0.0, np.floor(qlo * S - sigma * (np.sqrt(S * qlo * (1 - qlo)) + 1)) - 1)
        shi = min(S - 1.0, np.ceil(qhi * S + sigma * (np.sqrt(S * qhi * (1 - qhi)) + 1)) + 1)
        if shift:  # tests: a bracket displaced off the median forces the fallback
            sh = shift * (np.sqrt(S * 0.25) + 1)
            slo, shi = min(S - 1.0, slo + sh), min(S - 1.0, shi + sh)
        (p_lo, p_hi), below_bit = _radix_select(reduce, skeys, (int(slo), int(shi)), 2)
        lo = p_lo
        hi = min(M64, p_hi + (1 << below_bit))
    # b. collect: counts + key-range buckets, ONE all-reduce
    below = int(np.count_nonzero(keys < np.uint64(lo)))
    cand = keys[(keys >= np.uint64(lo)) & (keys < np.uint64(hi))] if hi < M64 else keys[keys >= np.uint64(lo)]
    binv = NBK / float(hi - lo)
    bk = _bucket_of(cand, lo, binv)
    cnt = cm.allreduce(np.concatenate([[below, cand.size], np.bincount(bk, minlength=NBK)]))
    below_all, cand_all, buckets = int(cnt[0]), int(cnt[1]), cnt[2:]
    hit = r0 >= below_all and r1 < below_all + cand_all
    if not spec:
        on_g()  # synchronous step: the G all-gather precedes the keys all-gather
    if hit:
        ranks = (ctypes.c_int64 * 2)(r0 - below_all, r1 - below_all)
        bsel, rin, tot = (ctypes.c_int * 2)(), (ctypes.c_int64 * 2)(), ctypes.c_int64()
        bc = (ctypes.c_ulonglong * NBK)(*[int(x) for x in buckets])
        ns = 2 if r1 != r0 else 1
        assert lib.svgd_plan_bucket_select(bc, NBK, ns, ranks, bsel, rin, ctypes.byref(tot)) == 0
        if spec and tot.value > cap:
            hit = False  # the device plan fails on oversized buckets (redo)
    if spec and not hit:
        # failed device plan: the speculative chain still ran (its keys
        # all-gather, the G all-gather); the caller redoes the step
        cm.allgather(np.zeros(cap + 1, dtype=np.int64), what="keys")
        on_g()
        return None
    if hit:
        # c. bucket select: ONE all-gather of the compacted keys
        mine = cand[np.isin(bk, [bsel[0], bsel[ns - 1]])]
        seg = np.zeros(tot.value + 1, dtype=np.int64)
        seg[0] = mine.size
        seg[1:1 + mine.size] = mine.view(np.int64)
        parts = cm.allgather(seg, what="keys")
        gathered = np.concatenate([p[1:1 + p[0]] for p in parts]).view(np.uint64)
        gb = _bucket_of(gathered, lo, binv)
        pool = {s: np.sort(gathered[gb == bsel[s]])[rin[s]] for s in range(ns)}
        vals = {r0: pool[0], r1: pool[ns - 1]}
        path = "bracket"
        fast = tot.value <= CAPG
    else:
        # fallback: streamed radix select over every key, all 64 bits
        (k0, k1), _ = _radix_select(cm.allreduce, keys, (r0, r1), 6)
        vals = {r0: np.uint64(k0), r1: np.uint64(k1)}
        path = "fallback"
        fast = False
    if spec:
        on_g()  # speculative step: every comm call of the median first
    out = [0.0 if kr < 0 else float(np.sqrt(np.uint64(vals[kr]).view(np.float64)))
           for kr in [lo_r.value, hi_r.value][:navg]]
    m_sel = float(np.uint64(vals[r0]).view(np.float64))
    rec = (lo, hi, cand_all) if path == "bracket" else None
    return sum(out) / len(out), path, kind, m_sel, fast, rec, (tot.value if hit else 0)


def run(rank, world, port, n, d, block, q, sigma=3.0, shift=0.0, steps=1, protocol="shipped",
        gcomm=True, lr=0.1, bound=2.0):
    try:
        import torch
        import torch.distributed as dist

        import oracle as O
        from svgdcpp_amd import _capi as C

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        cm = Comms(dist, torch, gcomm)
        lib = C.lib()
        X = O.splitmix((n, d), 3.0, 21)
        mus = O.splitmix((3, d), 3.0, 22)
        covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(3)])

        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        lib.svgd_plan_rows(n, world, rank, ctypes.byref(r0), ctypes.byref(r1))
        row0, row1 = r0.value, r1.value
        chunk = -(-n // world)

        def gather_rows(shard, group="comm", what="rows"):
            buf = np.zeros((chunk, d))
            buf[: shard.shape[0]] = shard
            return np.concatenate(cm.allgather(buf, group=group, what=what))[:n]

        T = lib.svgd_plan_pair_tiles(n, block, world, rank)
        I, J = ctypes.c_int64(), ctypes.c_int64()
        tiles = []
        for t in range(T):
            lib.svgd_plan_pair_tile(n, block, world, rank, t, ctypes.byref(I), ctypes.byref(J))
            tiles.append((I.value, J.value))
        opt = O.Adam((row1 - row0, d), lr, 0.9, 0.999)
        lower, upper = -np.full(d, bound), np.full(d, bound)
        trk = Tracker()
        last_fast = False
        last_tot = 0
        hist = []
        for _ in range(steps):
            Xt = X.copy()
            # 1. G for own rows (the host gradient)
            G_own = O.logp_grad_gmm(X[row0:row1], mus, covs)
            keys = np.concatenate([np.zeros(0, dtype=np.uint64)] +
                                  [_sqdist_keys(X, a, b, block) for a, b in tiles])
            total = int(cm.allreduce(np.array([keys.size]))[0])
            cm.log.pop()  # (the pair-count check is the test's, not the protocol's)
            mark = len(cm.log)
            box = {}

            def on_g():  # (a redo reuses the step's G: gathered once)
                if "G" not in box:
                    box["G"] = gather_rows(G_own, group="gcomm", what="G")

            # 2. the median: speculative when the last selection allowed it
            spec = last_fast
            res = _median(cm, lib, X, keys, protocol, sigma, shift, trk, spec, on_g, spec_cap(last_tot))
            redo = res is None
            if redo:
                # a failed device plan (resolve_pending): the speculative
                # step's update and X all-gather ran; X_t, m_t, v_t are
                # restored and all-gathered, and the step is redone
                # synchronously with a sampled bracket
                gather_rows(X[row0:row1], what="X")
                gather_rows(X[row0:row1], what="X_restore")
                trk.pred = -1.0
                res = _median(cm, lib, X, keys, protocol, sigma, shift, trk, False, on_g)
            med, path, kind, m_sel, fast, rec, last_tot = res
            if rec is not None:
                trk.record(m_sel, *rec)
            else:
                trk.n = 0
            last_fast = fast
            a = np.log(n) / med ** 2
            # 4. phi_hat + Adam + clamp for own rows, X all-gathered
            ph = O.phi(X, box["G"], a, rows=(row0, row1))
            Xs = X[row0:row1].copy()
            O.apply_update(Xs, opt.step(ph), lower, upper)
            X = gather_rows(Xs, what="X")
            hist.append(dict(X=Xt, X_new=X.copy(), G_all=box["G"], a=a, med=med, path=path,
                             bracket=kind, spec=spec, redo=redo, total=total,
                             colls=list(cm.log[mark:])))
        if rank == 0:
            q.put(("ok", dict(steps=hist, mus=mus, covs=covs, lr=lr, bound=bound)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))
