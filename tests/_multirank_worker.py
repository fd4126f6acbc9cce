"""Rank body of tests/test_multirank_cpu.py (gloo, one process per rank).

Re-enacts the sharded step protocol the library runs over RCCL
(svgd_capi.cpp median_begin / sample_bracket / collect_counts /
median_finish), with the same host planning functions from
libsvgdcpp_amd.so and numpy + the oracle as the arithmetic:

  1. rows [row0, row1) = svgd_plan_rows; G for own rows; all-gather of the
     equal ceil(n/P)-row chunks;
  2. median (GaussianRBFKernel.hpp:164-188, 222-254), exact:
     a. bracket: rank r draws pairs [S r/P, S (r+1)/P) of ONE counter-based
        sample sequence; two 11-bit radix passes over the sample keys, each
        with ONE all-reduce of the two selections' histograms, resolve the
        sample order statistics sigma either side of the target quantiles to
        22 bits -> bracket [lo, hi) (set by the last k_select_scan);
     b. collect over this rank's svgd_plan_pair_tiles tiles: keys below lo are
        counted, keys in [lo, hi) kept and histogrammed in NBK key-range
        buckets; ONE all-reduce of [below, candidates, NBK bucket counts];
     c. bracket hit: svgd_plan_bucket_select (the library's own host function)
        names the bucket(s) of the order statistics; each rank compacts its
        keys in them, ONE all-gather of the segments, every rank selects the
        same keys; bracket miss: streamed radix select over every key (one
        all-reduce per 11-bit digit) -- the library's fallback.  (The library
        usually plans the buckets on the device instead -- k_plan_select, the
        same scan over the same all-reduced counts, so every rank reaches the
        same plan without the host round trip; this re-enactment keeps the
        host planner, which the synchronous path and redo still use);
  3. phi_hat, Adam and clamp for own rows; all-gather the new X.
"""
import ctypes
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

RADIX = 11
NBK = 2048  # svgd_kernels.h
M64 = (1 << 64) - 1


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


def _allreduce_sum(dist, torch, arr):
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
    dist.all_reduce(t)
    return t.numpy()


def _radix_select(dist, torch, keys, ranks, passes, counter):
    """Dual radix select from bit 63 down, `passes` digits of RADIX bits, one
    all-reduce of both selections' histograms per digit.  Returns the resolved
    prefixes and the bit below them."""
    prefix = [0, 0]
    rank = list(ranks)
    hi_bit = 63
    for _ in range(passes):
        lo_bit = max(0, hi_bit - RADIX)
        width = hi_bit - lo_bit
        hists = []
        for s in range(2):
            sel = keys[(keys >> np.uint64(hi_bit)) == np.uint64(prefix[s] >> hi_bit)] if hi_bit < 64 else keys
            digit = ((sel >> np.uint64(lo_bit)) & np.uint64((1 << width) - 1)).astype(np.int64)
            hists.append(np.bincount(digit, minlength=1 << RADIX))
        h = _allreduce_sum(dist, torch, np.concatenate(hists))
        counter[0] += 1
        for s in range(2):
            cum = np.cumsum(h[s * (1 << RADIX):(s + 1) * (1 << RADIX)])
            b = int(np.searchsorted(cum, rank[s], side="right"))
            rank[s] -= int(cum[b - 1]) if b > 0 else 0
            prefix[s] |= b << lo_bit
        hi_bit = lo_bit
        if hi_bit == 0:
            break
    return prefix, hi_bit


def _exact_median(dist, torch, lib, X, keys, sample_size, sigma, counter, shift=0.0):
    n = X.shape[0]
    world, rank = dist.get_world_size(), dist.get_rank()
    M = n * (n - 1) // 2
    lo_r, hi_r = ctypes.c_int64(), ctypes.c_int64()
    navg = lib.svgd_plan_median_ranks(n, ctypes.byref(lo_r), ctypes.byref(hi_r))
    sel = sorted({r for r in (lo_r.value, hi_r.value) if r >= 0})
    if not sel:
        return 0.0, "direct"
    r0, r1 = sel[0], sel[-1]
    # a. sampled bracket (sample_bracket)
    S = min(sample_size, M)
    g0, g1 = S * rank // world, S * (rank + 1) // world
    skeys = _sample_keys(X, g0, g1)
    qlo, qhi = r0 / M, r1 / M
    slo = max(0.0, np.floor(qlo * S - sigma * (np.sqrt(S * qlo * (1 - qlo)) + 1)) - 1)
    shi = min(S - 1.0, np.ceil(qhi * S + sigma * (np.sqrt(S * qhi * (1 - qhi)) + 1)) + 1)
    if shift:  # tests: a bracket displaced off the median forces the fallback
        sh = shift * (np.sqrt(S * 0.25) + 1)
        slo, shi = min(S - 1.0, slo + sh), min(S - 1.0, shi + sh)
    (p_lo, p_hi), below_bit = _radix_select(dist, torch, skeys, (int(slo), int(shi)), 2, counter)
    lo = p_lo
    hi = min(M64, p_hi + (1 << below_bit))
    # b. collect: counts + key-range buckets, one all-reduce
    below = int(np.count_nonzero(keys < np.uint64(lo)))
    cand = keys[(keys >= np.uint64(lo)) & (keys < np.uint64(hi))] if hi < M64 else keys[keys >= np.uint64(lo)]
    binv = NBK / float(hi - lo)
    t = (cand - np.uint64(lo)).astype(np.float64) * binv
    bk = np.where(t < NBK - 1, np.where(t > 0, t, 0).astype(np.int64), NBK - 1)
    cnt = _allreduce_sum(dist, torch, np.concatenate([[below, cand.size], np.bincount(bk, minlength=NBK)]))
    counter[0] += 1
    below_all, cand_all, buckets = int(cnt[0]), int(cnt[1]), cnt[2:]
    if r0 >= below_all and r1 < below_all + cand_all:
        # c. bucket select: the library's plan, one all-gather of the keys
        ranks = (ctypes.c_int64 * 2)(r0 - below_all, r1 - below_all)
        bsel, rin, tot = (ctypes.c_int * 2)(), (ctypes.c_int64 * 2)(), ctypes.c_int64()
        bc = (ctypes.c_ulonglong * NBK)(*[int(x) for x in buckets])
        ns = 2 if r1 != r0 else 1
        assert lib.svgd_plan_bucket_select(bc, NBK, ns, ranks, bsel, rin, ctypes.byref(tot)) == 0
        mine = cand[np.isin(bk, [bsel[0], bsel[ns - 1]])]
        seg = np.zeros(tot.value + 1, dtype=np.int64)
        seg[0] = mine.size
        seg[1:1 + mine.size] = mine.view(np.int64)
        parts = [torch.zeros(seg.size, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(seg))
        counter[0] += 1
        pool = {}
        for s in range(ns):
            b = bsel[s]
            gathered = np.concatenate([p.numpy()[1:1 + p.numpy()[0]] for p in parts]).view(np.uint64)
            inb = np.sort(gathered[
                np.isin(np.where(((gathered - np.uint64(lo)).astype(np.float64) * binv) < NBK - 1,
                                 np.maximum((gathered - np.uint64(lo)).astype(np.float64) * binv, 0).astype(np.int64),
                                 NBK - 1), [b])])
            pool[s] = inb[rin[s]]
        vals = {r0: pool[0], r1: pool[ns - 1]}
        path = "bracket"
    else:
        # fallback: streamed radix select over every key, all 64 bits
        (k0, k1), _ = _radix_select(dist, torch, keys, (r0, r1), 6, counter)
        vals = {r0: np.uint64(k0), r1: np.uint64(k1)}
        path = "fallback"
    out = []
    for kr in [lo_r.value, hi_r.value][:navg]:
        out.append(0.0 if kr < 0 else float(np.sqrt(np.uint64(vals[kr]).view(np.float64))))
    return sum(out) / len(out), path


def run(rank, world, port, n, d, block, q, sample_size=4096, sigma=3.0, shift=0.0):
    try:
        import torch
        import torch.distributed as dist

        import oracle as O
        from svgdcpp_amd import _capi as C

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        lib = C.lib()
        X = O.splitmix((n, d), 3.0, 21)
        mus = O.splitmix((3, d), 3.0, 22)
        covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(3)])

        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        lib.svgd_plan_rows(n, world, rank, ctypes.byref(r0), ctypes.byref(r1))
        row0, row1 = r0.value, r1.value
        chunk = -(-n // world)

        def allgather_rows(shard):
            buf = np.zeros((chunk, d))
            buf[: shard.shape[0]] = shard
            parts = [torch.zeros(chunk, d, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(buf))
            return torch.cat(parts).numpy()[:n]

        # 1. G for own rows, all-gathered
        G_all = allgather_rows(O.logp_grad_gmm(X[row0:row1], mus, covs))

        # 2. median over this rank's pair tiles
        T = lib.svgd_plan_pair_tiles(n, block, world, rank)
        I, J = ctypes.c_int64(), ctypes.c_int64()
        keys = [np.zeros(0, dtype=np.uint64)]
        for t in range(T):
            lib.svgd_plan_pair_tile(n, block, world, rank, t, ctypes.byref(I), ctypes.byref(J))
            keys.append(_sqdist_keys(X, I.value, J.value, block))
        keys = np.concatenate(keys)
        total = int(_allreduce_sum(dist, torch, np.array([keys.size]))[0])
        counter = [0]
        med, path = _exact_median(dist, torch, lib, X, keys, sample_size, sigma, counter, shift)
        a = np.log(n) / med ** 2

        # 3. phi_hat + Adam + clamp for own rows, all-gather X
        ph = O.phi(X, G_all, a, rows=(row0, row1))
        opt = O.Adam((row1 - row0, d), 0.1, 0.9, 0.999)
        Xs = X[row0:row1].copy()
        lower, upper = -np.full(d, 2.0), np.full(d, 2.0)
        O.apply_update(Xs, opt.step(ph), lower, upper)
        X_new = allgather_rows(Xs)

        if rank == 0:
            q.put(("ok", dict(total=total, a=a, med=med, path=path, collectives=counter[0], G_all=G_all,
                              X_new=X_new, X=X, mus=mus, covs=covs)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))
