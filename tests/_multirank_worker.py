"""Rank body of tests/test_multirank_cpu.py (gloo, one process per rank).

Re-enacts the sharded step the library runs over RCCL (svgd_capi.cpp,
DESIGN.md §5), with the same planning functions from libsvgdcpp_amd.so and
the oracle as the arithmetic:

  1. rows [row0, row1) = svgd_plan_rows; G for own rows; all-gather X|G
     in equal ceil(n/P)-row chunks;
  2. median: each rank keys the pairs of its svgd_plan_pair_tiles tiles, the
     ranks all-reduce 11-bit radix histograms to select the target order
     statistics (svgd_plan_median_ranks) -- the device's dual radix select;
  3. phi_hat, Adam and clamp for own rows; all-gather the new X.
"""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

RADIX = 11


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


def _allreduce_sum(dist, torch, arr):
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
    dist.all_reduce(t)
    return t.numpy()


def _select_rank(dist, torch, keys, k):
    """k-th smallest (0-based) key of the union of all ranks' keys."""
    prefix, shift, rank = np.uint64(0), 64, k
    width_mask = np.uint64(0)
    while shift > 0:
        s = max(0, shift - RADIX)
        bits = shift - s
        sel = keys[(keys & width_mask) == prefix] if width_mask else keys
        digit = ((sel >> np.uint64(s)) & np.uint64((1 << bits) - 1)).astype(np.int64)
        hist = _allreduce_sum(dist, torch, np.bincount(digit, minlength=1 << bits))
        cum = np.cumsum(hist)
        b = int(np.searchsorted(cum, rank, side="right"))
        rank -= int(cum[b - 1]) if b > 0 else 0
        prefix |= np.uint64(b) << np.uint64(s)
        width_mask |= np.uint64((1 << bits) - 1) << np.uint64(s)
        shift = s
    return prefix


def run(rank, world, port, n, d, block, q):
    try:
        import torch
        import torch.distributed as dist

        import oracle as O
        from svgdcpp_amd import _capi as C
        import ctypes

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
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        navg = lib.svgd_plan_median_ranks(n, ctypes.byref(lo), ctypes.byref(hi))
        vals = []
        for kr in [lo.value, hi.value][:navg]:
            vals.append(0.0 if kr < 0 else float(np.sqrt(_select_rank(dist, torch, keys, kr).view(np.float64))))
        med = sum(vals) / len(vals)
        a = np.log(n) / med ** 2

        # 3. phi_hat + Adam + clamp for own rows, all-gather X
        ph = O.phi(X, G_all, a, rows=(row0, row1))
        opt = O.Adam((row1 - row0, d), 0.1, 0.9, 0.999)
        Xs = X[row0:row1].copy()
        lower, upper = -np.full(d, 2.0), np.full(d, 2.0)
        O.apply_update(Xs, opt.step(ph), lower, upper)
        X_new = allgather_rows(Xs)

        if rank == 0:
            q.put(("ok", dict(total=total, a=a, med=med, G_all=G_all, X_new=X_new, X=X, mus=mus, covs=covs)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))
