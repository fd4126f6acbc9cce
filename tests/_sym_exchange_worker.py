"""Rank body of tests/test_sym_exchange_cpu.py: the sharded symmetric phi
pass's protocol (svgd_capi.cpp run_phi, DESIGN §4.1 "Sharded") with gloo in
place of RCCL and numpy as the arithmetic.  Rank r takes the (tile, 64-column
sub-tile) units svgd_plan_sym_units gives it, adds every unit's pair terms
to BOTH particles (row side; column side off the diagonal tiles, whose row
side already holds every ordered pair of the square), then the per-particle
sums are reduce-scattered (here an all-reduce, as the host-shm backend does)
and phi is formed for the rank's rows (svgd_plan_rows)."""
import ctypes
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run(rank, world, port, n, d, block, a, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        import oracle as O
        from svgdcpp_amd import _capi as C

        dist.init_process_group("gloo", rank=rank, world_size=world)
        lib = C.lib()
        X = O.splitmix((n, d), 2.0, 77)
        G = O.splitmix((n, d), 1.0, 78)
        nsub = block // 64
        nb = (n + block - 1) // block
        u0, u1, Ia, Ib = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        blkg = (ctypes.c_int * (2 * nb))()
        rbase = (ctypes.c_int * nb)()
        lib.svgd_plan_sym_units(n, block, nsub, world, rank, 1, ctypes.byref(u0), ctypes.byref(u1), blkg, rbase,
                                ctypes.byref(Ia), ctypes.byref(Ib))
        S = np.zeros((n, d))
        pairs = 0
        for u in range(u0.value, u1.value):
            t, sq = divmod(u, nsub)
            I, J = ctypes.c_int64(), ctypes.c_int64()
            lib.svgd_plan_pair_tile(n, block, 1, 0, t, ctypes.byref(I), ctypes.byref(J))
            I, J = I.value, J.value
            rows = np.arange(I * block, min(n, (I + 1) * block))
            cols = np.arange(J * block + 64 * sq, min(n, J * block + 64 * (sq + 1)))
            if rows.size == 0 or cols.size == 0:
                continue
            diff = X[rows, None, :] - X[None, cols, :]  # x_i - x_j
            K = np.exp(-a * np.sum(diff * diff, axis=2))
            # row side: K_ij (G_j + 2a (x_i - x_j)) -> i
            S[rows] += K @ G[cols] + 2.0 * a * np.einsum("ij,ijk->ik", K, diff)
            if I != J:  # column side: K_ij (G_i + 2a (x_j - x_i)) -> j
                S[cols] += K.T @ G[rows] - 2.0 * a * np.einsum("ij,ijk->jk", K, diff)
                pairs += rows.size * cols.size
            else:
                pairs += rows.size * cols.size  # ordered pairs of the square's columns (incl. i = j)
        tot = torch.from_numpy(S)
        dist.all_reduce(tot)  # the reduce-scatter's sums (every rank keeps its rows below)
        pc = torch.tensor([pairs], dtype=torch.int64)
        dist.all_reduce(pc)
        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        lib.svgd_plan_rows(n, world, rank, ctypes.byref(r0), ctypes.byref(r1))
        phi = tot.numpy()[r0.value:r1.value] / n
        rows_phi = [None] * world
        dist.all_gather_object(rows_phi, (r0.value, r1.value, phi))
        if rank == 0:
            q.put(("ok", {"X": X, "G": G, "rows": rows_phi, "pairs": int(pc.item())}))
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))
