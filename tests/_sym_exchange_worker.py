"""Rank body of tests/test_sym_exchange_cpu.py: the sharded symmetric phi
pass's protocol (svgd_capi.cpp run_phi, DESIGN §4.1 "Sharded") with gloo in
place of RCCL and numpy as the arithmetic.  Rank r takes the (tile, 64-column
sub-tile) units svgd_plan_sym_units gives it, adds every unit's pair terms
to BOTH particles (row side; column side off the diagonal tiles, whose row
side already holds every ordered pair of the square), then the point-to-point
exchange of svgd_plan_sym_exchange: rank r sends each peer q the range of q's
rows its units touch and receives from each peer the range of its own rows
that peer touches (every particle sum outside the planned ranges must be
exactly zero), adds the pieces in rank order and forms phi for its rows
(svgd_plan_rows)."""
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
            t_, q_ = ctypes.c_int64(), ctypes.c_int64()
            assert lib.svgd_plan_sym_unit(n, block, nsub, u, ctypes.byref(t_), ctypes.byref(q_)) == 0
            t, sq = t_.value, q_.value
            I, J = ctypes.c_int64(), ctypes.c_int64()
            lib.svgd_plan_pair_tile(n, block, 1, 0, t, ctypes.byref(I), ctypes.byref(J))
            I, J = I.value, J.value
            rows = np.arange(I * block, min(n, (I + 1) * block))
            cols = np.arange(J * block + 64 * sq, min(n, J * block + 64 * (sq + 1)))
            assert cols.size > 0  # (padding-only sub-tiles are no units)
            if rows.size == 0:
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
        def plan(src, dst):
            a0, a1 = ctypes.c_int64(), ctypes.c_int64()
            lib.svgd_plan_sym_exchange(n, block, nsub, world, src, dst, ctypes.byref(a0), ctypes.byref(a1))
            return a0.value, a1.value

        # every particle this rank's units add to lies in a planned range
        covered = np.zeros(n, dtype=bool)
        for dst in range(world):
            a0, a1 = plan(rank, dst)
            covered[a0:a1] = True
        assert not np.any(S[~covered]), "a contribution outside the planned exchange ranges"
        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        lib.svgd_plan_rows(n, world, rank, ctypes.byref(r0), ctypes.byref(r1))
        r0, r1 = r0.value, r1.value
        # grouped point-to-point: the sends and receives of one step, then the
        # pieces added in rank order (k_sym_apply's order)
        reqs, pieces = [], {}
        for q_ in range(world):
            if q_ == rank:
                continue
            a0, a1 = plan(rank, q_)
            if a1 > a0:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(S[a0:a1])), q_))
            b0, b1 = plan(q_, rank)
            if b1 > b0:
                buf = torch.empty((b1 - b0, d), dtype=torch.float64)
                reqs.append(dist.irecv(buf, q_))
                pieces[q_] = (b0, buf)
        for rq in reqs:
            rq.wait()
        tot = np.zeros((r1 - r0, d))
        for q_ in range(world):
            if q_ == rank:
                tot += S[r0:r1]
            elif q_ in pieces:
                b0, buf = pieces[q_]
                tot[b0 - r0:b0 - r0 + buf.shape[0]] += buf.numpy()
        pc = torch.tensor([pairs], dtype=torch.int64)
        dist.all_reduce(pc)
        phi = tot / n
        rows_phi = [None] * world
        dist.all_gather_object(rows_phi, (r0, r1, phi))
        if rank == 0:
            q.put(("ok", {"X": X, "G": G, "rows": rows_phi, "pairs": int(pc.item())}))
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))
