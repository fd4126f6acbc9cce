"""Rank body of tests/test_gpu_multirank.py: one process per rank, all ranks
on cuda device 0, collectives through the SVGD_HOSTCOMM host backend (RCCL
refuses two ranks on one device).  Exercises the library's sharded step --
row shards, pair-tile median with all-reduced counts/histograms, all-gathers
of G and X -- on the real kernels."""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run(rank, world, name, n, d, steps, q, env=None):
    try:
        os.environ["SVGD_HOSTCOMM"] = name
        os.environ.update(env or {})
        import oracle as O
        import svgdcpp_amd as S
        from svgdcpp_amd import _capi as C

        X0 = O.splitmix((n, d), 3.0, 41)
        if os.environ.get("SVGD_TEST_OUTLIERS"):  # far particles: a log2e max|xc|^2 > 300
            X0[:3] += float(os.environ["SVGD_TEST_OUTLIERS"])
        mus = O.splitmix((3, d), 3.0, 42)
        covs = [np.eye(d) * (1.0 + 0.25 * c) for c in range(3)]
        ctx = S.Context(d, n, device=0, world=world, rank=rank)
        ctx.set_particles(X0)
        ctx.set_optimizer(C.SVGD_OPT_ADAM, 0.05, 0.9, 0.999, 1e-8)
        ctx.set_bounds(-np.full(d, 2.5), np.full(d, 2.5))
        model = S.GaussianSum(list(mus), list(covs))
        scales = []
        ctx.diagnostics()
        for _ in range(steps):
            ctx.step_with_model(model)
            scales.append(ctx.last_scale()[:3])
        X = ctx.get_particles()
        shard = (ctx.row0, ctx.row1)
        diag = dict(ctx.diagnostics())
        diag["phi_kernel"] = ctx.phi_kernel_name()
        if os.environ.get("TEST_PHI_CHECK"):
            # one more sharded phi of X_T (this rank's rows): scale, the
            # all-gather of G and the phi exchange, against the oracle in the test
            G = model.log_model_grad(X[shard[0]:shard[1]])
            a, _ = ctx.median_scale()
            diag["phi_rows"] = ctx.phi(G, a)
            diag["phi_a"] = a
            diag["phi_kernel_check"] = ctx.phi_kernel_name()
        ctx.close()
        q.put(("ok", rank, X, scales, shard, diag))
    except Exception:
        q.put(("err", rank, traceback.format_exc(), None, None, None))
