"""Headline benchmark: SVGD inner step, N=65536 particles, d=8, GMM(k=4), fp64.

    python bench.py [--gpus N] [--steps K] [--warmup W]

BASELINE.json metric: particle-updates/s (N x steps / s) at N=65536, d=8
(cfg3).  One step = SVGD::Step of the reference (SVGD.hpp:373-400):
median-heuristic scale of X_t, host-side grad log p(X_t) for this rank's rows
(C++ closed form, OpenMP), phi_hat, Adam increment, X update -- all of it
inside the timed region, X resident in HBM.  For N GPUs (one process each,
torchrun) the particles are sharded by rows and the context all-gathers X and
G over RCCL every step; N is fixed (strong scaling, as the metric specifies).

The JSON line also carries
  roofline     -- the phi kernel (dominant) measured with HIP events on the
                  library's own stream: algorithmic flop per launch
                  (rows x N x (5d+4)) / average launch time,
                  against the FP64 peak (78.6 TF/s, MI355X spec; vector = matrix).
  cpu_baseline -- the CPU oracle (a port of the reference's arithmetic) on the
                  host cores of this box for a bounded row sample of the same
                  workload (rank 0, N=1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "particle-updates/sec (N×iters/s) + per-step ms, N=65536 d=8, 1/2/4/8 GPU"
FP64_PEAK_TFLOPS = 78.6  # MI355X spec (not in MI355X_MICROARCH.md; vector = matrix for fp64)
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix = vector (v_mfma_f32_16x16x4_f32)


def splitmix(shape, scale, seed):
    """splitmix64 -> uniform[-1,1) (SURVEY §8(d) synthetic inputs), vectorised."""
    cnt = int(np.prod(shape))
    with np.errstate(over="ignore"):
        s = (np.uint64(seed) + np.arange(1, cnt + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = s.copy()
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    return (scale * (u * 2.0 - 1.0)).reshape(shape)


def workload(n, d, k):
    """cfg3 (and cfg4): GMM with k unweighted unnormalised components."""
    X0 = splitmix((n, d), 3.0, 0x5EED)
    mus = splitmix((k, d), 3.0, 0x5EEE)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    return X0, mus, covs


# SURVEY §8(d) configurations (the default cfg3 is the headline metric; the
# others are reported on request: --config cfg2 / cfg5)
CONFIGS = {
    "cfg2": dict(n=16384, d=2, desc="N=16384 d=2 multivariate normal (mvn_example parameters)"),
    "cfg3": dict(n=65536, d=8, desc="N=65536 d=8 GMM(k=4)"),
    "cfg4": dict(n=262144, d=8, desc="N=262144 d=8 GMM(k=4)"),
    "cfg5": dict(n=65536, d=64, dtype="f32", desc="N=65536 d=64 multivariate normal, fp32 compute"),
}


def config_workload(name, n, d, k):
    if name == "cfg2":
        mu = np.array([[-0.6871, 0.8010]])
        cov = 5.0 * np.array([[[0.2260, 0.1652], [0.1652, 0.6779]]])
        return splitmix((n, d), 3.0, 0x5EED), mu, cov
    if name == "cfg5":
        return splitmix((n, d), 3.0, 0x5EED), splitmix((1, d), 0.5, 0x5EEE), np.eye(d)[None]
    return workload(n, d, k)


def _host_cpu():
    """CPU model (as lscpu prints it) and the cores this process may run on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    return model, cores


def _cpu_sample(o, X0, mus, covs, rows):
    n, d = X0.shape
    t0 = time.perf_counter()
    o.median_rows_work(X0, 0, rows)
    G = o.logp_grad_gmm(X0, mus, covs)  # all rows: phi needs every G_j
    ph = o.phi(X0, G, 0.5, rows=(0, rows))  # the value of a is irrelevant to the cost
    Xs = X0[:rows].copy()
    o.apply_update(Xs, o.Adam((rows, d), 0.1, 0.9, 0.999).step(ph))
    return time.perf_counter() - t0


def cpu_baseline(X0, mus, covs, rows, rows_1t):
    """Oracle (CPU port of the reference arithmetic) on a row sample of one step:
    median work of `rows` rows, their log-gradients, phi_hat and Adam -- with
    the OpenMP threads of this box (OMP_NUM_THREADS) and with one thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o

    n, d = X0.shape
    rows, rows_1t = min(rows, n), min(rows_1t, n)
    threads = int(o.num_threads())
    dt = _cpu_sample(o, X0, mus, covs, rows)
    o.set_threads(1)
    dt1 = _cpu_sample(o, X0, mus, covs, rows_1t)
    o.set_threads(threads)
    model, host_cores = _host_cpu()
    return {
        "value": rows / dt,
        "unit": "particle-updates/s",
        "cores": threads,
        "kind": "port",
        "host_cpu": model,
        "host_cores": host_cores,
        "value_1thread": rows_1t / dt1,
        "sample": f"one step of the N={n} d={d} Gaussian-sum(k={len(mus)}) workload restricted to {rows} particle rows "
                  f"(their median pair share, grad log p of all N, phi_hat of {rows} rows against all N, "
                  f"Adam); {dt:.2f} s on {threads} OpenMP threads; 1 thread: {rows_1t} rows in {dt1:.2f} s",
    }


def spawn_ranks(nproc):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU) before anything touches a GPU, wait, exit with the worst status."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--d", type=int, default=None)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--cpu-rows", type=int, default=32768)
    ap.add_argument("--cpu-rows-1t", type=int, default=2048)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dtype", choices=["f64", "f32"], default=None,
                    help="compute dtype of the O(N^2) work (default: the config's; cfg5 is f32)")
    ap.add_argument("--device-model", action="store_true",
                    help="grad log p on the device (SURVEY 8(f) rank 1) instead of the host; "
                         "not the north-star configuration")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import svgdcpp_amd as S
    from svgdcpp_amd import _capi as C

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal only: every rank on one device (SVGD_BENCH_DEVICE=0)
    if os.environ.get("SVGD_BENCH_DEVICE") is not None:
        local_rank = int(os.environ["SVGD_BENCH_DEVICE"])
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)

    cfg = CONFIGS[args.config]
    n = args.n or cfg["n"]
    d = args.d or cfg["d"]
    k = args.k
    dtype = args.dtype or cfg.get("dtype", "f64")
    X0, mus, covs = config_workload(args.config, n, d, k)
    k = len(mus)

    uid = None
    if world > 1:
        box = [S.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    ctx = S.Context(d, n, device=local_rank, world=world, rank=rank, unique_id=uid,
                    dtype=C.SVGD_F32 if dtype == "f32" else C.SVGD_F64)
    ctx.set_particles(X0)
    ctx.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    model = S.GaussianSum(list(mus), list(covs))
    if args.device_model:
        ctx.set_device_model(model)

    def step():
        if args.device_model:
            ctx.step_device()
        else:
            ctx.step_with_model(model)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    ctx.sync()
    ctx.check(ctx.lib.svgd_get_timing(ctx.h, None, None, None))  # drop warmup events
    ctx.check(ctx.lib.svgd_set_timing(ctx.h, 1))

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0

    phi_ms, med_ms, cnt = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    ctx.check(ctx.lib.svgd_get_timing(ctx.h, ctypes.byref(phi_ms), ctypes.byref(med_ms), ctypes.byref(cnt)))
    a, med, path = ctx.last_scale()
    rows = ctx.row1 - ctx.row0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        phi_avg_s = phi_ms.value / max(1, cnt.value) / 1e3
        flops_launch = float(rows) * n * (5 * d + 4)
        achieved = flops_launch / phi_avg_s / 1e12 if phi_avg_s > 0 else None
        peak = FP32_PEAK_TFLOPS if dtype == "f32" else FP64_PEAK_TFLOPS
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "phi_pmc_traffic.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("n") == n and pmc.get("d") == d and pmc.get("world") == world:
                traffic = pmc.get("bytes_per_launch")
        issue = None  # SQ counters of the same kernel (committed profile, not this run)
        issue_path = os.path.join(ROOT, "profiles", "phi_pmc_issue.json")
        if os.path.exists(issue_path):
            with open(issue_path) as f:
                iss = json.load(f)
            if iss.get("n") == n and iss.get("d") == d and iss.get("world") == world and dtype == "f64":
                issue = iss
        out = {
            "metric": METRIC,
            "value": n * args.steps / elapsed,
            "unit": "particle-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (splitmix64 X0 = 3*U[-1,1]^d, GMM means 3*U[-1,1]^d, cov_k = (1+0.25k) I)",
            "config": {
                "workload": f"{args.config}: N={n} d={d} {'GMM(k=%d)' % k if k > 1 else 'MVN'} "
                            f"RBF-median + Adam(0.1,0.9,0.999), {dtype} compute, "
                            f"{'device' if args.device_model else 'host'} grad log p per step",
                "n": n, "d": d, "k": k, "parallelism": f"rows{world}",
            },
            "roofline": {
                # fp64 d <= 16: VALU row stream (f64 MFMA shares the VALU issue
                # slots on gfx950); otherwise the MFMA tile kernel
                # avg_launch_ms: HIP events around the phi phase on the
                # context's stream -- record prep + the phi kernel + its reduce
                # (with the fused optimizer update on the row path); the phi
                # kernel is > 99 % of it at cfg3 (profiles/r02_*kernel_stats*)
                "kernel": ("k_phi_rows (fused RBF + grad + phi contraction, fp64 VALU row stream)"
                           if dtype == "f64" and d <= 16 else
                           "k_phi_f32s (fused RBF + grad + phi contraction, streamed fp32 MFMA tiles)"
                           if dtype == "f32" and d > 12 else
                           "k_phi (fused RBF + grad + phi contraction, MFMA tiles)"),
                "timed_span": ("k_prep_rec + k_phi_rows + k_phi_reduce (fused update)"
                               if dtype == "f64" and d <= 16 else
                               "k_prep_v + k_swz_f32 + k_cvt_f32 + k_phi_f32s"
                               if dtype == "f32" and d > 12 else "k_prep_v + k_phi (+ cvt)"),
                "bound": "valu" if dtype == "f64" and d <= 16 else "mfma",
                "achieved": achieved,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": (achieved / peak) if achieved else None,
                "traffic": traffic,
                "avg_launch_ms": phi_avg_s * 1e3,
                "flop_per_launch": flops_launch,
            },
            "phases_ms_per_step": {"phi": phi_ms.value / max(1, args.steps),
                                   "median": med_ms.value / max(1, args.steps)},
            "median_path": ["direct", "bracket", "fallback", "rebracket"][path],
            "scale_a": a,
        }
        if issue is not None:
            # issue-slot view beside the flop fraction: the fp64 VALU pipe's
            # share of issue slots used, and the clock the chip holds under this
            # load (DVFS) -- the flop fraction at that clock is the ceiling this
            # instruction mix can reach
            clk = issue["clock_ghz_under_load"]
            out["roofline"].update({
                "valu_issue_util": issue["valu_issue_util"],
                "clock_ghz_under_load": clk,
                "frac_at_load_clock": (achieved / (peak * clk / 2.4)) if achieved else None,
                "issue_source": issue["source"],
            })
        if args.config != "cfg3" or args.device_model or dtype != "f64":
            desc = cfg["desc"]
            if dtype != cfg.get("dtype", "f64"):
                desc = desc.replace("fp32 compute", "fp64 compute") + (", fp32 compute" if dtype == "f32" and "fp32" not in desc else "")
            out["metric"] = (f"particle-updates/s, {desc}"
                             f"{', device grad log p' if args.device_model else ''} (not the headline config)")
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(X0, mus, covs, args.cpu_rows, args.cpu_rows_1t)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
