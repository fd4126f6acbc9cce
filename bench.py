"""Headline benchmark: SVGD inner step, N=65536 particles, d=8, GMM(k=4), fp64.

    python bench.py [--gpus N] [--steps K] [--warmup W]

BASELINE.json metric: particle-updates/s (N x steps / s) at N=65536, d=8
(cfg3).  One step = SVGD::Step of the reference (SVGD.hpp:373-400):
median-heuristic scale of X_t, host-side grad log p(X_t) for this rank's rows
(C++ closed form, OpenMP), phi_hat, Adam increment, X update -- all of it
inside the timed region, X resident in HBM.  For N GPUs (one process each,
torchrun) the particles are sharded by rows and the context all-gathers X and
G over RCCL every step; N is fixed (strong scaling, as the metric specifies).

Protocol: W warm-up steps, then `--repeats` (5) timed runs of
exactly K steps, each bracketed by barrier + device sync; value/ms_per_step
are the median run (per run the slowest rank).  Then one untimed diagnostic
pass of K steps with extra HIP events (the phi kernel alone, the device's
wait for G, collectives).

The JSON line also carries
  roofline     -- the phi kernel (dominant): algorithmic flop per launch
                  (rows x N x (5d+4)) / its average launch time
                  from HIP events around that launch alone (diagnostic pass),
                  against the FP64 peak (78.6 TF/s, MI355X spec; vector =
                  matrix); frac_at_load_clock uses the gfx clock amdsmi read
                  during the same pass.
  phases / host / diag -- where a step's time goes: the phi and median
                  phases (timed runs), the host gradient's wall clocks, the
                  device's wait for G before the phi chain (diagnostic pass).
  gpu_timed / gpu_diag -- amdsmi clock, power, throttle residency over the
                  timed runs / the diagnostic pass.
  cpu_baseline -- the CPU oracle (a port of the reference's arithmetic) on all
                  host cores this process may use, for a bounded row sample of
                  the same workload (rank 0, N=1 only), plus a 1-thread number.
  per_rank     -- (N > 1) every rank's phases, host and diagnostic times.
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
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense


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
# cpu_rows: the cpu_baseline's row sample (its median work is rows x N/2
# distances, ~10-30 s of the port's work on the box's 16 threads)
CONFIGS = {
    "cfg2": dict(n=16384, d=2, cpu_rows=16384, desc="N=16384 d=2 multivariate normal (mvn_example parameters)"),
    "cfg3": dict(n=65536, d=8, cpu_rows=32768, desc="N=65536 d=8 GMM(k=4)"),
    "cfg4": dict(n=262144, d=8, cpu_rows=8192, desc="N=262144 d=8 GMM(k=4)"),
    "cfg5": dict(n=65536, d=64, dtype="f32", cpu_rows=8192, desc="N=65536 d=64 multivariate normal, fp32 compute"),
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


def _cpu_quota():
    """CPUs this process's cgroup may use (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


class GpuMonitor:
    """Samples the GPU's clock, power and throttle residency through amdsmi
    (host-side sysfs/SMU reads; nothing is queued on the GPU) in a thread,
    so the line carries the clock THIS run held, not one from another box."""

    ACC = ("ppt_residency_acc", "socket_thm_residency_acc", "prochot_residency_acc",
           "hbm_thm_residency_acc", "vr_thm_residency_acc")

    def __init__(self, device, period=0.02):
        import threading

        self.ok, self.err, self.h, self.samples = False, None, None, []
        self.period, self.static = period, {}
        self._stop = threading.Event()
        self._th = None
        try:
            import amdsmi

            self.smi = amdsmi
            amdsmi.amdsmi_init()
            bdf = _pci_bus_id(device)
            hs = amdsmi.amdsmi_get_processor_handles()
            for h in hs:
                if bdf and amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == bdf.lower():
                    self.h = h
            if self.h is None and len(hs) == 1:
                self.h = hs[0]
            if self.h is None:
                raise RuntimeError(f"no amdsmi handle for {bdf} among {len(hs)}")
            self.static["bdf"] = bdf
            try:
                cap = amdsmi.amdsmi_get_power_cap_info(self.h)
                self.static["power_cap_w"] = cap["power_cap"] / 1e6
                self.static["default_power_cap_w"] = cap["default_power_cap"] / 1e6
            except Exception as e:  # noqa: BLE001 - diagnostics only
                self.static["power_cap_err"] = str(e)[:80]
            try:
                ci = amdsmi.amdsmi_get_clock_info(self.h, amdsmi.AmdSmiClkType.GFX)
                self.static["gfxclk_max_mhz"] = ci.get("max_clk")
            except Exception as e:  # noqa: BLE001
                self.static["clock_info_err"] = str(e)[:80]
            self.ok = True
        except Exception as e:  # noqa: BLE001 - no amdsmi: the line says so
            self.err = f"{type(e).__name__}: {str(e)[:120]}"

    def _read(self):
        m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
        clks = m.get("current_gfxclks")
        if isinstance(clks, (list, tuple)):
            clks = [c for c in clks if isinstance(c, (int, float)) and 0 < c < 10000]
        clk = (sum(clks) / len(clks)) if clks else m.get("current_gfxclk")
        out = {"t": time.perf_counter(), "gfxclk": clk, "power": m.get("current_socket_power"),
               "hotspot": m.get("temperature_hotspot"), "throttle": m.get("indep_throttle_status"),
               "acc_count": m.get("accumulation_counter")}
        for k in self.ACC:
            out[k] = m.get(k)
        return out

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._read())
            except Exception as e:  # noqa: BLE001
                self.err = f"{type(e).__name__}: {str(e)[:120]}"
                return
            self._stop.wait(self.period)

    def start(self):
        import threading

        if not self.ok:
            return self
        self.samples = []
        self._stop.clear()
        self._th = threading.Thread(target=self._loop, daemon=True)
        self._th.start()
        return self

    def stop(self):
        if self._th is not None:
            self._stop.set()
            self._th.join()
            self._th = None
        return self.summary()

    def summary(self):
        if not self.ok:
            return {"source": "amdsmi", "error": self.err}
        s = [x for x in self.samples if isinstance(x.get("gfxclk"), (int, float))]
        out = {"source": "amdsmi gpu_metrics (current_gfxclks mean over XCDs), this run",
               "samples": len(self.samples), **self.static}
        if s:
            c = sorted(x["gfxclk"] for x in s)
            out.update(gfxclk_mhz_median=c[len(c) // 2], gfxclk_mhz_min=c[0], gfxclk_mhz_max=c[-1])
        p = sorted(x["power"] for x in self.samples if isinstance(x.get("power"), (int, float)))
        if p:
            out.update(power_w_median=p[len(p) // 2], power_w_max=p[-1])
        t = [x["hotspot"] for x in self.samples if isinstance(x.get("hotspot"), (int, float))]
        if t:
            out["hotspot_c_max"] = max(t)
        th = sorted({x["throttle"] for x in self.samples if isinstance(x.get("throttle"), int)})
        if th:
            out["indep_throttle_status_seen"] = th
        # residency accumulators: share of the sampled span spent throttled
        if len(self.samples) >= 2:
            a, b = self.samples[0], self.samples[-1]
            if all(isinstance(x.get("acc_count"), int) for x in (a, b)) and b["acc_count"] > a["acc_count"]:
                dn = b["acc_count"] - a["acc_count"]
                for k in self.ACC:
                    if isinstance(a.get(k), int) and isinstance(b.get(k), int):
                        out[k.replace("_acc", "_frac")] = (b[k] - a[k]) / dn
        return out


def _pci_bus_id(device):
    """PCI bus id of a HIP device (hipDeviceGetPCIBusId), for the amdsmi handle."""
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) == 0:
            return buf.value.decode()
    except OSError:
        pass
    return None


def _cpu_sample(o, X0, mus, covs, rows):
    n, d = X0.shape
    t0 = time.perf_counter()
    o.median_rows_work(X0, 0, rows)
    G = o.logp_grad_gmm(X0, mus, covs)  # all rows: phi needs every G_j
    ph = o.phi(X0, G, 0.5, rows=(0, rows))  # the value of a is irrelevant to the cost
    Xs = X0[:rows].copy()
    o.apply_update(Xs, o.Adam((rows, d), 0.1, 0.9, 0.999).step(ph))
    return time.perf_counter() - t0


def accuracy_rows(n):
    """Rows whose phi_hat the line checks against the oracle: both ends and
    512 around n / 2 (as tests/test_gpu_fullsize.py samples them)."""
    return [(0, 256), (n // 2 - 256, n // 2 + 256), (n - 256, n)]


def phi_accuracy(o, X0, G0, a0, phi0, dtype):
    """The device's phi_hat of X0 (untimed, before the warm-up) on the
    accuracy rows against the oracle's fp64 phi_hat from the same (X, G, a):
    the observed error, next to the bar the GPU tests assert."""
    err, ref_max = 0.0, 0.0
    for r0, r1 in accuracy_rows(X0.shape[0]):
        ref = o.phi(X0, G0, a0, rows=(r0, r1))
        err = max(err, float(np.max(np.abs(phi0[r0:r1] - ref))))
        ref_max = max(ref_max, float(np.max(np.abs(ref))))
    out = {"rows": sum(r1 - r0 for r0, r1 in accuracy_rows(X0.shape[0])), "scale_a": a0,
           "phi_max_abs_err": err, "phi_max_abs": ref_max, "phi_err_rel_to_max": err / ref_max if ref_max else None,
           "reference": "oracle fp64 phi_hat (SVGD.hpp:407-454) of the same X, G, a"}
    out["bar"] = "<= 1e-4 max|phi| (F32, SURVEY A.9)" if dtype == "f32" else "<= 1e-10 absolute (fp64)"
    return out


def cpu_baseline(X0, mus, covs, rows, rows_1t, repeats=3, acc=None):
    """Oracle (CPU port of the reference arithmetic) on a row sample of one step:
    median work of `rows` rows, their log-gradients, phi_hat and Adam -- with
    the OpenMP threads of this box (OMP_NUM_THREADS) and with one thread;
    `repeats` timings each, the median reported.  acc = (G0, a0, phi0, dtype):
    also the device's phi_hat accuracy on a row sample (phi_accuracy)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o

    n, d = X0.shape
    rows, rows_1t = min(rows, n), min(rows_1t, n)
    # every core this process may use: the affinity mask, capped by the
    # cgroup's CPU quota when one is set (threads beyond it only get throttled)
    model, affinity = _host_cpu()
    quota = _cpu_quota()
    threads = max(1, min(affinity, int(quota)) if quota else affinity)
    keep = int(o.num_threads())
    o.set_threads(threads)
    dts = sorted(_cpu_sample(o, X0, mus, covs, rows) for _ in range(repeats))
    o.set_threads(1)
    dt1s = sorted(_cpu_sample(o, X0, mus, covs, rows_1t) for _ in range(repeats))
    accuracy = phi_accuracy(o, X0, *acc) if acc is not None else None
    o.set_threads(keep)
    dt, dt1 = dts[len(dts) // 2], dt1s[len(dt1s) // 2]
    return {
        "accuracy": accuracy,
        "value": rows / dt,
        "repeats": {"n": repeats, "rule": "median", "value_runs": [rows / t for t in dts],
                    "value_1thread_runs": [rows_1t / t for t in dt1s]},
        "unit": "particle-updates/s",
        "cores": threads,
        "kind": "port",
        "host_cpu": model,
        "host_cores": affinity,
        "cpu_quota": quota,
        "cores_rule": "min(len(sched_getaffinity), cgroup cpu.max quota)",
        "value_1thread": rows_1t / dt1,
        "sample": f"one step of the N={n} d={d} Gaussian-sum(k={len(mus)}) workload restricted to {rows} particle rows "
                  f"(their median pair share, grad log p of all N, phi_hat of {rows} rows against all N, "
                  f"Adam); {dt:.2f} s on {threads} OpenMP threads; 1 thread: {rows_1t} rows in {dt1:.2f} s",
        # why the thread scaling is far below `cores`: the reference's median
        # is std::nth_element + max_element over the N^2 distance list
        # (GaussianRBFKernel.hpp:222-254), serial in the reference, and the
        # port keeps it serial (the sample's rows x N/2 distances)
        "dominant_cost": f"the serial nth_element of the reference's ComputeMedian over the sample's "
                         f"{rows} x {n // 2} pair distances (serial in the reference as well)",
    }


def _kernel_src_sha():
    """First 16 hex digits of sha256 over the device sources (the key of the
    committed PMC profiles: a kernel edit leaves them unmatched)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("svgd_kernels.hip", "svgd_collect.hip", "svgd_kernels.h"):
        with open(os.path.join(ROOT, "svgdcpp_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def spawn_ranks(nproc, argv=None, poll=0.05, grace=20.0):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU) before anything touches a GPU and poll them.  The first rank that
    exits non-zero ends the others (a dead rank would leave them blocked in a
    collective until an outside timeout, with no line written): SIGTERM, then
    SIGKILL after `grace` seconds.  Returns 0, or the first failure's status
    (128 + signal for a rank killed by a signal)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    argv = [os.path.abspath(__file__)] + sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + argv, env=env))
    alive, rc = list(procs), 0
    while alive and rc == 0:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0:
                rc = r if r > 0 else 128 - r
                print(f"bench.py: rank {procs.index(p)} exited with status {r}; ending the other ranks",
                      file=sys.stderr, flush=True)
                break
        else:
            time.sleep(poll)
    for p in alive:
        p.terminate()
    deadline = time.time() + grace
    for p in alive:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
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
    ap.add_argument("--cpu-rows", type=int, default=None, help="cpu_baseline row sample (default: the config's)")
    ap.add_argument("--cpu-rows-1t", type=int, default=2048)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--repeats", type=int, default=5, help="timed runs of K steps; the median is reported")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="measurement only: time rank 0's share of a P-rank step on one GPU "
                         "(no collectives; results are not the step's) -- not a headline line")
    ap.add_argument("--no-diag", action="store_true", help="skip the untimed diagnostic pass")
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
                    dtype=C.SVGD_F32 if dtype == "f32" else C.SVGD_F64,
                    sim_world=args.sim_world if args.sim_world > 1 else None)
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
    ctx.diagnostics()  # (reset)
    # the timed runs carry no timing events at all (the product path: an
    # event between two kernels costs a ~6 us dispatch gap); the phase split
    # comes from the diagnostic pass below
    ctx.check(ctx.lib.svgd_set_timing(ctx.h, 0))

    # the median of `repeats` timed runs of exactly K steps, each
    # bracketed by barrier + device sync; the GPU's clock/power sampled by
    # amdsmi over the same span
    mon = GpuMonitor(local_rank).start()
    runs = []
    for _ in range(args.repeats):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        ctx.sync()
        torch.cuda.synchronize()
        barrier()
        runs.append(time.perf_counter() - t0)
    gpu_timed = mon.stop()
    phi_ms, med_ms, cnt = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    host_timed = ctx.diagnostics()  # host-side clocks of the timed steps (always on)

    # diagnostic pass (untimed): the phi kernel alone, the device's wait for
    # G before the phi chain, collectives -- extra events, so not in the runs
    diag = None
    gpu_diag = None
    if not args.no_diag:
        ctx.check(ctx.lib.svgd_set_timing(ctx.h, 2))
        mon.start()
        for _ in range(args.steps):
            step()
        ctx.sync()
        gpu_diag = mon.stop()
        diag = ctx.diagnostics()
        ctx.check(ctx.lib.svgd_get_timing(ctx.h, ctypes.byref(phi_ms), ctypes.byref(med_ms), ctypes.byref(cnt)))
        ctx.check(ctx.lib.svgd_set_timing(ctx.h, 0))

    a, med, path = ctx.last_scale()
    rows = ctx.row1 - ctx.row0
    elapsed = sorted(runs)[len(runs) // 2]  # this rank's median run
    if dist is not None:
        t = torch.tensor(runs, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # per run: the slowest rank
        runs = [float(x) for x in t.tolist()]
        elapsed = sorted(runs)[len(runs) // 2]

    def per_step(v, k):
        return v / k if k else None

    mine = {
        "rank": rank, "rows": rows,
        # phase events at phase boundaries, from the diagnostic pass (level 2:
        # its extra events make these spans a few us longer than the timed
        # steps'):
        # "phi" runs from the median's end (so it holds any wait for G) to the
        # update's end, "median" from the previous step's end (so it holds the
        # gap between steps) to the scale; the diagnostic pass separates both
        "phases_ms_per_step": {"phi_incl_wait_for_g": per_step(phi_ms.value, args.steps if diag is not None else 0),
                               "median_incl_step_gap": per_step(med_ms.value, args.steps if diag is not None else 0),
                               "source": "diagnostic pass"},
        "host_ms_per_step": {"grad": per_step(host_timed["host_grad_ms"], host_timed["steps"]),
                             "xwait": per_step(host_timed["host_xwait_ms"], host_timed["steps"]),
                             "job": per_step(host_timed["host_job_ms"], host_timed["steps"]),
                             "caller_wait": per_step(host_timed["host_wait_ms"], host_timed["steps"]),
                             "threads": host_timed["host_threads"],
                             # the gradient's threads: min(OMP threads / 2, cgroup quota / ranks);
                             # a --sim-world rank models one GPU's share of a P-GPU node (CPUs are
                             # leased per GPU): this box's whole quota
                             "cpu_quota": host_timed["cpu_quota"],
                             "ranks_sharing_quota": 1 if args.sim_world > 1 else world},
        # speculative steps whose median bracket was predicted from the last
        # medians (no sample), and of those the ones redone after a miss
        "tracked_brackets": {"steps": int(host_timed["steps"]), "predicted": int(host_timed["trk_steps"]),
                             "missed": int(host_timed["trk_miss"]),
                             # the predicted brackets' mean share of the pairs (the
                             # collect stages and finishes those exactly)
                             "mean_band_share": (host_timed["trk_band"] / host_timed["trk_steps"]
                                                 if host_timed.get("trk_steps") else None)},
    }
    # phi launches per step: 2 when the context runs phi in row halves
    # (P > 1 with few gradient threads per rank)
    parts = max(1, round(diag["phi_kernel_n"] / args.steps)) if diag is not None and diag["phi_kernel_n"] else 1
    if diag is not None:
        mine["diag_ms_per_step"] = {
            "phi_kernel": per_step(diag["phi_kernel_ms"], diag["phi_kernel_n"] / parts),
            "phi_launches_per_step": parts,
            "phi_wait_for_g": per_step(diag["phi_wait_ms"], diag["phi_wait_n"]),
            "collectives": per_step(diag["coll_ms"], args.steps),
            "g_allgather": per_step(diag["gather_g_ms"], args.steps),
            "host_grad": per_step(diag["host_grad_ms"], diag["steps"]),
        }
        mine["n_ranks_seen"] = int(diag["ranks"])
    mine["phi_kernel"] = ctx.phi_kernel_name()
    per_rank = [mine]
    if dist is not None:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    if rank == 0:
        phi_step_ms = (mine.get("diag_ms_per_step") or {}).get("phi_kernel")
        phi_kernel_ms = phi_step_ms / parts if phi_step_ms else None  # one launch
        flops_launch = float(rows) * n * (5 * d + 4) / parts
        achieved = flops_launch / (phi_kernel_ms / 1e3) / 1e12 if phi_kernel_ms else None
        peak = FP32_PEAK_TFLOPS if dtype == "f32" else FP64_PEAK_TFLOPS
        b3 = None
        if ctx.phi_kernel_name().startswith("k_phi_b3"):
            # fp32 products as six bf16 part products on the bf16 matrix cores:
            # the MFMA work per ordered pair is 6 x 2 x (KP + 16 NCB) flops
            # (Gram over KP padded dims, P.V over the padded V width), so the
            # ceiling for the algorithmic flops is the bf16 dense peak scaled
            # by algorithmic / MFMA flops
            kp = 32 if d <= 32 else 64
            ncb = d // 16 if d % 16 == 0 else (d + 16) // 16
            mfma_pair = 6.0 * 2.0 * (kp + 16 * ncb)
            peak = BF16_PEAK_TFLOPS * (5 * d + 4) / mfma_pair
            b3 = {"peak_basis": f"bf16 dense MFMA peak {BF16_PEAK_TFLOPS:.0f} TF/s x algorithmic / MFMA flops "
                                f"per pair ({5 * d + 4} / {mfma_pair:.0f}: six bf16 part products per fp32 product)",
                  "fp32_mfma_peak_frac": (achieved / FP32_PEAK_TFLOPS) if achieved else None,
                  "bf16_mfma_tflops": (achieved * mfma_pair / (5 * d + 4)) if achieved else None}
        # committed PMC passes (not this run) count only for the same kernel
        # (name + template arguments, svgd_phi_kernel_name), the same kernel
        # source (hash of svgd_kernels.hip) and the same workload (N, d, P)
        wkey = args.sim_world if args.sim_world > 1 else world  # the profiles' world
        kname = ctx.phi_kernel_name()
        src_sha = _kernel_src_sha()

        def committed(name):
            path = os.path.join(ROOT, "profiles", name)
            if not os.path.exists(path):
                return None
            with open(path) as f:
                recs = json.load(f)
            for p in recs if isinstance(recs, list) else [recs]:  # one record per kernel / workload
                if (p.get("n") == n and p.get("d") == d and p.get("world") == wkey and kname in p.get("kernel", "")
                        and p.get("src_sha16") == src_sha):
                    return p
            return None

        pmc = committed("phi_pmc_traffic.json")
        traffic = pmc.get("bytes_per_launch") if pmc else None
        issue = committed("phi_pmc_issue.json")
        row_kernel = dtype == "f64" and d <= 16
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
            "repeats": {"n": len(runs), "rule": "value/ms_per_step = median run (max over ranks per run)",
                        "ms_per_step": [r / args.steps * 1e3 for r in runs]},
            "roofline": {
                # fp64 d <= 16: VALU row stream (f64 MFMA shares the VALU issue
                # slots on gfx950); otherwise the MFMA tile kernel.
                # avg_launch_ms: HIP events around the phi kernel launch alone
                # (diagnostic pass after the timed runs; k_phi_rows without
                # its reduce), so it is comparable with rocprof's kernel mean
                "kernel": ("k_phi_sym (fused RBF + grad + phi contraction, symmetric: one Gram and one exp "
                           "per unordered pair feed both particles; fp64 VALU)"
                           if kname.startswith("k_phi_sym") else
                           "k_phi_rows (fused RBF + grad + phi contraction, fp64 VALU row stream)"
                           if row_kernel else
                           "k_phi_b3 (fused RBF + grad + phi contraction, fp32-accurate on the bf16 "
                           "matrix cores: three-part operands, six part products)"
                           if b3 else
                           "k_phi_f32s (fused RBF + grad + phi contraction, streamed fp32 MFMA tiles)"
                           if dtype == "f32" and d > 12 else
                           "k_phi (fused RBF + grad + phi contraction, MFMA tiles)"),
                "timed_span": "the phi kernel launch alone (HIP events, diagnostic pass)",
                "bound": "valu" if row_kernel else "mfma",
                "achieved": achieved,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": (achieved / peak) if achieved else None,
                "traffic": traffic,
                "traffic_source": (pmc or {}).get("source") if traffic else
                                  f"none committed for {kname} at this source hash / workload",
                "kernel_launched": kname,
                "avg_launch_ms": phi_kernel_ms,
                "flop_per_launch": flops_launch,
            },
            "phases_ms_per_step": mine["phases_ms_per_step"],
            "host_ms_per_step": mine["host_ms_per_step"],
            "tracked_brackets": mine["tracked_brackets"],
            "diag_ms_per_step": mine.get("diag_ms_per_step"),
            "gpu_timed": gpu_timed,
            "gpu_diag": gpu_diag,
            "median_path": ["direct", "bracket", "fallback", "rebracket"][path],
            "scale_a": a,
            # every SVGD_* variable of this run (library knobs; none by default)
            "env_knobs": {k: v for k, v in sorted(os.environ.items()) if k.startswith("SVGD_")},
        }
        if b3:
            out["roofline"].update(b3)
        if world > 1:
            out["per_rank"] = per_rank
        clk = (gpu_diag or {}).get("gfxclk_mhz_median")
        if achieved and clk:
            # the flop fraction against the peak at the clock this run held
            # under the phi kernel (amdsmi, same run): the ceiling this
            # instruction mix can reach on this box
            out["roofline"]["clock_mhz_under_load"] = clk
            out["roofline"]["frac_at_load_clock"] = achieved / (peak * clk / 2400.0)
        if issue is not None:
            out["roofline"].update({"valu_issue_util": issue["valu_issue_util"],
                                    "issue_source": issue["source"]})
        if args.sim_world > 1:
            out["metric"] = (f"per-rank step time of a {args.sim_world}-GPU run, simulated on one GPU "
                             f"(rank 0's rows and pair share, no collectives; not the headline)")
            out["value"] = None
            out["sim_world"] = args.sim_world
        elif args.config != "cfg3" or args.device_model or dtype != "f64":
            desc = cfg["desc"]
            if dtype != cfg.get("dtype", "f64"):
                desc = desc.replace("fp32 compute", "fp64 compute") + (", fp32 compute" if dtype == "f32" and "fp32" not in desc else "")
            out["metric"] = (f"particle-updates/s, {desc}"
                             f"{', device grad log p' if args.device_model else ''} (not the headline config)")
        if world == 1 and not args.no_cpu:
            # the device's phi_hat of X0 for the CPU leg's accuracy record,
            # after the timed runs (X0 set again: the centring, median and phi
            # of X0 are those of a fresh context).  Run before the warm-up it
            # left the first timed runs up to 55 % slower (profiles/r05_acc_prepass_ab.txt)
            acc = None
            if args.sim_world <= 1:
                ctx.set_particles(X0)
                G0 = model.log_model_grad(X0)
                a0, _ = ctx.median_scale()
                acc = (G0, a0, ctx.phi(G0, a0), dtype)
            out["cpu_baseline"] = cpu_baseline(X0, mus, covs, args.cpu_rows or cfg["cpu_rows"], args.cpu_rows_1t,
                                               acc=acc)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
