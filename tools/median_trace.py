"""The selected median of D^2 per step (bench.py's workload and step), for
offline study of the bracket predictor (svgd_capi.cpp trk_predict).
Usage: python tools/median_trace.py cfg5 130 out.json"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    name, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import torch
    import svgdcpp_amd as S
    from svgdcpp_amd import _capi as C

    torch.cuda.set_device(0)
    cfg = bench.CONFIGS[name]
    X0, mus, covs = bench.config_workload(name, cfg["n"], cfg["d"], 4)
    ctx = S.Context(cfg["d"], cfg["n"], device=0, dtype=C.SVGD_F32 if cfg.get("dtype") == "f32" else C.SVGD_F64)
    ctx.set_particles(X0)
    ctx.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    model = S.GaussianSum(list(mus), list(covs))
    meds, paths = [], []
    for t in range(steps):
        ctx.step_with_model(model)
        a, m, p = ctx.last_scale()
        meds.append(m)
        paths.append(p)
    json.dump({"config": name, "med": meds, "path": paths, "diag": ctx.diagnostics()}, open(out, "w"))
    print(name, "done", meds[:3], meds[-3:])


if __name__ == "__main__":
    main()
