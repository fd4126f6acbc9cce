"""The median over consecutive steps (GPU).

Every step's scale must be the exact median heuristic of that step's X_t
(GaussianRBFKernel.hpp:164-188, ComputeMedian :222-254, called once per
SVGD::Step, SVGD.hpp:373-400), whichever selection path the step takes:

* SVGD_BUCKET_CAP=0: every step runs the per-digit radix passes, whose
  select state is set from kernel arguments -- steps queued back to back with
  no host sync between them must give the same trajectory, bit for bit, as
  steps with a sync (and an oracle check) after each;
* the default bucket select with the speculative device plan;
* the automatic bracket sample size (sample_size left at 0 with M above
  direct_max_pairs) on the row-stream path (d <= 16, scattered pairs) and the
  tile paths (d > 16 fp64, and F32: whole 64 x 64 sample tiles).
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _run(oracle, X, dtype, model, steps, check):
    n, d = X.shape
    c = S.Context(d, n, dtype=dtype)
    c.set_particles(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    c.set_median_tuning(direct_max_pairs=0)  # bracket path; sample size stays automatic
    scales = []
    for step in range(steps):
        Xt = c.get_particles() if check else None
        c.step_with_model(model)
        if check:
            a, med, path = c.last_scale()
            assert path != C.SVGD_MEDIAN_DIRECT
            _, med_ref = oracle.median_scale(Xt)
            # fp64 keys: the exact median; F32 keys: fp32 pair distances
            rel = 1e-12 if dtype == C.SVGD_F64 else 1e-5
            assert med == pytest.approx(med_ref, rel=rel), step
            scales.append((a, med))
    a, med, _ = c.last_scale()
    out = c.get_particles()
    c.close()
    return out, (a, med), scales


@pytest.mark.parametrize("cap", ["0", None], ids=["radix-path", "bucket-path"])
@pytest.mark.parametrize("n,d,dtype", [(3000, 5, C.SVGD_F64), (2500, 20, C.SVGD_F64),
                                       (2600, 8, C.SVGD_F32)],
                         ids=["rows-f64", "tiles-f64", "tiles-f32"])
def test_back_to_back_steps_exact(oracle, monkeypatch, n, d, dtype, cap):
    if cap is None:
        monkeypatch.delenv("SVGD_BUCKET_CAP", raising=False)
    else:
        monkeypatch.setenv("SVGD_BUCKET_CAP", cap)
    monkeypatch.delenv("SVGD_MEDIAN_SAMPLE", raising=False)
    X = oracle.splitmix((n, d), 3.0, n + 7 * d)
    mus = oracle.splitmix((2, d), 2.0, 5)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.5 * k) for k in range(2)])
    Xq, last_q, _ = _run(oracle, X, dtype, model, 5, check=False)  # queued back to back
    Xs, last_s, scales = _run(oracle, X, dtype, model, 5, check=True)  # synced + oracle
    assert last_q == last_s == scales[-1]
    assert np.array_equal(Xq, Xs)
