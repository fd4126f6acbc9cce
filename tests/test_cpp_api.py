"""SVGDCpp-compatible C++ API (include/Core, Model, Kernel, Optimizer).

Builds the C++ example programs and tests/cpp/test_api.cpp against
libsvgdcpp_amd.so (``make cpp``) and runs them: the host-only checks on CPU,
the SVGD-class-vs-manual-loop checks (reference tests/test_svgd.cpp) on GPU.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")


def _make_cpp():
    r = subprocess.run(["make", "-s", "-C", ROOT, "cpp"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("mvn_example", "gmm_example", "test_api"):
        assert os.path.exists(os.path.join(BUILD, name)), name


def _run(args, timeout=300):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout, cwd=BUILD)


def test_cpp_api_builds_and_host_checks_pass():
    _make_cpp()
    r = _run([os.path.join(BUILD, "test_api"), "cpu"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


@pytest.mark.gpu
def test_cpp_svgd_class_matches_manual_loop():
    _make_cpp()
    r = _run([os.path.join(BUILD, "test_api")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def _matrix_after(text, header):
    """The d x n matrix printed after `header` (Eigen-style rows) -> (n, d)."""
    lines = text.split(header + "\n", 1)[1].split("\n")
    rows = []
    for ln in lines:
        try:
            rows.append([float(v) for v in ln.split()])
        except ValueError:
            break
        if not ln.strip():
            break
    rows = [r for r in rows if r]
    return np.array(rows).T


def _notebook_match(printed, expected):
    """Printed 6-significant-digit values equal the notebook's to the digit."""
    for a, b in zip(np.ravel(printed), np.ravel(expected)):
        assert f"{a:.6g}" == f"{b:.6g}" or abs(a - b) <= 1e-5 * max(abs(b), 1e-3), (a, b)


@pytest.mark.gpu
def test_cpp_examples_run(golden_dir):
    """The C++ examples over the device path reproduce the reference notebooks'
    printed final coordinates (mvn_example.ipynb:3658-3668,
    gmm_example.ipynb:6396-6416) to every printed digit."""
    _make_cpp()
    with open(os.path.join(golden_dir, "notebooks.json")) as f:
        nb = json.load(f)
    for name in ("mvn", "gmm"):
        r = _run([os.path.join(BUILD, f"{name}_example")])
        assert r.returncode == 0, r.stdout + r.stderr
        _notebook_match(_matrix_after(r.stdout, "Initial particle coordinates"), nb[name]["initial"])
        _notebook_match(_matrix_after(r.stdout, "Final particle coordinates"), nb[name]["final"])
    r = _run([os.path.join(BUILD, "gmm_example"), "4096", "50"])
    assert r.returncode == 0, r.stdout + r.stderr
    near = int(r.stdout.split("Particles nearer component A: ")[1].split()[0])
    # both mixture components are populated
    assert 0.2 * 4096 < near < 0.8 * 4096, r.stdout


# ------------------------------------------- intermediate-matrix log parity --

def _parse_log(path):
    """SVGD.hpp:345-365 text -> [(G (n,d), K_log (n,n), Kg_log (d n, n), X (n,d))] per step."""
    text = open(path).read()
    steps = []
    for block in re.split(r"========== Step \d+ ==========\n", text)[1:]:
        parts = {}
        for name in ("LogModelGrad", "Kernel", "KernelGrad", "CoordMat"):
            body = block.split(name + "=\n", 1)[1].split("\n\n", 1)[0]
            parts[name] = np.array([[float(v) for v in ln.split()] for ln in body.strip().split("\n")])
        steps.append((parts["LogModelGrad"].T, parts["Kernel"], parts["KernelGrad"], parts["CoordMat"].T))
    return steps


def _cosine_grad(X):
    """test_svgd.cpp:78-90 model gradient, (n, 2)."""
    x0, x1 = X[:, 0], X[:, 1]
    p = 7.5 * np.cos(x0) + 10.0 * np.cos(x1) + 3.0 * x0 * x1 - 6.0
    return np.stack([(-7.5 * np.sin(x0) + 3.0 * x1) / p, (-10.0 * np.sin(x1) + 3.0 * x0) / p], axis=1)


def _check_log(oracle, which, tmp_path, model_grad, scale_fn):
    log = str(tmp_path / f"log_{which}.txt")
    r = _run([os.path.join(BUILD, "test_api"), "log", which, log])
    assert r.returncode == 0, r.stdout + r.stderr
    X = _matrix_after(r.stdout, "INITIAL")
    steps = _parse_log(log)
    n, d = X.shape
    for G_log, K_log, Kg_log, X_new in steps:
        G = model_grad(X)
        a = scale_fn(X)
        _, K, Kg = oracle.phi(X, G, a, materialise=True)
        np.testing.assert_allclose(G_log, G, rtol=0, atol=1e-12)
        # Kernel(j, i) = k(x_j, x_i) = oracle K[i, j]; KernelGrad(j d + k, i) = Kg[i, j, k]
        np.testing.assert_allclose(K_log, K.T, rtol=0, atol=1e-12)
        np.testing.assert_allclose(Kg_log, np.transpose(Kg, (1, 2, 0)).reshape(n * d, n), rtol=0, atol=1e-12)
        X = X_new
    return X, steps


def test_cpp_generic_kernel_host_path_log_and_golden(oracle, golden_dir, tmp_path):
    """SURVEY 8(f) 4 + 3 on the host path (no GPU): the reference's own
    fixed-kernel scenario (test_svgd.cpp:66-203) with a closed-form generic
    kernel reproduces the pinned golden trajectory, and every logged
    LogModelGrad / Kernel / KernelGrad matches the oracle's materialised
    matrices at the logged X_t (<= 1e-12)."""
    _make_cpp()
    X, steps = _check_log(oracle, "host", tmp_path, _cosine_grad, lambda X: 1.0)
    assert len(steps) == 15
    with open(os.path.join(golden_dir, "test_svgd_n10.json")) as f:
        g = json.load(f)
    np.testing.assert_allclose(X, np.array(g["final"]), rtol=0, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["const", "median"])
def test_cpp_device_log_matches_oracle(oracle, tmp_path, which):
    """SURVEY 8(f) 3 on the device path: the logged matrices of a constant
    (M = I) and a median-scaled RBF run match the oracle at the logged X_t."""
    _make_cpp()
    if which == "const":
        _check_log(oracle, which, tmp_path, _cosine_grad, lambda X: 1.0)
    else:
        mu = np.array([-0.6871, 0.8010])
        cov = 5.0 * np.array([[0.2260, 0.1652], [0.1652, 0.6779]])
        _check_log(oracle, which, tmp_path, lambda X: oracle.logp_grad_gmm(X, mu[None], cov[None]),
                   lambda X: oracle.median_scale(X)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", ["1", "0"])
def test_cpp_sharded_run_matches_one_rank(tmp_path, pipelined):
    """SVGDOptions World / Rank (C++ API, SVGD.hpp:27-52 + the extension):
    two ranks of tests/cpp/test_dist.cpp on one GPU (host shared-memory
    collectives, SVGD_HOSTCOMM; every step's collective sequence compared
    across ranks) against the same program on one rank.  pipelined = 1: a
    built-in Gaussian model (the one-call svgd_step_host_model step); 0: a
    user subclass (the split begin / LogModelGradBatch of the rank's rows /
    finish).  Both ranks end with the same matrix; it matches one rank's to
    fp64 rounding of phi's column splits (<= 1e-10)."""
    import uuid

    _make_cpp()
    exe = os.path.join(BUILD, "test_dist")
    n, d, steps = 9001, 4, 8
    env = dict(os.environ, SVGD_HOSTCOMM="svgd_cpp_" + uuid.uuid4().hex[:10], SVGD_DEBUG_COLL="1")
    outs = [str(tmp_path / f"r{r}.bin") for r in range(2)]
    procs = [subprocess.Popen([exe, "2", str(r), str(n), str(d), str(steps), outs[r], pipelined], env=env,
                              cwd=BUILD, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    try:
        logs = [p.communicate(timeout=300)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), logs
    one = str(tmp_path / "one.bin")
    r = _run([exe, "1", "0", str(n), str(d), str(steps), one, pipelined])
    assert r.returncode == 0, r.stdout + r.stderr
    X = [np.fromfile(f, dtype=np.float64).reshape(n, d) for f in outs + [one]]
    assert np.all(np.isfinite(X[2]))
    assert np.array_equal(X[0], X[1])
    assert np.max(np.abs(X[0] - X[2])) <= 1e-10
