"""SVGDCpp-compatible C++ API (include/Core, Model, Kernel, Optimizer).

Builds the C++ example programs and tests/cpp/test_api.cpp against
libsvgdcpp_amd.so (``make cpp``) and runs them: the host-only checks on CPU,
the SVGD-class-vs-manual-loop checks (reference tests/test_svgd.cpp) on GPU.
"""
import os
import subprocess

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


@pytest.mark.gpu
def test_cpp_examples_run():
    _make_cpp()
    r = _run([os.path.join(BUILD, "mvn_example")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Final particle coordinates" in r.stdout
    r = _run([os.path.join(BUILD, "gmm_example"), "4096", "50"])
    assert r.returncode == 0, r.stdout + r.stderr
    near = int(r.stdout.split("Particles nearer component A: ")[1].split()[0])
    # both mixture components are populated
    assert 0.2 * 4096 < near < 0.8 * 4096, r.stdout
