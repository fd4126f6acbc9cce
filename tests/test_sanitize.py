"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

`make sanitize` builds the planner (plan.cpp), the host Gaussian-sum models
(host_models.cpp) and the CPU oracle with -fsanitize=address,undefined into a
self-checking driver (tests/cpp/sanitize_host.cpp) and runs it; any sanitizer
report aborts the driver (-fno-sanitize-recover=all).  The HIP host code is
exercised by the -m gpu tests (no GPU sanitizers on this pool).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_code_under_asan_ubsan():
    r = subprocess.run(["make", "-C", ROOT, "sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all checks passed" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
