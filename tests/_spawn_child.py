"""Child of tests/test_bench_spawn.py: a stand-in rank of bench.py --gpus N.
FAIL_RANK exits 3 at once; the others sleep SLEEP seconds (a rank blocked in
a collective), then exit 0."""
import os
import sys
import time

if int(os.environ["RANK"]) == int(os.environ.get("FAIL_RANK", "-1")):
    sys.exit(3)
time.sleep(float(os.environ.get("SLEEP", "60")))
