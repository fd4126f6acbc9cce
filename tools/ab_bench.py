"""A/B of two builds of the library on one box: runs bench.py with
svgdcpp_amd._capi.LIB_PATH pointed at the given .so (argv[1]), passing the
rest of argv to bench.py.  Used for same-box comparisons (box-to-box spread
of the phi kernel is ~10 %)."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svgdcpp_amd._capi as C  # noqa: E402

C.LIB_PATH = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
