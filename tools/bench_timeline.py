"""bench.py under the diagnosis build, then the device timeline of its last windows (block log of
every pipeline kernel, diaglog.hpp).

THETARRT_LIB=theta-rrt_amd/libthetarrt_phases.so python tools/bench_timeline.py [last_us] [bench args]
"""
import ctypes as C
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import phases  # noqa: E402

last_us = float(sys.argv[1]) if len(sys.argv) > 1 else 2500.0
sys.argv = [os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-pmc", "--no-events"] + sys.argv[2:]
try:
    runpy.run_path(sys.argv[0], run_name="__main__")
except SystemExit:
    pass
from theta_rrt_amd import _native  # noqa: E402
phases.print_timeline(C.CDLL(_native.LIB_PATH), last_us)
