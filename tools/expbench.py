"""bench.py on the experiment build of the library (build/exp/libcassbloom.so,
`make -C lsmt_amd/csrc EXTRA=-DCB_EXPERIMENTS BUILD=../../build/exp/obj
OUT=../../build/exp/libcassbloom.so`): the A/B knobs (CB_BUILD_*, CB_PROBE_*,
CB_SET_*, CB_BIN_T) are compiled only there. Usage: python tools/expbench.py
[bench.py args]; set the knobs in the environment."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lsmt_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "build", "exp", "libcassbloom.so")
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
