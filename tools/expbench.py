"""bench.py on the experiment build of the library (build/exp/libcassbloom.so,
`make -C lsmt_amd/csrc EXTRA=-DCB_EXPERIMENTS BUILD=../../build/exp/obj
OUT=../../build/exp/libcassbloom.so`): the A/B knobs (CB_BUILD_*, CB_PROBE_*,
CB_SET_*, CB_BIN_T, CB_ORDER_FENCE) are compiled only there. Usage: python
tools/expbench.py [bench.py args]; set the knobs in the environment.

The loader module is installed under its package name before the package is
imported: lsmt_amd/__init__.py loads the library at import, so setting
LIB_PATH after `import lsmt_amd` would leave the product library loaded (as
every round-4 sweep before this fix did: their knob settings never applied)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
EXP = os.environ.get("EXPBENCH_LIB") or os.path.join(ROOT, "build", "exp", "libcassbloom.so")  # another build to A/B

spec = importlib.util.spec_from_file_location("lsmt_amd._lib", os.path.join(ROOT, "lsmt_amd", "_lib.py"))
_lib = importlib.util.module_from_spec(spec)
sys.modules["lsmt_amd._lib"] = _lib
spec.loader.exec_module(_lib)
_lib.LIB_PATH = EXP
L = _lib.load()
import lsmt_amd  # noqa: E402,F401  (binds the already-loaded experiment library)

assert lsmt_amd._lib is _lib and _lib.load()._name == EXP, "experiment library not the one loaded"
print(f"expbench: {EXP}", file=sys.stderr, flush=True)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
