"""C2's golden check on the experiment library under the current knob
settings (e.g. CB_BUILD_SUB=1): 2^20 keys into m = 2^27, the packed bits'
SHA-256 against tests/golden/golden.json, on the tiled path. Prints one JSON
line. Usage: CB_BUILD_SUB=1 python tools/exp_c2_check.py"""
import hashlib
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("lsmt_amd._lib", os.path.join(ROOT, "lsmt_amd", "_lib.py"))
_lib = importlib.util.module_from_spec(spec)
sys.modules["lsmt_amd._lib"] = _lib
spec.loader.exec_module(_lib)
_lib.LIB_PATH = os.path.join(ROOT, "build", "exp", "libcassbloom.so")
_lib.load()


def main():
    import numpy as np

    import lsmt_amd
    from lsmt_amd import workload
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as fh:
        g = json.load(fh)["c2"]
    lsmt_amd.set_path(2)
    f = lsmt_amd.BloomFilter(g["m"])
    f.insert_batch(workload.c2_build_keys(g["n"]))
    got = hashlib.sha256(np.ascontiguousarray(f.packed().view(np.uint8)).tobytes()).hexdigest()
    ok = got == g["packed_sha256"]
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("CB_")}, "c2_golden": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
