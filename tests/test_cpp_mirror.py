"""The C++ host mirror (lsmt_amd/csrc/bloom_filter.hpp) and a plain-C client
of include/cassbloom.h, both linked against libcassbloom.so."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "tests")


def _ensure_built():
    if not (os.path.exists(os.path.join(BIN, "test_bloom_filter")) and
            os.path.exists(os.path.join(BIN, "test_capi_c"))):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)


def test_c_client_links_and_runs_without_gpu():
    _ensure_built()
    r = subprocess.run([os.path.join(BIN, "test_capi_c")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "gfx950" in r.stdout


@pytest.mark.gpu
def test_cpp_mirror_on_gpu(gpu):
    _ensure_built()
    r = subprocess.run([os.path.join(BIN, "test_bloom_filter")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([os.path.join(BIN, "test_capi_c"), "--gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c abi gpu ok" in r.stdout
