"""The C-ABI library loads on a CPU-only host and exports every symbol the
public header declares. No compute calls are made here."""
import ctypes
import subprocess

from lsmt_amd import _lib


def test_library_loads_and_exports_header_symbols():
    L = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/cassbloom.h but not exported"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported


def test_library_is_gfx950_code_object():
    # the fat binary embeds the offload bundle id of its only target
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_version_and_path_knob():
    L = _lib.load()
    assert b"gfx950" in L.cb_version()
    assert L.cb_set_path(3) == _lib.CB_EINVAL
    assert L.cb_set_path(0) == _lib.CB_OK


def test_null_argument_errors_without_gpu():
    L = _lib.load()
    assert L.cb_filter_bits(None, None) == _lib.CB_EINVAL
    assert L.cb_filter_destroy(None) == _lib.CB_OK
    assert L.cb_filter_insert_fixed(None, None, 16, 1, None) == _lib.CB_EINVAL
    assert b"null" in L.cb_last_error()
    n = ctypes.c_uint64()
    assert L.cb_filter_to_bytes(None, None, 0, ctypes.byref(n)) == _lib.CB_EINVAL
