"""The C-ABI library loads on a CPU-only host and exports every symbol the
public header declares. No compute calls are made here."""
import ctypes
import subprocess

import numpy as np

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


def _zone_encode(L, lo, hi):
    from lsmt_amd import _lib
    lb = ctypes.create_string_buffer(lo or b"", max(len(lo or b""), 1))
    hb = ctypes.create_string_buffer(hi or b"", max(len(hi or b""), 1))
    zb = _lib.ZoneBounds(ctypes.cast(lb, ctypes.c_void_p), len(lo or b""), lo is not None,
                         ctypes.cast(hb, ctypes.c_void_p), len(hi or b""), hi is not None)
    n = ctypes.c_uint64()
    rc = L.cb_meta_encode(None, ctypes.byref(zb), None, 0, ctypes.byref(n))
    if rc:
        return rc, None
    out = ctypes.create_string_buffer(max(n.value, 1))
    rc = L.cb_meta_encode(None, ctypes.byref(zb), out, n.value, ctypes.byref(n))
    return rc, out.raw[: n.value]


def test_meta_zone_only_encode_matches_oracle():
    # host-only framing of TableMeta{zone_map} (no filter: no device work)
    from lsmt_amd import _lib
    from oracle import oracle
    L = _lib.load()
    for lo, hi in [(b"k", b"k"), (None, None), (b"", None), (None, b"z"), ("é".encode(), "✓".encode()),
                   (b"a" * 200, b"b" * 300)]:
        rc, got = _zone_encode(L, lo, hi)
        assert rc == 0
        assert got == oracle.meta_encode(None, oracle.OracleZone(lo, hi)), (lo, hi)


def test_meta_encode_rejects_non_utf8_like_rust_strings():
    from lsmt_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(9)
    samples = [b"\xff", b"\xc0\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe2\x9c", "ok✓".encode()]
    samples += [rng.integers(0x70, 0x100, rng.integers(1, 6), dtype=np.uint8).tobytes() for _ in range(500)]
    for s in samples:
        try:
            s.decode("utf-8")
            ok = True
        except UnicodeDecodeError:
            ok = False
        rc, _ = _zone_encode(L, s, b"z")
        assert (rc == 0) == ok, s


def test_table_handle_array_is_reused_only_for_the_same_open_tables():
    # get_many's C array of table handles (lsmt_amd.bloom._table_array) is
    # kept per sequence while it names the same handle objects; a closed table
    # (Table.close() replaces its handle object), a replaced or reordered
    # table, or another sequence gets a fresh array with the current handles
    from lsmt_amd import bloom

    class T:
        def __init__(self, v):
            self._h = ctypes.c_void_p(v)

    ts = [T(0x1000 + 64 * i) for i in range(300)]
    a = bloom._table_array(ts)
    assert bloom._table_array(ts) is a
    assert [a[i] for i in range(300)] == [0x1000 + 64 * i for i in range(300)]
    ts[7]._h = ctypes.c_void_p()  # closed
    b = bloom._table_array(ts)
    assert b is not a and b[7] is None
    ts[3], ts[4] = ts[4], ts[3]
    c = bloom._table_array(ts)
    assert c is not b and (c[3], c[4]) == (0x1000 + 64 * 4, 0x1000 + 64 * 3)
    rev = ts[::-1]
    d = bloom._table_array(rev)
    assert d[0] == 0x1000 + 64 * 299 and bloom._table_array(ts) is c
    assert len(bloom._table_array([])) == 1  # the C ABI never reads it (nt = 0)
