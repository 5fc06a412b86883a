"""ctypes wrapper over the C oracle (oracle/bloom_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the parity checker / CPU baseline. The product
path (lsmt_amd) never imports this module.

Restates /root/reference/src/bloom.rs:17-77 (see bloom_oracle.h for the
line-by-line mapping).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

OB_OK = 0
OB_EINVAL = -1
OB_EZEROM = -2
OB_ENOMEM = -3
OB_EDECODE = -5


class _Filter(ctypes.Structure):
    _fields_ = [("bits", ctypes.POINTER(ctypes.c_uint8)), ("m", ctypes.c_uint64)]


class _Zone(ctypes.Structure):
    _fields_ = [("min", ctypes.POINTER(ctypes.c_uint8)), ("min_len", ctypes.c_uint64), ("has_min", ctypes.c_int),
                ("max", ctypes.POINTER(ctypes.c_uint8)), ("max_len", ctypes.c_uint64), ("has_max", ctypes.c_int)]


class _Meta(ctypes.Structure):
    _fields_ = [("has_bloom", ctypes.c_int), ("bloom", _Filter), ("has_zone", ctypes.c_int), ("zone", _Zone)]


class _Table(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("nlines", ctypes.c_uint64),
                ("start", ctypes.POINTER(ctypes.c_uint64)), ("end", ctypes.POINTER(ctypes.c_uint64))]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        FP = ctypes.POINTER(_Filter)
        L.ob_new.argtypes = [FP, u64]
        L.ob_free.argtypes = [FP]
        L.ob_free.restype = None
        L.ob_raw_hashes.argtypes = [P, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.ob_raw_hashes.restype = None
        L.ob_hashes.argtypes = [P, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.ob_insert.argtypes = [FP, P, u64]
        L.ob_may_contain.argtypes = [FP, P, u64]
        L.ob_insert_fixed.argtypes = [FP, P, u32, u64]
        L.ob_insert_var.argtypes = [FP, P, P, u64]
        L.ob_probe_fixed.argtypes = [P, u32, P, u32, u64, P, i32]
        L.ob_probe_var.argtypes = [P, u32, P, P, u64, P, i32]
        L.ob_encode.argtypes = [FP, P, u64]
        L.ob_encode.restype = u64
        L.ob_decode.argtypes = [P, u64, FP]
        ZP = ctypes.POINTER(_Zone)
        L.ob_zone_init.argtypes = [ZP]
        L.ob_zone_init.restype = None
        L.ob_zone_free.argtypes = [ZP]
        L.ob_zone_free.restype = None
        L.ob_zone_set.argtypes = [ZP, P, u64, i32, P, u64, i32]
        L.ob_zone_update.argtypes = [ZP, P, u64]
        L.ob_zone_contains.argtypes = [ZP, P, u64]
        L.ob_probe_gated_var.argtypes = [P, P, u32, P, P, u64, P]
        MP = ctypes.POINTER(_Meta)
        L.ob_meta_encode.argtypes = [FP, ZP, P, u64]
        L.ob_meta_encode.restype = u64
        L.ob_meta_decode.argtypes = [P, u64, MP]
        L.ob_meta_free.argtypes = [MP]
        L.ob_meta_free.restype = None
        L.ob_utf8_valid.argtypes = [P, u64]
        TP = ctypes.POINTER(_Table)
        L.ob_table_index.argtypes = [P, u64, TP]
        L.ob_table_free.argtypes = [TP]
        L.ob_table_free.restype = None
        L.ob_table_search.argtypes = [TP, P, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.ob_table_search.restype = ctypes.c_int64
        L.ob_b64_decode.argtypes = [P, u64, P]
        L.ob_b64_decode.restype = ctypes.c_int64
        L.ob_b64_encode.argtypes = [P, u64, P]
        L.ob_b64_encode.restype = u64
        L.ob_get_many.argtypes = [P, u32, P, P, P, u64, P, P, P, u64, ctypes.POINTER(u64)]
        L.ob_table_rebuild.argtypes = [TP, u64, FP, ZP, ctypes.POINTER(u64)]
        L.ob_sstable_create.argtypes = [P, P, P, P, u64, P, u64]
        L.ob_sstable_create.restype = u64
        L.ob_gen_keys.argtypes = [u64, u64, u64, P]
        L.ob_gen_keys.restype = None
        L.ob_splitmix64.argtypes = [u64]
        L.ob_splitmix64.restype = u64
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleFilter:
    """Byte-per-bit Bloom filter — the reference's `BloomFilter` on the CPU."""

    def __init__(self, m: int, _raw: _Filter | None = None):
        self._f = _Filter()
        if _raw is not None:
            self._f = _raw
        else:
            rc = lib().ob_new(ctypes.byref(self._f), m)
            if rc:
                raise MemoryError(rc)

    def __del__(self):
        try:
            lib().ob_free(ctypes.byref(self._f))
        except Exception:
            pass

    @property
    def m(self) -> int:
        return int(self._f.m)

    def bools(self) -> np.ndarray:
        """The Vec<bool> array (m bytes of 0/1), copied."""
        if self.m == 0:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array(self._f.bits, shape=(self.m,)).copy()

    def insert(self, key: bytes) -> None:
        buf = ctypes.create_string_buffer(key, len(key))
        rc = lib().ob_insert(ctypes.byref(self._f), buf, len(key))
        if rc == OB_EZEROM:
            raise ZeroDivisionError("attempt to calculate the remainder with a divisor of zero")

    def may_contain(self, key: bytes) -> bool:
        buf = ctypes.create_string_buffer(key, len(key))
        rc = lib().ob_may_contain(ctypes.byref(self._f), buf, len(key))
        if rc == OB_EZEROM:
            raise ZeroDivisionError("attempt to calculate the remainder with a divisor of zero")
        return bool(rc)

    def insert_fixed(self, keys: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        n, kl = keys.shape
        rc = lib().ob_insert_fixed(ctypes.byref(self._f), _ptr(keys), kl, n)
        if rc:
            raise RuntimeError(f"ob_insert_fixed rc={rc}")

    def insert_var(self, data: np.ndarray, offsets: np.ndarray) -> None:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        rc = lib().ob_insert_var(ctypes.byref(self._f), _ptr(data), _ptr(offsets), len(offsets) - 1)
        if rc:
            raise RuntimeError(f"ob_insert_var rc={rc}")

    def to_bytes(self) -> bytes:
        L = lib()
        n = L.ob_encode(ctypes.byref(self._f), None, 0)
        out = np.zeros(max(n, 1), np.uint8)
        L.ob_encode(ctypes.byref(self._f), _ptr(out), n)
        return out[:n].tobytes()

    @classmethod
    def from_bytes(cls, data: bytes) -> "OracleFilter":
        raw = _Filter()
        buf = np.frombuffer(data, np.uint8).copy() if data else np.zeros(1, np.uint8)
        rc = lib().ob_decode(_ptr(buf), len(data), ctypes.byref(raw))
        if rc:
            raise ValueError(f"decode error rc={rc}")
        return cls(0, _raw=raw)


def raw_hashes(key: bytes) -> tuple[int, int]:
    h1, h2 = ctypes.c_uint64(), ctypes.c_uint64()
    buf = ctypes.create_string_buffer(key, len(key))
    lib().ob_raw_hashes(buf, len(key), ctypes.byref(h1), ctypes.byref(h2))
    return h1.value, h2.value


def probe_fixed(filters, keys: np.ndarray, threads: int = 1) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, kl = keys.shape
    nf = len(filters)
    words = (n + 63) // 64
    hits = np.zeros((nf, words), np.uint64)
    arr = (ctypes.POINTER(_Filter) * max(nf, 1))(*[ctypes.pointer(f._f) for f in filters])
    rc = lib().ob_probe_fixed(ctypes.cast(arr, ctypes.c_void_p), nf, _ptr(keys), kl, n, _ptr(hits), threads)
    if rc:
        raise RuntimeError(f"ob_probe_fixed rc={rc}")
    return hits


def probe_var(filters, data: np.ndarray, offsets: np.ndarray, threads: int = 1) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    nf = len(filters)
    hits = np.zeros((nf, (n + 63) // 64), np.uint64)
    arr = (ctypes.POINTER(_Filter) * max(nf, 1))(*[ctypes.pointer(f._f) for f in filters])
    rc = lib().ob_probe_var(ctypes.cast(arr, ctypes.c_void_p), nf, _ptr(data if len(data) else np.zeros(1, np.uint8)),
                            _ptr(offsets), n, _ptr(hits), threads)
    if rc:
        raise RuntimeError(f"ob_probe_var rc={rc}")
    return hits


class OracleZone:
    """ZoneMap (src/zonemap.rs) on the CPU."""

    def __init__(self, lo: bytes | None = None, hi: bytes | None = None):
        self._z = _Zone()
        lib().ob_zone_init(ctypes.byref(self._z))
        if lo is not None or hi is not None:
            lb = ctypes.create_string_buffer(lo or b"", max(len(lo or b""), 1))
            hb = ctypes.create_string_buffer(hi or b"", max(len(hi or b""), 1))
            lib().ob_zone_set(ctypes.byref(self._z), lb, len(lo or b""), lo is not None, hb, len(hi or b""),
                              hi is not None)

    def __del__(self):
        try:
            lib().ob_zone_free(ctypes.byref(self._z))
        except Exception:
            pass

    def update(self, key: bytes) -> None:
        buf = ctypes.create_string_buffer(key, max(len(key), 1))
        lib().ob_zone_update(ctypes.byref(self._z), buf, len(key))

    def contains(self, key: bytes) -> bool:
        buf = ctypes.create_string_buffer(key, max(len(key), 1))
        return bool(lib().ob_zone_contains(ctypes.byref(self._z), buf, len(key)))

    @property
    def bounds(self):
        z = self._z
        lo = bytes(z.min[: z.min_len]) if z.has_min else None
        hi = bytes(z.max[: z.max_len]) if z.has_max else None
        return lo, hi


def probe_gated(filters, zones, data: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """SsTable::get's gate for every (key, table): zone.contains && may_contain."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    nf = len(filters)
    hits = np.zeros((nf, (n + 63) // 64), np.uint64)
    fa = (ctypes.POINTER(_Filter) * max(nf, 1))(*[ctypes.pointer(f._f) for f in filters])
    za = (ctypes.POINTER(_Zone) * max(nf, 1))(*[ctypes.pointer(z._z) if z is not None else None for z in zones])
    rc = lib().ob_probe_gated_var(ctypes.cast(fa, ctypes.c_void_p), ctypes.cast(za, ctypes.c_void_p), nf,
                                  _ptr(data if len(data) else np.zeros(1, np.uint8)), _ptr(offsets), n, _ptr(hits))
    if rc:
        raise RuntimeError(f"ob_probe_gated_var rc={rc}")
    return hits


def meta_encode(bloom: "OracleFilter | None", zone: "OracleZone | None") -> bytes:
    """TableMeta{bloom, zone_map}.encode (src/sstable.rs:74-81)."""
    L = lib()
    fp = ctypes.byref(bloom._f) if bloom is not None else None
    zp = ctypes.byref(zone._z) if zone is not None else None
    n = L.ob_meta_encode(fp, zp, None, 0)
    out = np.zeros(max(n, 1), np.uint8)
    L.ob_meta_encode(fp, zp, _ptr(out), n)
    return out[:n].tobytes()


def meta_decode(data: bytes):
    """TableMeta::decode (src/sstable.rs:97). Returns (bloom bools | None,
    (min, max) | None); raises ValueError on a decode error."""
    m = _Meta()
    buf = np.frombuffer(data, np.uint8).copy() if data else np.zeros(1, np.uint8)
    rc = lib().ob_meta_decode(_ptr(buf), len(data), ctypes.byref(m))
    if rc:
        raise ValueError(f"TableMeta decode error rc={rc}")
    try:
        bloom = None
        if m.has_bloom:
            bloom = (np.ctypeslib.as_array(m.bloom.bits, shape=(m.bloom.m,)).copy() if m.bloom.m
                     else np.zeros(0, np.uint8))
        zone = None
        if m.has_zone:
            z = m.zone
            zone = (bytes(z.min[: z.min_len]) if z.has_min else None,
                    bytes(z.max[: z.max_len]) if z.has_max else None)
        return bloom, zone
    finally:
        lib().ob_meta_free(ctypes.byref(m))


def utf8_valid(b: bytes) -> bool:
    buf = np.frombuffer(b, np.uint8).copy() if b else np.zeros(1, np.uint8)
    return bool(lib().ob_utf8_valid(_ptr(buf), len(b)))


def _buf(b: bytes) -> np.ndarray:
    return np.frombuffer(b, np.uint8).copy() if b else np.zeros(1, np.uint8)


class OracleTable:
    """An SSTable data file split into lines as SsTable::get does (src/sstable.rs:142-146)."""

    def __init__(self, data):
        self.data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray)
                                         else data, dtype=np.uint8)
        self._keep = self.data if len(self.data) else np.zeros(1, np.uint8)
        self._t = _Table()
        rc = lib().ob_table_index(_ptr(self._keep), len(self.data), ctypes.byref(self._t))
        if rc:
            raise MemoryError(rc)

    def __del__(self):
        try:
            lib().ob_table_free(ctypes.byref(self._t))
        except Exception:
            pass

    @property
    def nlines(self) -> int:
        return int(self._t.nlines)

    def rebuild(self, m: int = 1024):
        """SsTable::load's rebuild (src/sstable.rs:109-120): (OracleFilter,
        OracleZone) from the lines' keys, or raises UnicodeDecodeError-like
        ValueError(bad line) when a key is not UTF-8."""
        raw = _Filter()
        z = OracleZone()
        lib().ob_zone_free(ctypes.byref(z._z))
        bad = ctypes.c_uint64()
        rc = lib().ob_table_rebuild(ctypes.byref(self._t), m, ctypes.byref(raw), ctypes.byref(z._z),
                                    ctypes.byref(bad))
        f = OracleFilter(m, _raw=raw)
        if rc == -7:
            raise ValueError(f"key on line {bad.value} is not UTF-8")
        if rc:
            raise RuntimeError(rc)
        return f, z

    def search(self, key: bytes):
        """SsTable::binary_search: (line index, encoded value bytes) or (-1, None)."""
        vs, vl = ctypes.c_uint64(), ctypes.c_uint64()
        kb = _buf(key)
        r = lib().ob_table_search(ctypes.byref(self._t), _ptr(kb), len(key), ctypes.byref(vs), ctypes.byref(vl))
        if r < 0:
            return -1, None
        return int(r), self.data[vs.value: vs.value + vl.value].tobytes()


def b64_decode(data: bytes) -> bytes | None:
    b = _buf(data)
    out = np.zeros(max(len(data), 1), np.uint8)
    r = lib().ob_b64_decode(_ptr(b), len(data), _ptr(out))
    return None if r < 0 else out[:r].tobytes()


def b64_encode(data: bytes) -> bytes:
    b = _buf(data)
    out = np.zeros(max(4 * ((len(data) + 2) // 3), 1), np.uint8)
    r = lib().ob_b64_encode(_ptr(b), len(data), _ptr(out))
    return out[:r].tobytes()


def get_many(tables, hits, data: np.ndarray, offsets: np.ndarray):
    """Database::get's newest-first walk (tables[0] newest) for a key batch.
    Returns (which int32[n], val_off uint64[n+1], vals bytes)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    nt = len(tables)
    which = np.zeros(max(n, 1), np.int32)
    voff = np.zeros(n + 1, np.uint64)
    tarr = (ctypes.POINTER(_Table) * max(nt, 1))(*[ctypes.pointer(t._t) for t in tables])
    hp = None
    if hits is not None:
        hits = np.ascontiguousarray(hits, dtype=np.uint64)
        hp = _ptr(hits)
    total = ctypes.c_uint64()
    L = lib()
    args = [ctypes.cast(tarr, ctypes.c_void_p), nt, hp, _ptr(data if len(data) else np.zeros(1, np.uint8)),
            _ptr(offsets), n, _ptr(which), _ptr(voff)]
    rc = L.ob_get_many(*args, None, 0, ctypes.byref(total))
    if rc:
        raise RuntimeError(rc)
    vals = np.zeros(max(total.value, 1), np.uint8)
    rc = L.ob_get_many(*args, _ptr(vals), total.value, ctypes.byref(total))
    if rc:
        raise RuntimeError(rc)
    return which[:n], voff, vals[: total.value].tobytes()


def _ragged(items):
    offs = np.zeros(len(items) + 1, np.uint64)
    np.cumsum([len(x) for x in items], out=offs[1:])
    data = np.frombuffer(b"".join(items), np.uint8).copy() if offs[-1] else np.zeros(1, np.uint8)
    return data, offs


def sstable_create(entries) -> bytes:
    """SsTable::create's data file for [(key bytes, value bytes)]."""
    kd, ko = _ragged([k for k, _ in entries])
    vd, vo = _ragged([v for _, v in entries])
    L = lib()
    n = len(entries)
    total = L.ob_sstable_create(_ptr(kd), _ptr(ko), _ptr(vd), _ptr(vo), n, None, 0)
    out = np.zeros(max(total, 1), np.uint8)
    L.ob_sstable_create(_ptr(kd), _ptr(ko), _ptr(vd), _ptr(vo), n, _ptr(out), total)
    return out[:total].tobytes()


def gen_keys(seed: int, n: int, first: int = 0) -> np.ndarray:
    out = np.empty((n, 16), np.uint8)
    if n:
        lib().ob_gen_keys(seed, first, n, _ptr(out))
    return out
