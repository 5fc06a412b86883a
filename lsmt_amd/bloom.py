"""Host-side mirror of the reference's ``BloomFilter`` over the gfx950 C ABI.

Same surface as /root/reference/src/bloom.rs so the reference's callers and
tests read the same:

    BloomFilter.new(size)          src/bloom.rs:17-21
    f.insert(item)                 src/bloom.rs:40-44
    f.may_contain(item) -> bool    src/bloom.rs:48-51
    f.to_proto() / from_proto(p)   src/bloom.rs:54-63
    f.to_bytes() / from_bytes(b)   src/bloom.rs:66-77

The filter bits live in HBM. Per-key ``insert`` calls are queued on the host
and flushed as ONE batched build launch before the filter is next read: this
is how SsTable::create's per-key loop (src/sstable.rs:62-65) turns into a
single GPU build without changing the caller. ``may_contain`` on one key is a
synchronous single-key probe; the read-path fan-out over many tables
(src/lib.rs:129-134) uses the batched :func:`probe`.

Errors follow the reference's panics: inserting into or probing an m == 0
filter raises ZeroDivisionError (``h % 0``, src/bloom.rs:36); malformed proto
bytes raise ValueError (``decode(..).unwrap()``, src/bloom.rs:75).

There is no CPU fallback: every operation goes through libcassbloom.so.
"""
from __future__ import annotations

import ctypes
import operator
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import CassBloomError, check

__all__ = ["BloomFilter", "BloomProto", "FilterSet", "probe", "insert_many", "set_path",
           "last_path", "device_count", "DeviceKeys", "KeyBatch", "ZoneMap", "zone_bounds", "TableMeta", "Table", "get_many", "sstable_create"]


def _L():
    return _lib.load()


def _raise(rc: int) -> None:
    if rc == _lib.CB_EZEROM:
        raise ZeroDivisionError("attempt to calculate the remainder with a divisor of zero")
    if rc == _lib.CB_EDECODE:
        msg = _L().cb_last_error()
        raise ValueError(msg.decode() if msg else "BloomProto decode error")
    check(rc)


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = _L().cb_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_path(path: int) -> None:
    """0 auto, 1 direct (per-key atomics/gathers), 2 tiled (LDS tiles)."""
    check(_L().cb_set_path(path))


def last_path() -> int:
    return int(_L().cb_last_path())


def set_dense(mode: int) -> None:
    """FilterSet probes of dense batches: 0 by density (default), 1 the
    region-partitioned probe whenever the set allows it, -1 never
    (cb_set_dense; last_path() is 6 after a dense probe)."""
    check(_L().cb_set_dense(int(mode)))


# ---- key batches ---------------------------------------------------------------

def _ptr_of(x):
    """(address, keepalive) for numpy arrays, torch tensors, or raw ints."""
    if x is None:
        return None, None
    if isinstance(x, int):
        return x, None
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            x = np.ascontiguousarray(x)
        return x.ctypes.data, x
    if hasattr(x, "data_ptr"):  # torch tensor (device or host)
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return x.data_ptr(), x
    raise TypeError(f"unsupported buffer type {type(x)!r}")


@dataclass
class KeyBatch:
    """A batch of keys as the C ABI takes them: fixed-length rows
    (``keys``: uint8[n, key_len]) or ragged (``data`` + ``offsets[n+1]``).
    Buffers may be numpy (host) or device tensors."""
    n: int
    key_len: int = 0
    keys: object = None
    data: object = None
    offsets: object = None

    @property
    def is_var(self) -> bool:
        return self.offsets is not None


def DeviceKeys(tensor) -> KeyBatch:
    """Fixed-length keys already resident in HBM (torch uint8 [n, key_len])."""
    n, kl = tensor.shape
    return KeyBatch(n=int(n), key_len=int(kl), keys=tensor)


def as_batch(keys) -> KeyBatch:
    if isinstance(keys, KeyBatch):
        return keys
    if isinstance(keys, np.ndarray):
        if keys.dtype != np.uint8 or keys.ndim != 2:
            raise TypeError("fixed-length keys must be a uint8 array of shape [n, key_len]")
        return KeyBatch(n=keys.shape[0], key_len=keys.shape[1], keys=np.ascontiguousarray(keys))
    if hasattr(keys, "data_ptr") and getattr(keys, "ndim", 0) == 2:
        return DeviceKeys(keys)
    items = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    offs = np.zeros(len(items) + 1, np.uint64)
    if items:
        np.cumsum([len(k) for k in items], out=offs[1:])
    data = np.frombuffer(b"".join(items), np.uint8) if offs[-1] else np.zeros(1, np.uint8)
    return KeyBatch(n=len(items), data=np.ascontiguousarray(data), offsets=offs)


def _stream(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)  # torch.cuda.Stream


# ---- proto mirror ----------------------------------------------------------------

@dataclass
class BloomProto:
    """Mirror of ``BloomProto { repeated bool bits = 1; }`` (src/bloom.rs:9-13)."""
    bits: np.ndarray = field(default_factory=lambda: np.zeros(0, bool))


@dataclass
class ZoneMap:
    """Mirror of ``ZoneMap { min, max: Option<String> }`` (src/zonemap.rs:3-8).

    Bounds are bytes, ordered as Rust orders ``str`` (byte-wise, a proper
    prefix first). This host object only carries a table's bounds; the
    per-key gate runs on the device (``FilterSet.probe(..., gated=True)``)."""
    min: bytes | None = None
    max: bytes | None = None

    def update(self, key) -> None:
        """zonemap.rs:21-32."""
        k = key.encode() if isinstance(key, str) else bytes(key)
        if self.min is None or k < self.min:
            self.min = k
        if self.max is None or k > self.max:
            self.max = k

    def contains(self, key) -> bool:
        """zonemap.rs:37-42: min <= key <= max, true if a bound is missing."""
        if self.min is None or self.max is None:
            return True
        k = key.encode() if isinstance(key, str) else bytes(key)
        return self.min <= k <= self.max


@dataclass
class TableMeta:
    """Mirror of ``TableMeta { bloom: Option<BloomProto>, zone_map:
    Option<ZoneMapProto> }`` (src/sstable.rs:31-37), the SSTable ``.meta``
    file. Encoding and decoding run through the C ABI; the filter's bits are
    expanded / packed on the device."""
    bloom: "BloomFilter | None" = None
    zone_map: ZoneMap | None = None

    def encode(self) -> bytes:
        """TableMeta.encode (SsTable::create, src/sstable.rs:74-81)."""
        zb, keep = _zone_struct(self.zone_map)
        fh = self.bloom.handle if self.bloom is not None else None
        if self.bloom is not None:
            self.bloom.flush()
        n = ctypes.c_uint64()
        zp = ctypes.byref(zb) if zb is not None else None
        _raise(_L().cb_meta_encode(fh, zp, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint8)
        _raise(_L().cb_meta_encode(fh, zp, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[: n.value].tobytes()

    @classmethod
    def decode(cls, data: bytes, device: int = 0) -> "TableMeta":
        """TableMeta::decode; raises ValueError (CB_EDECODE) on malformed bytes.
        A missing field decodes to None, as in the proto."""
        bloom, info, buf = _meta_decode(data, device)
        return cls(bloom if info.has_bloom else None, _zone_from_info(info, buf) if info.has_zone else None)

    @staticmethod
    def load(data: bytes, device: int = 0) -> "tuple[BloomFilter, ZoneMap]":
        """The metadata half of SsTable::load (src/sstable.rs:96-108): a missing
        bloom is BloomFilter::new(1024), a missing zone map ZoneMap::default()."""
        bloom, info, buf = _meta_decode(data, device)
        return bloom, (_zone_from_info(info, buf) if info.has_zone else ZoneMap())


def _zone_struct(z: "ZoneMap | None"):
    if z is None:
        return None, None
    lo = z.min.encode() if isinstance(z.min, str) else z.min
    hi = z.max.encode() if isinstance(z.max, str) else z.max
    lb = ctypes.create_string_buffer(lo or b"", max(len(lo or b""), 1))
    hb = ctypes.create_string_buffer(hi or b"", max(len(hi or b""), 1))
    zb = _lib.ZoneBounds(ctypes.cast(lb, ctypes.c_void_p), len(lo or b""), lo is not None,
                         ctypes.cast(hb, ctypes.c_void_p), len(hi or b""), hi is not None)
    return zb, (lb, hb)


def _meta_decode(data: bytes, device: int):
    buf = np.frombuffer(bytes(data), np.uint8).copy() if data else np.zeros(1, np.uint8)
    h = ctypes.c_void_p()
    info = _lib.MetaInfo()
    _raise(_L().cb_meta_decode(buf.ctypes.data, len(data), int(device), ctypes.byref(h), ctypes.byref(info)))
    return BloomFilter(0, device=device, _handle=h.value), info, buf


def _zone_from_info(info, buf: np.ndarray) -> ZoneMap:
    base = buf.ctypes.data
    z = info.zone

    def span(p, n, has):
        if not has:
            return None
        return buf[p - base: p - base + n].tobytes() if n else b""
    return ZoneMap(span(z.min or 0, z.min_len, z.has_min), span(z.max or 0, z.max_len, z.has_max))


def zone_bounds(keys, device: int = 0, stream=None) -> tuple[int, int] | None:
    """(index of first smallest key, index of first largest key), computed on
    the device; None for an empty batch."""
    b = as_batch(keys)
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    s = _stream(stream)
    if b.is_var:
        dp, k1 = _ptr_of(b.data)
        offp, k2 = _ptr_of(b.offsets)
        _raise(_L().cb_zone_bounds_var(dp, offp, b.n, int(device), ctypes.byref(lo), ctypes.byref(hi), s))
    else:
        kp, k1 = _ptr_of(b.keys)
        _raise(_L().cb_zone_bounds_fixed(kp, b.key_len, b.n, int(device), ctypes.byref(lo),
                                         ctypes.byref(hi), s))
    if b.n == 0:
        return None
    return int(lo.value), int(hi.value)


# ---- the filter --------------------------------------------------------------------

class BloomFilter:
    """A Bloom filter of ``size`` bits resident in HBM (src/bloom.rs:4-7)."""

    def __init__(self, size: int, device: int = 0, _handle: int | None = None):
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = ctypes.c_void_p(_handle)
        else:
            _raise(_L().cb_filter_create(int(size), int(device), ctypes.byref(self._h)))
        m = ctypes.c_uint64()
        check(_L().cb_filter_bits(self._h, ctypes.byref(m)))
        self._m = int(m.value)
        d = ctypes.c_int()
        check(_L().cb_filter_device(self._h, ctypes.byref(d)))
        self._device = int(d.value)
        self._pending: list[bytes] = []

    # src/bloom.rs:17-21
    @classmethod
    def new(cls, size: int, device: int = 0) -> "BloomFilter":
        return cls(size, device)

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _L().cb_filter_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def m(self) -> int:
        return self._m

    @property
    def device(self) -> int:
        return self._device

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def __len__(self) -> int:
        return self._m

    # ---- build -------------------------------------------------------------
    def insert(self, item) -> None:
        """src/bloom.rs:40-44. Queued; flushed as one batched launch."""
        if self._m == 0:
            raise ZeroDivisionError("attempt to calculate the remainder with a divisor of zero")
        self._pending.append(item.encode() if isinstance(item, str) else bytes(item))

    def flush(self, stream=None) -> None:
        if self._pending:
            batch, self._pending = self._pending, []
            self.insert_batch(batch, stream=stream)

    def insert_batch(self, keys, stream=None) -> None:
        """Batched insert of every key (the flush build, src/sstable.rs:62-65)."""
        b = as_batch(keys)
        if self._pending:
            pend, self._pending = self._pending, []
            self.insert_batch(pend, stream=stream)
        s = _stream(stream)
        if b.is_var:
            dp, k1 = _ptr_of(b.data)
            op, k2 = _ptr_of(b.offsets)
            _raise(_L().cb_filter_insert_var(self._h, dp, op, b.n, s))
        else:
            kp, k1 = _ptr_of(b.keys)
            _raise(_L().cb_filter_insert_fixed(self._h, kp, b.key_len, b.n, s))

    def clear(self, stream=None) -> None:
        self._pending = []
        check(_L().cb_filter_clear(self._h, _stream(stream)))

    # ---- probe -------------------------------------------------------------
    def may_contain(self, item) -> bool:
        """src/bloom.rs:48-51 for one key (synchronous; answered from the
        host mirror of the words when it is on, see host_mirror)."""
        self.flush()
        key = item.encode() if isinstance(item, str) else bytes(item)
        buf = ctypes.create_string_buffer(key, max(len(key), 1))
        out = ctypes.c_int(0)
        _raise(_L().cb_may_contain(self._h, ctypes.cast(buf, ctypes.c_void_p), len(key), ctypes.byref(out)))
        return bool(out.value)

    def host_mirror(self, mode: int = 1) -> None:
        """Single-key may_contain source (cb_filter_host_mirror): 1 the host
        mirror of the words (refreshed by one copy after each write), 0 a
        one-key GPU probe per call, -1 auto (mirror when m <= 2^24)."""
        check(_L().cb_filter_host_mirror(self._h, int(mode)))

    def host_mirror_info(self) -> tuple[bool, bool]:
        """(mirror on, mirror holds the latest write)."""
        on, cur = ctypes.c_int(), ctypes.c_int()
        check(_L().cb_filter_host_mirror_info(self._h, ctypes.byref(on), ctypes.byref(cur)))
        return bool(on.value), bool(cur.value)

    def may_contain_batch(self, keys, stream=None) -> np.ndarray:
        hits = probe([self], keys, stream=stream)
        n = as_batch(keys).n
        return unpack_hits(hits, n)[0]

    # ---- persistence -------------------------------------------------------
    def bools(self, stream=None) -> np.ndarray:
        """The Vec<bool> contents as uint8 0/1 (to_proto's bits)."""
        self.flush(stream)
        out = np.zeros(max(self._m, 1), np.uint8)
        _raise(_L().cb_filter_export_bools(self._h, out.ctypes.data, _stream(stream)))
        return out[: self._m]

    def packed(self, stream=None) -> np.ndarray:
        self.flush(stream)
        nw = (self._m + 31) // 32
        out = np.zeros(max(nw, 1), np.uint32)
        _raise(_L().cb_filter_export_packed(self._h, out.ctypes.data, _stream(stream)))
        return out[:nw]

    def load_packed(self, words: np.ndarray, stream=None) -> None:
        self._pending = []
        w = np.ascontiguousarray(words, dtype=np.uint32)
        _raise(_L().cb_filter_import_packed(self._h, w.ctypes.data if w.size else None, w.size, _stream(stream)))

    def to_proto(self) -> BloomProto:  # src/bloom.rs:54-58
        return BloomProto(bits=self.bools().astype(bool))

    @classmethod
    def from_proto(cls, proto: BloomProto, device: int = 0) -> "BloomFilter":  # src/bloom.rs:61-63
        bits = np.ascontiguousarray(np.asarray(proto.bits, dtype=bool).view(np.uint8))
        f = cls(bits.shape[0], device)
        if bits.shape[0]:
            _raise(_L().cb_filter_import_bools(f._h, bits.ctypes.data, bits.shape[0], None))
        return f

    def to_bytes(self) -> bytes:  # src/bloom.rs:66-70
        self.flush()
        n = ctypes.c_uint64()
        _raise(_L().cb_filter_to_bytes(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(max(int(n.value), 1), np.uint8)
        _raise(_L().cb_filter_to_bytes(self._h, out.ctypes.data, int(n.value), ctypes.byref(n)))
        return out[: int(n.value)].tobytes()

    @classmethod
    def from_bytes(cls, data: bytes, device: int = 0) -> "BloomFilter":  # src/bloom.rs:74-77
        buf = np.frombuffer(bytes(data), np.uint8) if data else np.zeros(1, np.uint8)
        h = ctypes.c_void_p()
        _raise(_L().cb_filter_from_bytes(buf.ctypes.data, len(data), device, ctypes.byref(h)))
        return cls(0, _handle=h.value)


# ---- batched multi-filter build (concurrent flushes) ---------------------------------

def insert_many(filters: Sequence["BloomFilter"], keys_per_filter, stream=None) -> None:
    """filters[i].insert of every row of keys_per_filter[i] (uint8 [n_i, L]
    arrays or device tensors, one key length L), all built together."""
    nf = len(filters)
    if nf == 0:
        return
    for f in filters:
        f.flush(stream)
    batches = [as_batch(k) for k in keys_per_filter]
    if len(batches) != nf or any(b.is_var for b in batches):
        raise ValueError("one fixed-length key array per filter")
    kl = {b.key_len for b in batches if b.n}
    if len(kl) > 1:
        raise ValueError("all key arrays must share one key length")
    key_len = kl.pop() if kl else 0
    keep = []
    ptrs = (ctypes.c_void_p * nf)()
    ns = (ctypes.c_uint64 * nf)()
    for i, b in enumerate(batches):
        p, k = _ptr_of(b.keys) if b.n else (None, None)
        keep.append(k)
        ptrs[i] = p
        ns[i] = b.n
    hs = (ctypes.c_void_p * nf)(*[f.handle.value for f in filters])
    _raise(_L().cb_filter_insert_fixed_many(ctypes.cast(hs, ctypes.c_void_p), nf,
                                            ctypes.cast(ptrs, ctypes.c_void_p), key_len,
                                            ctypes.cast(ns, ctypes.c_void_p), _stream(stream)))


# ---- batched multi-filter probe ------------------------------------------------------

def probe(filters: Sequence[BloomFilter], keys, out=None, stream=None) -> np.ndarray:
    """may_contain of every key against every filter (Database::get's fan-out,
    src/lib.rs:129-134). Returns (or fills ``out``) uint64[nf, ceil(n/64)]:
    bit k%64 of word [f][k/64] = filters[f].may_contain(key k)."""
    b = as_batch(keys)
    nf = len(filters)
    for f in filters:
        f.flush(stream)
    words = (b.n + 63) // 64
    if out is None:
        out = np.zeros((nf, max(words, 1)), np.uint64)
        result = out[:, :words]
    else:
        result = out
    arr = (ctypes.c_void_p * max(nf, 1))(*[f.handle.value for f in filters])
    op, keep = _ptr_of(out)
    s = _stream(stream)
    if b.is_var:
        dp, k1 = _ptr_of(b.data)
        offp, k2 = _ptr_of(b.offsets)
        _raise(_L().cb_probe_var(ctypes.cast(arr, ctypes.c_void_p), nf, dp, offp, b.n, op, s))
    else:
        kp, k1 = _ptr_of(b.keys)
        _raise(_L().cb_probe_fixed(ctypes.cast(arr, ctypes.c_void_p), nf, kp, b.key_len, b.n, op, s))
    return result


class FilterSet:
    """Up to ``width`` filters of one size m, bit-sliced in HBM for the
    read-path fan-out (Database::get, src/lib.rs:129-134): one probe call
    answers may_contain for every slot with two word (or row) reads per key.
    width 32 or 64, or a wide set of any multiple of 64 up to 4096 slots
    (rows of width/64 uint64 words: the reference's real shape of hundreds of
    m = 1024 tables, src/sstable.rs:44,59, src/lib.rs:72,105). A derived copy —
    the BloomFilter handles remain the source of truth."""

    def __init__(self, m: int, width: int = 32, device: int = 0):
        self._h = ctypes.c_void_p()
        _raise(_L().cb_set_create(int(m), int(width), int(device), ctypes.byref(self._h)))
        self.m, self.width, self.device = int(m), int(width), int(device)

    @classmethod
    def from_filters(cls, filters: Sequence[BloomFilter], width: int | None = None,
                     stream=None) -> "FilterSet":
        if not filters:
            raise ValueError("need at least one filter")
        width = width or (32 if len(filters) <= 32 else 64 if len(filters) <= 64 else
                          (len(filters) + 63) // 64 * 64)
        s = cls(filters[0].m, width, device=filters[0].device)
        s.assign_all(filters, stream=stream)
        return s

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _L().cb_set_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def used(self) -> int:
        u = ctypes.c_uint32()
        check(_L().cb_set_info(self._h, None, None, ctypes.byref(u)))
        return int(u.value)

    def assign(self, slot: int, f: BloomFilter, stream=None) -> None:
        f.flush(stream)
        _raise(_L().cb_set_assign(self._h, int(slot), f.handle, _stream(stream)))

    def assign_all(self, filters: Sequence[BloomFilter], stream=None) -> None:
        for f in filters:
            f.flush(stream)
        arr = (ctypes.c_void_p * max(len(filters), 1))(*[f.handle.value for f in filters])
        _raise(_L().cb_set_assign_all(self._h, ctypes.cast(arr, ctypes.c_void_p), len(filters),
                                      _stream(stream)))

    def clear_slot(self, slot: int, stream=None) -> None:
        _raise(_L().cb_set_clear_slot(self._h, int(slot), _stream(stream)))

    def set_zone(self, slot: int, zone: "ZoneMap | tuple", stream=None) -> None:
        """Slot's zone map := zone (ZoneMap or (min, max) bytes/str/None)."""
        lo, hi = (zone.min, zone.max) if isinstance(zone, ZoneMap) else zone
        lo = lo.encode() if isinstance(lo, str) else lo
        hi = hi.encode() if isinstance(hi, str) else hi
        lb = np.frombuffer(lo, np.uint8) if lo else np.zeros(1, np.uint8)
        hb = np.frombuffer(hi, np.uint8) if hi else np.zeros(1, np.uint8)
        _raise(_L().cb_set_zone(self._h, int(slot), lb.ctypes.data_as(ctypes.c_void_p), len(lo or b""),
                                lo is not None, hb.ctypes.data_as(ctypes.c_void_p), len(hi or b""),
                                hi is not None, _stream(stream)))

    def zone(self, slot: int) -> ZoneMap:
        ll, hl = ctypes.c_uint64(), ctypes.c_uint64()
        hasl, hash_ = ctypes.c_int(), ctypes.c_int()
        check(_L().cb_set_zone_get(self._h, int(slot), None, 0, ctypes.byref(ll), ctypes.byref(hasl), None, 0,
                                   ctypes.byref(hl), ctypes.byref(hash_)))
        lb = np.zeros(max(ll.value, 1), np.uint8)
        hb = np.zeros(max(hl.value, 1), np.uint8)
        check(_L().cb_set_zone_get(self._h, int(slot), lb.ctypes.data_as(ctypes.c_void_p), lb.size, ctypes.byref(ll),
                                   ctypes.byref(hasl), hb.ctypes.data_as(ctypes.c_void_p), hb.size,
                                   ctypes.byref(hl), ctypes.byref(hash_)))
        return ZoneMap(lb[: ll.value].tobytes() if hasl.value else None,
                       hb[: hl.value].tobytes() if hash_.value else None)

    def load_meta(self, slot: int, data: bytes, stream=None) -> None:
        """Decode one table's ``.meta`` (TableMeta) straight into ``slot``:
        filter bits and zone map (the restart path, src/sstable.rs:96-108)."""
        buf = np.frombuffer(bytes(data), np.uint8).copy() if data else np.zeros(1, np.uint8)
        _raise(_L().cb_set_load_meta(self._h, int(slot), buf.ctypes.data, len(data), _stream(stream)))

    def zone_from_keys(self, slot: int, keys, stream=None) -> None:
        """ZoneMap::update over a key batch, on the device (src/sstable.rs:62-65)."""
        b = as_batch(keys)
        s = _stream(stream)
        if b.is_var:
            dp, k1 = _ptr_of(b.data)
            offp, k2 = _ptr_of(b.offsets)
            _raise(_L().cb_set_zone_from_keys_var(self._h, int(slot), dp, offp, b.n, s))
        else:
            kp, k1 = _ptr_of(b.keys)
            _raise(_L().cb_set_zone_from_keys_fixed(self._h, int(slot), kp, b.key_len, b.n, s))

    def probe_pack(self, keys, hits, pack, cap: int, gated: bool = False, stream=None) -> None:
        """The probe writing the exchange pack too (cb_set_probe_pack_fixed):
        keys uint8[n, key_len], hits int64[used][ceil(n/64)] and pack int32
        [pack_words(n, cap)], all device tensors."""
        n = int(keys.shape[0])
        kp, k1 = _ptr_of(keys)
        hp, k2 = _ptr_of(hits)
        pp, k3 = _ptr_of(pack)
        _raise(_L().cb_set_probe_pack_fixed(self._h, kp, int(keys.shape[1]), n, int(bool(gated)), hp, pp, int(cap),
                                            _stream(stream)))

    @staticmethod
    def pack_words(n: int, cap: int) -> int:
        out = ctypes.c_uint64()
        check(_L().cb_set_pack_words(int(n), int(cap), ctypes.byref(out)))
        return int(out.value)

    def probe(self, keys, out=None, stream=None, gated: bool = False) -> np.ndarray:
        """uint64[used, ceil(n/64)]: row s = slot s's may_contain bits; with
        gated=True, SsTable::get's full gate zone.contains && may_contain
        (src/sstable.rs:138)."""
        b = as_batch(keys)
        used = self.used
        words = (b.n + 63) // 64
        if out is None:
            out = np.zeros((max(used, 1), max(words, 1)), np.uint64)
            result = out[:used, :words]
        else:
            result = out
        op, keep = _ptr_of(out)
        s = _stream(stream)
        if b.is_var:
            dp, k1 = _ptr_of(b.data)
            offp, k2 = _ptr_of(b.offsets)
            fn = _L().cb_set_probe_gated_var if gated else _L().cb_set_probe_var
            _raise(fn(self._h, dp, offp, b.n, op, s))
        else:
            kp, k1 = _ptr_of(b.keys)
            fn = _L().cb_set_probe_gated_fixed if gated else _L().cb_set_probe_fixed
            _raise(fn(self._h, kp, b.key_len, b.n, op, s))
        return result


# ---- SSTable data files and the batched read path (src/sstable.rs:133-179, src/lib.rs:128-134)

class Table:
    """One SSTable data file (``key \t base64(value) \n`` lines, sorted;
    src/sstable.rs:57-72) resident in HBM with its line index, built on the
    device. ``data``: bytes, a uint8 numpy array, or a uint8 device tensor."""

    def __init__(self, data, device: int = 0, stream=None):
        self._h = ctypes.c_void_p()
        if isinstance(data, (bytes, bytearray, memoryview)):
            data = np.frombuffer(bytes(data), np.uint8)
        n = int(data.numel()) if hasattr(data, "numel") else int(len(data))
        ptr, keep = _ptr_of(data if n else np.zeros(1, np.uint8))
        _raise(_L().cb_table_create(ptr, n, int(device), _stream(stream), ctypes.byref(self._h)))
        self.device = int(device)

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _L().cb_table_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def wait(self) -> None:
        """Finalise a table from sstable_create(wait=False): wait for its
        enqueued work, take its results (raises its deferred error, if any)."""
        _raise(_L().cb_table_wait(self._h))
        self.__dict__.pop("_inputs", None)

    @property
    def nlines(self) -> int:
        n = ctypes.c_uint64()
        check(_L().cb_table_info(self._h, ctypes.byref(n), None))
        return int(n.value)

    @property
    def nbytes(self) -> int:
        n = ctypes.c_uint64()
        check(_L().cb_table_info(self._h, None, ctypes.byref(n)))
        return int(n.value)

    def data(self) -> bytes:
        """The data file's bytes (what storage.put writes, src/sstable.rs:73)."""
        n = self.nbytes
        out = np.zeros(max(n, 1), np.uint8)
        check(_L().cb_table_copy(self._h, 0, n, out.ctypes.data))
        return out[:n].tobytes()

    @classmethod
    def _adopt(cls, handle: int, device: int) -> "Table":
        t = cls.__new__(cls)
        t._h = ctypes.c_void_p(handle)
        t.device = device
        return t

    def _zone(self, which: int) -> bytes:
        """ZoneMap bound kept by cb_sstable_create: 0 = min, 1 = max (host copy)."""
        n = ctypes.c_uint64()
        check(_L().cb_table_zone(self._h, int(which), None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(int(n.value), 1))
        check(_L().cb_table_zone(self._h, int(which), buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def rebuild(self, m: int = 1024, stream=None) -> "tuple[BloomFilter, ZoneMap]":
        """SsTable::load's rebuild from the data file when `.meta` is missing or
        undecodable (src/sstable.rs:109-120), on the device: (bloom, zone_map)
        over the keys of the lines that have a TAB. A key that is not UTF-8
        raises UnicodeDecodeError, as the reference's load returns Err."""
        h = ctypes.c_void_p()
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        rc = _L().cb_table_rebuild(self._h, int(m), _stream(stream), ctypes.byref(h), ctypes.byref(lo),
                                   ctypes.byref(hi))
        if rc == _lib.CB_EUTF8:
            msg = _L().cb_last_error().decode()
            raise UnicodeDecodeError("utf-8", b"", 0, 1, msg)
        _raise(rc)
        z = ZoneMap()
        if lo.value != 0xFFFFFFFFFFFFFFFF:
            st, kl, _ = self.lines()
            raw = self.data()
            for li in (lo.value, hi.value):
                z.update(raw[int(st[li]):int(st[li]) + int(kl[li])])
        return BloomFilter(0, _handle=h.value), z

    @property
    def well_formed(self) -> bool:
        """A TAB on every line and strictly increasing keys (what SsTable::create
        writes): searched through the prefix/fence index."""
        v = ctypes.c_int()
        check(_L().cb_table_well_formed(self._h, ctypes.byref(v)))
        return bool(v.value)

    @staticmethod
    def force_exact(on: bool) -> None:
        """Tables created while on always replay the reference's exact
        (lo+hi)/2 search trajectory (tests / bench)."""
        check(_L().cb_table_force_exact(int(bool(on))))

    @staticmethod
    def bucket_limit(max_bytes: int) -> None:
        """The most device bytes one table's read-path key buckets may take
        (0: none for tables read from now on; default 1 GiB, and never over a
        quarter of the free device memory). Tables past it are searched
        without buckets: same answers, slower reads."""
        check(_L().cb_table_bucket_limit(int(max_bytes)))

    def lines(self):
        """(start uint64[n], key_len uint32[n] (0xFFFFFFFF = no TAB), line_len uint32[n])."""
        n = self.nlines
        st = np.zeros(max(n, 1), np.uint64)
        kl = np.zeros(max(n, 1), np.uint32)
        ll = np.zeros(max(n, 1), np.uint32)
        check(_L().cb_table_lines(self._h, st.ctypes.data, kl.ctypes.data, ll.ctypes.data))
        return st[:n], kl[:n], ll[:n]

    def search(self, keys, out=None, stream=None) -> np.ndarray:
        """SsTable::binary_search per key: int64 line index or -1."""
        b = as_batch(keys)
        if out is None:
            out = np.zeros(max(b.n, 1), np.int64)
            res = out[: b.n]
        else:
            res = out
        op, keep = _ptr_of(out)
        s = _stream(stream)
        if b.is_var:
            dp, k1 = _ptr_of(b.data)
            offp, k2 = _ptr_of(b.offsets)
            _raise(_L().cb_table_search_var(self._h, dp, offp, b.n, op, s))
        else:
            kp, k1 = _ptr_of(b.keys)
            _raise(_L().cb_table_search_fixed(self._h, kp, b.key_len, b.n, op, s))
        return res


def sstable_create(entries, m: int = 1024, device: int = 0, stream=None, wait: bool = True):
    """SsTable::create (src/sstable.rs:51-87) on the device. entries: a list of
    (key, value) pairs (str/bytes), or a (keys, values) pair of ragged
    KeyBatches. Returns (Table, BloomFilter of m bits, ZoneMap).

    The C call only enqueues (cb_sstable_create_bounded: device offsets are
    sized by their data buffers, no host round trip); the table finalises on
    first use. wait=False returns (Table, BloomFilter, None) without waiting
    for the zone bounds (Table.wait() or any read of the table finalises it);
    the key and value buffers must then stay alive until it has."""
    if isinstance(entries, tuple) and len(entries) == 2 and isinstance(entries[0], KeyBatch):
        kb, vb = entries
    else:
        kb = as_batch([k for k, _ in entries])
        vb = as_batch([v for _, v in entries])
    if not kb.is_var:
        kb = _to_var(kb)
    if not vb.is_var:
        vb = _to_var(vb)
    if kb.n != vb.n:
        raise ValueError("keys and values differ in count")
    th, fh = ctypes.c_void_p(), ctypes.c_void_p()
    kd, k1 = _ptr_of(kb.data)
    ko, k2 = _ptr_of(kb.offsets)
    vd, k3 = _ptr_of(vb.data)
    vo, k4 = _ptr_of(vb.offsets)

    def nbytes(x):
        return int(x.numel() * x.element_size()) if hasattr(x, "numel") else int(np.asarray(x).nbytes)
    if kb.n and hasattr(kb.offsets, "is_cuda") and kb.offsets.is_cuda:
        # device offsets: their data buffers bound the byte totals
        _raise(_L().cb_sstable_create_bounded(kd, ko, nbytes(kb.data), vd, vo, nbytes(vb.data), kb.n, int(m),
                                              int(device), _stream(stream), ctypes.byref(th), ctypes.byref(fh)))
    else:
        _raise(_L().cb_sstable_create(kd, ko, vd, vo, kb.n, int(m), int(device), _stream(stream), ctypes.byref(th),
                                      ctypes.byref(fh), None, None))
    table = Table._adopt(th.value, device)
    if not wait:
        table._inputs = (kb, vb)  # the enqueued work (and a fallback sort) reads them until finalised
    bloom = BloomFilter(0, device=device, _handle=fh.value)
    if not wait:
        return table, bloom, None
    zone = ZoneMap()
    if kb.n:
        zone = ZoneMap(table._zone(0), table._zone(1))
    return table, bloom, zone


def _to_var(b: KeyBatch) -> KeyBatch:
    keys = np.ascontiguousarray(b.keys)
    offs = (np.arange(0, b.key_len * (b.n + 1), b.key_len, dtype=np.uint64) if b.key_len
            else np.zeros(b.n + 1, np.uint64))
    data = keys.reshape(-1) if keys.size else np.zeros(1, np.uint8)
    return KeyBatch(n=b.n, data=data, offsets=offs)


_TABLE_ARRAYS: dict = {}  # id(sequence) -> (the tables' handle objects, their C array)
_HANDLE = operator.attrgetter("_h")


def _table_array(tables: Sequence[Table]):
    """The tables' handles as one C array, kept per sequence object while it
    holds the same open tables in the same order. A store passes its table
    list batch after batch (Database::get walks self.sstables, src/lib.rs:
    129-134), and converting 300 handles into a fresh ctypes array took ~70 us
    of host time per call, more than half the wide fan-out's device step.
    The check is one identity test per table against the handle objects
    stored here: Table.close() replaces a table's handle object, so a closed
    or different table never reuses a stored array (and holding the handle
    objects keeps no table alive)."""
    hs = list(map(_HANDLE, tables))
    hit = _TABLE_ARRAYS.get(id(tables))
    if hit is not None and hit[0] == hs:  # (ctypes handles compare by identity)
        return hit[1]
    arr = (ctypes.c_void_p * max(len(hs), 1))(*[h.value for h in hs])
    if len(_TABLE_ARRAYS) >= 8:
        _TABLE_ARRAYS.clear()  # (one call, so safe against another thread's insert)
    _TABLE_ARRAYS[id(tables)] = (hs, arr)
    return arr


def get_many(tables: Sequence[Table], keys, hits=None, hit_rows=None, stream=None, out=None, wait=True,
             filterset=None):
    """Database::get's newest-first walk for a key batch (tables[0] newest).
    hits: optional per-table gate bitmaps (e.g. FilterSet.probe(gated=True));
    table t uses row hit_rows[t] (default t). Returns (which int32[n]: table
    index or -1, val_off uint64[n+1], vals bytes).

    out=(which, val_off, vals) with preallocated (e.g. device) buffers runs
    one pass and returns (which, val_off, total); values are written only if
    vals is large enough for total. With wait=False (out, keys and hits on the
    device) the call only enqueues the work on stream and returns total None:
    val_off[n] holds it once the stream has run.

    filterset=FilterSet: Database::get in one launch (cb_set_get_many_*): each
    table's gate (its slot's ZoneMap and Bloom bits, as
    FilterSet.probe(gated=True)) is computed inside the search kernel, so no
    hit rows exist; hit_rows then names each table's slot (default t) and
    hits must be None. At most the set's width tables (a wide set: up to 4096
    in one launch)."""
    if filterset is not None and hits is not None:
        raise ValueError("filterset= computes the gate itself: pass hits=None")
    b = as_batch(keys)
    nt = len(tables)
    arr = _table_array(tables)
    hp, hk = _ptr_of(hits) if hits is not None else (None, None)
    rows = None
    if hit_rows is not None:
        rows = np.ascontiguousarray(hit_rows, dtype=np.uint32)
    rp = rows.ctypes.data if rows is not None else None
    total = ctypes.c_uint64()
    if not wait and out is None:
        raise ValueError("wait=False needs out= device buffers")
    tref = ctypes.byref(total) if wait else None
    s = _stream(stream)
    L = _L()
    if out is not None:
        which, voff, vals = out
        cap = int(vals.numel()) if hasattr(vals, "numel") else int(vals.nbytes)
    else:
        which = np.zeros(max(b.n, 1), np.int32)
        voff = np.zeros(b.n + 1, np.uint64)
    wp, k3 = _ptr_of(which)
    vo, k4 = _ptr_of(voff)
    if b.is_var:
        dp, k1 = _ptr_of(b.data)
        offp, k2 = _ptr_of(b.offsets)

        def call(vp, cap):
            if filterset is not None:
                _raise(L.cb_set_get_many_var(filterset._h, ctypes.cast(arr, ctypes.c_void_p), nt, rp, dp, offp, b.n,
                                             wp, vo, vp, cap, tref, s))
            else:
                _raise(L.cb_get_many_var(ctypes.cast(arr, ctypes.c_void_p), nt, hp, rp, dp, offp, b.n,
                                         wp, vo, vp, cap, tref, s))
    else:
        kp, k1 = _ptr_of(b.keys)

        def call(vp, cap):
            if filterset is not None:
                _raise(L.cb_set_get_many_fixed(filterset._h, ctypes.cast(arr, ctypes.c_void_p), nt, rp, kp, b.key_len,
                                               b.n, wp, vo, vp, cap, tref, s))
            else:
                _raise(L.cb_get_many_fixed(ctypes.cast(arr, ctypes.c_void_p), nt, hp, rp, kp, b.key_len, b.n,
                                           wp, vo, vp, cap, tref, s))
    if out is not None:
        call(_ptr_of(vals)[0], cap)
        return which, voff, (int(total.value) if wait else None)
    call(None, 0)
    vals = np.zeros(max(int(total.value), 1), np.uint8)
    call(vals.ctypes.data, int(total.value))
    return which[: b.n], voff, vals[: int(total.value)].tobytes()


def unpack_hits(hits: np.ndarray, n: int) -> np.ndarray:
    """uint64[nf, words] -> bool[nf, n]."""
    h = np.ascontiguousarray(hits, dtype="<u8")
    bits = np.unpackbits(h.view(np.uint8).reshape(h.shape[0], -1), axis=1, bitorder="little")
    return bits[:, :n].astype(bool)


# ---- multi-GPU exchange (lsmt_amd/shard.py) ---------------------

def _pack_blocks(nw: int) -> int:
    from .shard import PACK_BLOCK_WORDS
    return -(-int(nw) // PACK_BLOCK_WORDS)


def hits_compress(hits, pack, cap: int, stream=None) -> None:
    """pack (int32 device tensor) := {count, 0, set-bit positions[cap],
    directory} of hits ([rows][words] int64 device tensor): cb_hits_compress.
    cap is required: packs that are all-gathered share one stride (the
    largest shard's, cb_hits_pack_words), so every rank must pass the same cap
    and no rank may derive it from its own pack size."""
    rows, words = hits.shape
    cap = int(cap)
    if cap < 0 or int(pack.numel()) < 2 + cap + 2 * _pack_blocks(rows * words):
        raise ValueError("pack too small for cap positions and the directory")
    hp, k1 = _ptr_of(hits)
    pp, k2 = _ptr_of(pack)
    _raise(_L().cb_hits_compress(hp, rows, words, pp, cap, _stream(stream)))


def hits_expand(packs, world: int, row_off, full, cap: int, ok=None, stream=None) -> None:
    """full ([total_rows][words] int64 device tensor) := the OR of every
    rank's positions (packs: the all-gathered int32 [world * stride], stride
    = cb_hits_pack_words of the largest shard, every pack compressed with this
    same cap). ok: optional int32 device tensor, cleared to 0 when some rank's
    count exceeds cap (that rank's rows are then zeros in full)."""
    total_rows, words = full.shape
    bounds = [int(x) for x in row_off] + [int(total_rows)]
    max_rows = max(bounds[r + 1] - bounds[r] for r in range(world))
    if int(packs.numel()) < world * (2 + int(cap) + 2 * _pack_blocks(max_rows * words)):
        raise ValueError("packs too small for world packs of the largest shard's stride")
    off = (ctypes.c_uint64 * world)(*bounds[:world])
    pp, k1 = _ptr_of(packs)
    fp, k2 = _ptr_of(full)
    op, k3 = _ptr_of(ok)
    _raise(_L().cb_hits_expand(pp, world, int(cap), off, words, total_rows, fp, op, _stream(stream)))


def hits_expand_set(packs, world: int, row_off, n: int, full, cap: int, ok=None, stream=None) -> None:
    """full ([total_rows][ceil(n/64)] int64 device tensor) := every rank's
    rows from packs written by FilterSet.probe_pack (all-gathered int32,
    world x FilterSet.pack_words(n, cap)): cb_hits_expand_set."""
    total_rows = int(full.shape[0])
    off = (ctypes.c_uint64 * world)(*[int(x) for x in row_off])
    pp, k1 = _ptr_of(packs)
    fp, k2 = _ptr_of(full)
    op, k3 = _ptr_of(ok)
    _raise(_L().cb_hits_expand_set(pp, world, int(cap), off, int(n), total_rows, fp, op, _stream(stream)))
