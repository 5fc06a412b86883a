"""Synthetic, deterministic key batches for the BASELINE configs.

``key(seed, i)`` is the 16 lowercase hex characters (most-significant nibble
first) of ``splitmix64(seed * 2**32 + i)`` — 16 bytes of valid UTF-8, i.e. a
legal Rust ``&str`` for ``BloomFilter::insert``/``may_contain``
(/root/reference/src/bloom.rs:40,48). Generated with numpy on the host; the
bench copies them to HBM before the timed region.
"""
from __future__ import annotations

import numpy as np

_HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
_M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=False)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


# byte b -> its two lowercase hex chars, high nibble first in memory
_HEX2 = (_HEX[np.arange(256) >> 4].astype(np.uint16) | (_HEX[np.arange(256) & 15].astype(np.uint16) << 8))


def hex16(v: np.ndarray) -> np.ndarray:
    """uint64[n] -> uint8[n,16] lowercase hex, most-significant nibble first
    (one 2-char table lookup per byte of the big-endian value)."""
    be = np.ascontiguousarray(v, dtype=np.uint64).astype(">u8").view(np.uint8).reshape(-1, 8)
    return _HEX2[be].view(np.uint8).reshape(-1, 16)


def keys(seed: int, idx) -> np.ndarray:
    """key(seed, i) for every i in ``idx`` (array-like of ints) -> uint8[n,16]."""
    idx = np.asarray(idx, dtype=np.uint64)
    return hex16(splitmix64(np.uint64((seed << 32) & _M64) + idx))


def key_range(seed: int, n: int, first: int = 0) -> np.ndarray:
    return keys(seed, np.arange(first, first + n, dtype=np.uint64))


# ---- BASELINE configs ---------------------------------------

def c2_build_keys(n: int = 1 << 20) -> np.ndarray:
    """C2: N keys key(1, i) -> one m = 2^27 (16 MiB) filter."""
    return key_range(1, n)


def probe_lookups(n: int, nf: int, keys_per_filter: int, seed_base: int, absent_seed: int,
                  shift: int = 0) -> np.ndarray:
    """Lookup batch of the probe configs: even i -> present key
    key(seed_base + j mod nf, (j div nf + shift) mod keys_per_filter) with
    j = i/2; odd i -> absent key key(absent_seed, i). shift = 0 is the
    SURVEY.md §8d batch; other shifts give further batches over the same
    filters (bench.py's rotating-batch leg)."""
    i = np.arange(n, dtype=np.uint64)
    out = np.empty((n, 16), np.uint8)
    j = i[0::2] // np.uint64(2)
    seed = np.uint64(seed_base) + j % np.uint64(nf)
    kidx = (j // np.uint64(nf) + np.uint64(shift)) % np.uint64(keys_per_filter)
    with np.errstate(over="ignore"):
        out[0::2] = hex16(splitmix64(((seed << np.uint64(32)) & np.uint64(_M64)) + kidx))
    out[1::2] = keys(absent_seed, i[1::2])
    return out


def c3_filter_keys(f: int, keys_per_filter: int = 1 << 19) -> np.ndarray:
    """C3: filter f is built from key(100 + f, i), i < 2^19."""
    return key_range(100 + f, keys_per_filter)


def c3_lookups(n: int = 1 << 20, nf: int = 32, keys_per_filter: int = 1 << 19) -> np.ndarray:
    return probe_lookups(n, nf, keys_per_filter, seed_base=100, absent_seed=999)


def c4_filter_keys(f: int, keys_per_filter: int = 1 << 18) -> np.ndarray:
    """C4: filter f (of 64, m = 2^25) is built from key(200 + f, i)."""
    return key_range(200 + f, keys_per_filter)


def c5_filter_keys(f: int, keys_per_filter: int = 1 << 19) -> np.ndarray:
    """C5: filter f (of 256, m = 2^26) is built from key(1000 + f, i)."""
    return key_range(1000 + f, keys_per_filter)


def c5_lookups(n: int = 10_000_000, nf: int = 256, keys_per_filter: int = 1 << 19) -> np.ndarray:
    return probe_lookups(n, nf, keys_per_filter, seed_base=1000, absent_seed=9999)


def var_keys(rng: np.random.Generator, n: int, max_len: int = 48):
    """Ragged UTF-8-ish keys (bytes + offsets[n+1]) for the var-length paths,
    shaped like the product's "ns:pk|ck" keys (src/lib.rs:155)."""
    lens = rng.integers(0, max_len + 1, size=n, dtype=np.int64)
    offsets = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offsets[1:])
    data = rng.integers(0x20, 0x7F, size=int(offsets[-1]), dtype=np.uint8)
    return data, offsets


# ---- range-partitioned tables (zone-map gate) -------------

_HEX_DIGITS = b"0123456789abcdef"


def zone_tables(nt: int = 8, seed_base: int = 300, per_seed: int = 40_000) -> list[np.ndarray]:
    """nt tables whose key ranges are disjoint, as after range compaction: table
    f keeps the keys of key(seed_base + f, i < per_seed) whose first hex digit
    is one of its 16/nt digits. Each table's zone map is then a narrow slice of
    the key space, so SsTable::get's zone gate rejects most other-range keys."""
    span = 16 // nt
    out = []
    for f in range(nt):
        ks = key_range(seed_base + f, per_seed)
        digits = np.frombuffer(_HEX_DIGITS[span * f: span * (f + 1)], np.uint8)
        out.append(np.ascontiguousarray(ks[np.isin(ks[:, 0], digits)]))
    return out


def zone_lookups(tables: list[np.ndarray], n: int, absent_seed: int = 998, rng_seed: int = 5) -> np.ndarray:
    """Even i: a key drawn from the union of the tables; odd i: key(absent_seed, i/2)."""
    present = np.concatenate(tables)
    pick = np.random.default_rng(rng_seed).integers(0, len(present), n // 2)
    out = np.empty((n, 16), np.uint8)
    out[0::2] = present[pick]
    out[1::2] = key_range(absent_seed, n - n // 2)[: len(out[1::2])]
    return out


# ---- SSTable data files ------------------------------------

_B64 = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/", np.uint8)


def b64_rows(v: np.ndarray) -> np.ndarray:
    """Standard padded base64 of each row of a uint8 [n, L] array -> [n, 4*ceil(L/3)]."""
    n, L = v.shape
    pad = (-L) % 3
    x = np.concatenate([v, np.zeros((n, pad), np.uint8)], axis=1).reshape(n, -1, 3).astype(np.uint32)
    w = x[..., 0] << 16 | x[..., 1] << 8 | x[..., 2]
    out = np.stack([_B64[(w >> s) & 63] for s in (18, 12, 6, 0)], axis=-1).reshape(n, -1)
    if pad:
        out[:, out.shape[1] - pad:] = ord("=")
    return out


def sort_keys16(keys: np.ndarray) -> np.ndarray:
    """Rows of a uint8 [n, 16] array in Rust str order (byte-wise)."""
    w = keys.view(">u8").reshape(len(keys), 2)
    return keys[np.lexsort((w[:, 1], w[:, 0]))]


def table_value(keys: np.ndarray, table_id: int) -> np.ndarray:
    """The stored value of each key in table `table_id`: an 8-byte big-endian
    timestamp (insert_ts layout, src/lib.rs:111-115) then the key's first 8 bytes."""
    ts = np.frombuffer(np.array([table_id], dtype=">u8").tobytes(), np.uint8)
    return np.concatenate([np.broadcast_to(ts, (len(keys), 8)), keys[:, :8]], axis=1)


def sstable_bytes(keys: np.ndarray, values: np.ndarray) -> np.ndarray:
    """SsTable::create's data file (src/sstable.rs:57-72) for 16-byte keys:
    lines `key \\t base64(value) \\n` sorted by key."""
    order = np.lexsort(tuple(keys.view(">u8").reshape(len(keys), 2)[:, ::-1].T)) if len(keys) else []
    k = keys[order]
    v = b64_rows(values[order])
    n = len(k)
    tab = np.full((n, 1), ord("\t"), np.uint8)
    nl = np.full((n, 1), ord("\n"), np.uint8)
    return np.ascontiguousarray(np.concatenate([k, tab, v, nl], axis=1).reshape(-1))
