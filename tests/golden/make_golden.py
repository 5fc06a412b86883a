"""Generate the committed golden fixtures for the Bloom-filter path.

Independent restatement of /root/reference/src/bloom.rs:26-51 in Python
big-int arithmetic (masked to 64 bits = Rust's wrapping u64), plus a numpy
vectorised restatement for the large configs; the two are cross-checked here
on every small case before anything is written. Neither imports the C oracle
or the product library, so the fixtures pin both of them independently.

The Rust reference cannot be built in this image (no cargo/rustc): the
fixtures therefore follow the reference's formula, and are anchored on the
reference's own tests: tests/bloom_test.rs:3-8 (m=128, "hello" present),
tests/sstable_test.rs:10-14 ("a","b","c" at m=1024), tests/lsm_flush_test.rs
(m=1024, "k1","k2","missing"), tests/sstable_local_test.rs:7-12 ("k").

Usage:  python tests/golden/make_golden.py      (~1-2 min; writes golden.json)
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

M64 = (1 << 64) - 1
HERE = os.path.dirname(os.path.abspath(__file__))


# ---- pure-Python big-int restatement -----------------------------------------

def raw_hashes(key: bytes) -> tuple[int, int]:
    h1, h2 = 5381, 0  # src/bloom.rs:28,30
    for b in key:  # src/bloom.rs:31-34
        h1 = ((h1 << 5) + h1 + b) & M64
        h2 = (h2 * 31 + b) & M64
    return h1, h2


def positions(key: bytes, m: int) -> tuple[int, int]:
    h1, h2 = raw_hashes(key)
    return h1 % m, h2 % m  # src/bloom.rs:35-36


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key(seed: int, i: int) -> bytes:
    return format(splitmix64(((seed << 32) + i) & M64), "016x").encode()


# ---- numpy restatement (large configs) -----------------------------------------

def np_keys(seed: int, idx: np.ndarray) -> np.ndarray:
    x = np.uint64((seed << 32) & M64) + idx.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
    sh = np.arange(60, -4, -4, dtype=np.uint64)
    return hexd[((z[:, None] >> sh[None, :]) & np.uint64(15)).astype(np.intp)]


def np_raw_hashes(keys: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    n = keys.shape[0]
    h1 = np.full(n, 5381, np.uint64)
    h2 = np.zeros(n, np.uint64)
    with np.errstate(over="ignore"):
        for j in range(keys.shape[1]):
            b = keys[:, j].astype(np.uint64)
            h1 = (h1 << np.uint64(5)) + h1 + b
            h2 = h2 * np.uint64(31) + b
    return h1, h2


def np_build(keys: np.ndarray, m: int) -> np.ndarray:
    h1, h2 = np_raw_hashes(keys)
    bits = np.zeros(m, np.uint8)
    bits[(h1 % np.uint64(m)).astype(np.int64)] = 1
    bits[(h2 % np.uint64(m)).astype(np.int64)] = 1
    return bits


def np_probe(bits: np.ndarray, keys: np.ndarray) -> np.ndarray:
    m = bits.shape[0]
    h1, h2 = np_raw_hashes(keys)
    a = bits[(h1 % np.uint64(m)).astype(np.int64)]
    b = bits[(h2 % np.uint64(m)).astype(np.int64)]
    return (a & b).astype(bool)


def _pack64(bits01: np.ndarray) -> np.ndarray:
    """bool[n] -> uint64[ceil(n/64)]: bit k%64 of word k/64, LSB-first, tail zero."""
    words = (bits01.shape[0] + 63) // 64
    padded = np.zeros(words * 64, np.uint8)
    padded[: bits01.shape[0]] = bits01
    return np.packbits(padded, bitorder="little").view("<u8").astype(np.uint64)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def lookups(n: int, nf: int, kpf: int, base: int, absent: int) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    out = np.empty((n, 16), np.uint8)
    j = i[0::2] // np.uint64(2)
    f = j % np.uint64(nf)
    kidx = (j // np.uint64(nf)) % np.uint64(kpf)
    ev = np.empty((len(j), 16), np.uint8)
    for fs in range(nf):
        sel = f == np.uint64(fs)
        ev[sel] = np_keys(base + fs, kidx[sel])
    out[0::2] = ev
    out[1::2] = np_keys(absent, i[1::2])
    return out


def main() -> None:
    g: dict = {"source": "tests/golden/make_golden.py (Python big-int + numpy restatement of src/bloom.rs:26-51)"}

    # 1. known-answer raw hashes and positions
    kat_keys = [b"", b"hello", b"k", b"a", b"b", b"c", b"k1", b"k2", b"missing", b"0123456789abcdef",
                "ns:pk|ck".encode(), "utf8-é✓".encode(), bytes(range(256)), b"\xff" * 40]
    ms = [1, 2, 3, 128, 1000, 1024, 100003, 1 << 17, 1 << 25, 1 << 26, 1 << 27, (1 << 32) + 15, (1 << 61) - 1]
    kat = []
    for k in kat_keys:
        h1, h2 = raw_hashes(k)
        kat.append({"key_hex": k.hex(), "h1": str(h1), "h2": str(h2),
                    "pos": {str(m): [h1 % m, h2 % m] for m in ms}})
    g["kat"] = kat
    assert positions(b"hello", 128) == (25, 82)          # pins tests/bloom_test.rs:5-7
    assert positions(b"hello", 1024) == (153, 210)
    assert positions(b"k", 1024) == (528, 107)            # tests/sstable_local_test.rs:7
    assert positions(b"0123456789abcdef", 1 << 27) == (84411015, 17008296)

    # 2. the reference's own test scenarios as bit arrays (m = 1024 everywhere in the product)
    def build_py(keys, m):
        bits = bytearray(m)
        for k in keys:
            a, b = positions(k, m)
            bits[a] = 1
            bits[b] = 1
        return bytes(bits)

    def may_py(bits, k):
        a, b = positions(k, len(bits))
        return bool(bits[a]) and bool(bits[b])

    scen = {}
    for name, m, ins, probes in [
        ("bloom_test", 128, [b"hello"], [b"hello", b"world", b""]),
        ("sstable_test", 1024, [b"a", b"b", b"c"], [b"a", b"b", b"c", b"d"]),
        ("lsm_flush_test", 1024, [b"k1", b"k2"], [b"k1", b"k2", b"missing"]),
        ("sstable_local_test", 1024, [b"k"], [b"k", b"v"]),
    ]:
        bits = build_py(ins, m)
        scen[name] = {"m": m, "insert_hex": [k.hex() for k in ins], "set_bits": [i for i, v in enumerate(bits) if v],
                      "probe_hex": [k.hex() for k in probes], "probe": [may_py(bits, k) for k in probes],
                      "to_bytes_hex": (bytes([0x0A]) + _varint(m) + bits).hex()}
    assert scen["bloom_test"]["probe"][0] is True
    assert scen["lsm_flush_test"]["probe"][2] is False
    g["scenarios"] = scen

    # 3. synthetic keys: python vs numpy, first 2000 keys of seed 1 and their positions
    idx = np.arange(2000, dtype=np.uint64)
    npk = np_keys(1, idx)
    pyk = [key(1, i) for i in range(2000)]
    assert all(npk[i].tobytes() == pyk[i] for i in range(2000))
    h1n, h2n = np_raw_hashes(npk)
    for i in range(2000):
        assert (int(h1n[i]), int(h2n[i])) == raw_hashes(pyk[i])
    g["keys_seed1_first8"] = [k.decode() for k in pyk[:8]]
    g["keys_seed1_2000_sha256"] = hashlib.sha256(b"".join(pyk)).hexdigest()
    g["hashes_seed1_2000"] = {"h1_sha256": sha(h1n.astype("<u8")), "h2_sha256": sha(h2n.astype("<u8"))}

    # 4. C1: 10k keys key(1,i) into m=2^17 and m=100003; FP on 100k absent keys key(2,i)
    c1 = {}
    k10 = np_keys(1, np.arange(10_000, dtype=np.uint64))
    absent = np_keys(2, np.arange(100_000, dtype=np.uint64))
    for m in (1 << 17, 100003):
        bits = np_build(k10, m)
        # cross-check the numpy build against the big-int one
        assert bits.tobytes() == build_py([bytes(r) for r in k10], m)
        present = np_probe(bits, k10)
        assert present.all()
        fp = np_probe(bits, absent)
        c1[str(m)] = {"n": 10_000, "bools_sha256": sha(bits), "popcount": int(bits.sum()),
                      "fp_absent_100k": int(fp.sum()), "fp_hits_sha256": sha(_pack64(fp))}
    g["c1"] = c1

    # 5. C2: 1M keys key(1,i) -> m = 2^27
    n2, m2 = 1 << 20, 1 << 27
    bits = np_build(np_keys(1, np.arange(n2, dtype=np.uint64)), m2)
    g["c2"] = {"n": n2, "m": m2, "bools_sha256": sha(bits), "popcount": int(bits.sum()),
               "packed_sha256": sha(np.packbits(bits, bitorder="little"))}
    del bits

    # 6. C3: 32 filters m=2^26 from key(100+f, i<2^19); 2^20 lookups
    nf, m3, kpf, nl = 32, 1 << 26, 1 << 19, 1 << 20
    lk = lookups(nl, nf, kpf, 100, 999)
    rows = []
    pops = []
    for f in range(nf):
        b = np_build(np_keys(100 + f, np.arange(kpf, dtype=np.uint64)), m3)
        pops.append(int(b.sum()))
        rows.append(np_probe(b, lk))
    hits = np.stack([_pack64(r) for r in rows])
    g["c3"] = {"nf": nf, "m": m3, "keys_per_filter": kpf, "n_lookups": nl,
               "lookups_sha256": sha(lk), "filter_popcounts": pops,
               "hits_sha256": sha(hits.astype("<u8")), "hits_popcount": int(sum(int(r.sum()) for r in rows)),
               "hits_per_filter": [int(r.sum()) for r in rows]}

    # 7. zone maps (src/zonemap.rs:21-42) and the SsTable::get gate (src/sstable.rs:138).
    #    Python's bytes order is Rust's str order (byte-wise, a prefix sorts first).
    def zone_of(keys):
        lo = hi = None
        for k in keys:  # zonemap.rs:21-32
            if lo is None or k < lo:
                lo = k
            if hi is None or k > hi:
                hi = k
        return lo, hi

    def zone_has(z, k):  # zonemap.rs:37-42
        return z[0] is None or z[1] is None or z[0] <= k <= z[1]

    zsc = {}
    for name, m, ins, probes in [
        ("sstable_test", 1024, [b"a", b"b", b"c"], [b"a", b"b", b"c", b"d", b"", b"ab", b"c\x00"]),
        ("lsm_flush_test", 1024, [b"k1", b"k2"], [b"k1", b"k2", b"missing", b"k", b"k10", b"k3", b"j"]),
        ("sstable_local_test", 1024, [b"k"], [b"k", b"v", b"j", b"k\x00", b""]),
        ("utf8", 1024, ["é".encode(), "z".encode(), "✓".encode()],
         ["é".encode(), "e".encode(), "ê".encode(), "✓".encode(), "✔".encode(), b"\xff"]),
    ]:
        bits = build_py(ins, m)
        z = zone_of(ins)
        zsc[name] = {"m": m, "insert_hex": [k.hex() for k in ins], "min_hex": z[0].hex(), "max_hex": z[1].hex(),
                     "probe_hex": [k.hex() for k in probes],
                     "zone": [zone_has(z, k) for k in probes],
                     "gate": [zone_has(z, k) and may_py(bits, k) for k in probes]}
    assert zsc["sstable_local_test"]["gate"][0] is True          # tests/sstable_local_test.rs:14-15
    assert zsc["lsm_flush_test"]["gate"][2] is False             # tests/lsm_flush_test.rs:23
    assert zsc["sstable_test"]["gate"][:3] == [True, True, True]  # tests/sstable_test.rs:13-14

    # range-partitioned tables: table f keeps the keys of key(300+f, i<40000)
    # whose first hex digit is in {2f, 2f+1}; its zone is the min/max of those.
    nt, mz = 8, 50021  # small generic-mode m: Bloom FPs common, so the gate matters
    tables, zones = [], []
    for f in range(nt):
        ks = np_keys(300 + f, np.arange(40_000, dtype=np.uint64))
        first = ks[:, 0]
        keep = (first == ord("0123456789abcdef"[2 * f])) | (first == ord("0123456789abcdef"[2 * f + 1]))
        ks = ks[keep]
        tables.append(ks)
        zones.append(zone_of([bytes(r) for r in ks]))
    nlz = 100_000
    present = np.concatenate(tables)
    pick = np.random.default_rng(5).integers(0, len(present), nlz // 2)
    lkz = np.empty((nlz, 16), np.uint8)
    lkz[0::2] = present[pick]
    lkz[1::2] = np_keys(998, np.arange(nlz // 2, dtype=np.uint64))
    lk_bytes = [bytes(r) for r in lkz]
    ungated, gated = [], []
    for f in range(nt):
        b = np_build(tables[f], mz)
        bloom = np_probe(b, lkz)
        zmask = np.array([zone_has(zones[f], k) for k in lk_bytes])
        ungated.append(_pack64(bloom))
        gated.append(_pack64(bloom & zmask))
    g["zone"] = {"scenarios": zsc, "tables": nt, "m": mz, "seed_base": 300, "keys_per_seed": 40_000,
                 "n_lookups": nlz, "lookups_sha256": sha(lkz),
                 "table_sizes": [int(len(t)) for t in tables],
                 "zones_hex": [[z[0].hex(), z[1].hex()] for z in zones],
                 "hits_sha256": sha(np.stack(ungated).astype("<u8")),
                 "gated_sha256": sha(np.stack(gated).astype("<u8")),
                 "hits_popcount": int(sum(np.unpackbits(r.view(np.uint8)).sum() for r in ungated)),
                 "gated_popcount": int(sum(np.unpackbits(r.view(np.uint8)).sum() for r in gated))}

    # 8. TableMeta `.meta` codec (src/sstable.rs:31-37,74-81,96-108; zonemap.rs:11-17)
    g["meta"] = meta_fixtures(build_py)

    # 9. SSTable data files: split, binary search, base64, newest-first get
    #    (src/sstable.rs:57-72,133-179; src/lib.rs:128-134)
    g["sstable"] = sstable_fixtures()

    # 10. SsTable::create's data file (src/sstable.rs:56-72)
    g["create"] = create_fixtures()

    # 11-12. C4 (64 concurrent builds) and C5 (10M keys x 256 filters, per-rank slices)
    g["c4"] = c4_fixture()
    g["c5"] = c5_fixture()

    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(g, fh, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.json"))


# ---- TableMeta: independent pure-Python prost restatement --------------------------

def _ld(field: int, payload: bytes) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def meta_encode_py(bits: bytes | None, zone) -> bytes:
    """prost: a present optional message/string is written even when empty;
    BloomProto's repeated bool is packed and omitted when empty."""
    out = b""
    if bits is not None:
        out += _ld(1, _ld(1, bits) if bits else b"")
    if zone is not None:
        z = b""
        if zone[0] is not None:
            z += _ld(1, zone[0])
        if zone[1] is not None:
            z += _ld(2, zone[1])
        out += _ld(2, z)
    return out


class _Bad(Exception):
    pass


def _rd_varint(b: bytes, i: int) -> tuple[int, int]:
    v = 0
    for k in range(10):
        if i >= len(b):
            raise _Bad("eof")
        c = b[i]
        i += 1
        if k == 9 and c > 1:
            raise _Bad("varint overflow")
        v |= (c & 0x7F) << (7 * k)
        if not c & 0x80:
            return v, i
    raise _Bad("varint too long")


def _fields(b: bytes):
    """(field, wire_type, value) triples of one message level; fixed-width and
    group fields are validated and skipped (value None)."""
    i = 0
    while i < len(b):
        key, j = _rd_varint(b, i)
        if key > 0xFFFFFFFF:
            raise _Bad("key")
        f, wt = key >> 3, key & 7
        if f == 0:
            raise _Bad("tag 0")
        if wt == 0:
            v, i = _rd_varint(b, j)
        elif wt == 2:
            n, j = _rd_varint(b, j)
            if n > len(b) - j:
                raise _Bad("eof")
            v, i = b[j:j + n], j + n
        elif wt in (1, 3, 5):
            v, i = None, _skip_one(b, i, 0)
        else:
            raise _Bad("wire type")  # 4 (stray end-group), 6, 7
        yield f, wt, v


def _skip_one(b: bytes, i: int, depth: int) -> int:
    key, j = _rd_varint(b, i)
    if key > 0xFFFFFFFF:
        raise _Bad("key")
    f, wt = key >> 3, key & 7
    if f == 0:
        raise _Bad("tag 0")
    if wt == 0:
        return _rd_varint(b, j)[1]
    if wt == 1:
        if len(b) - j < 8:
            raise _Bad("eof")
        return j + 8
    if wt == 5:
        if len(b) - j < 4:
            raise _Bad("eof")
        return j + 4
    if wt == 2:
        n, j = _rd_varint(b, j)
        if n > len(b) - j:
            raise _Bad("eof")
        return j + n
    if wt == 3:
        if depth > 100:
            raise _Bad("recursion")
        while True:
            k2, jj = _rd_varint(b, j)
            if k2 & 7 == 4:
                if k2 >> 3 != f:
                    raise _Bad("group mismatch")
                return jj
            j = _skip_one(b, j, depth + 1)
    raise _Bad("wire type")


def _bloom_bits(payload: bytes) -> list[int]:
    bits = []
    for f, wt, v in _fields(payload):
        if f == 1:
            if wt == 2:
                j = 0
                while j < len(v):
                    x, j = _rd_varint(v, j)
                    bits.append(int(x != 0))
            elif wt == 0:
                bits.append(int(v != 0))
            else:
                raise _Bad("bits wire type")
    return bits


def meta_decode_py(b: bytes):
    """-> None on a decode error, else {has_bloom, m, set_bits, has_zone, min, max}."""
    try:
        bits, has_bloom, zone = [], False, None
        for f, wt, v in _fields(b):
            if f in (1, 2) and wt != 2:
                raise _Bad("wire type")
            if f == 1:
                has_bloom = True
                bits += _bloom_bits(v)  # merge: repeated bits append
            elif f == 2:
                zone = zone or [None, None]
                for zf, zwt, zv in _fields(v):
                    if zf in (1, 2):
                        if zwt != 2:
                            raise _Bad("wire type")
                        zv.decode("utf-8")  # prost: string must be UTF-8
                        zone[zf - 1] = zv  # last wins
    except (_Bad, UnicodeDecodeError):
        return None
    return {"has_bloom": has_bloom, "m": len(bits), "set_bits": [i for i, x in enumerate(bits) if x],
            "has_zone": zone is not None,
            "min_hex": zone[0].hex() if zone and zone[0] is not None else None,
            "max_hex": zone[1].hex() if zone and zone[1] is not None else None}


def meta_fixtures(build_py) -> dict:
    enc = {}
    for name, keys in [("sstable_local_test", [b"k"]), ("sstable_test", [b"a", b"b", b"c"]),
                       ("lsm_flush_test", [b"k1", b"k2"]), ("empty_table", [])]:
        bits = build_py(keys, 1024)  # SsTable::create: BloomFilter::new(1024)
        zone = (min(keys), max(keys)) if keys else (None, None)
        b = meta_encode_py(bits, zone)
        d = meta_decode_py(b)
        assert d["m"] == 1024 and d["set_bits"] == [i for i, v in enumerate(bits) if v]
        enc[name] = {"keys_hex": [k.hex() for k in keys], "len": len(b), "sha256": hashlib.sha256(b).hexdigest(),
                     "head_hex": b[:8].hex(), "tail_hex": b[-16:].hex()}
    assert enc["empty_table"]["tail_hex"].endswith("1200")  # zone_map: Some(ZoneMapProto{None, None})

    z_az = _ld(1, b"a") + _ld(2, b"z")
    bl3 = _ld(1, bytes([1, 0, 1]))
    cases = {
        "zone_then_bloom": _ld(2, z_az) + _ld(1, bl3),
        "bloom_split": _ld(1, bl3) + _ld(1, _ld(1, bytes([0, 1]))),
        "bloom_unpacked": _ld(1, bytes([0x08, 0x01, 0x08, 0x00, 0x08, 0x02])),
        "bloom_packed_multibyte_varint": _ld(1, _ld(1, bytes([0x80, 0x01, 0x00, 0x01]))),
        "zone_last_wins": _ld(2, z_az) + _ld(2, _ld(1, b"b")),
        "zone_empty_min": _ld(2, _ld(1, b"")),
        "zone_utf8": _ld(2, _ld(1, "é".encode()) + _ld(2, "✓".encode())),
        "unknown_fields": (_varint(3 << 3 | 0) + _varint(300) + _varint(4 << 3 | 1) + bytes(8) +
                           _ld(5, b"xyz") + _varint(6 << 3 | 5) + bytes(4) +
                           _varint(7 << 3 | 3) + _varint(1 << 3 | 0) + b"\x01" + _varint(7 << 3 | 4) + bl3[:0] +
                           _ld(1, bl3)),
        "empty": b"",
        "empty_bloom": _ld(1, b""),
        "err_bloom_wire_type": _varint(1 << 3 | 0) + b"\x01",
        "err_zone_wire_type": _ld(2, _varint(1 << 3 | 0) + b"\x01"),
        "err_min_not_utf8": _ld(2, _ld(1, b"\xff")),
        "err_surrogate": _ld(2, _ld(2, b"\xed\xa0\x80")),
        "err_overlong": _ld(2, _ld(1, b"\xc0\x80")),
        "err_truncated": _ld(1, bl3)[:-1],
        "err_tag0": b"\x02\x00",
        "err_bloom_inner": _ld(1, b"\x0a\x02\x80"),
        "err_stray_end_group": _varint(9 << 3 | 4),
        "err_varint_overflow": b"\x0a" + b"\xff" * 9 + b"\x02",
        "err_wire_type_7": _varint(3 << 3 | 7),
    }
    dec = {}
    for name, b in cases.items():
        d = meta_decode_py(b)
        assert (d is None) == name.startswith("err_"), name
        dec[name] = {"hex": b.hex(), "expect": d}
    assert dec["bloom_split"]["expect"]["set_bits"] == [0, 2, 4] and dec["bloom_split"]["expect"]["m"] == 5
    assert dec["bloom_unpacked"]["expect"]["set_bits"] == [0, 2] and dec["bloom_unpacked"]["expect"]["m"] == 3
    assert dec["zone_last_wins"]["expect"]["min_hex"] == b"b".hex()
    assert dec["zone_last_wins"]["expect"]["max_hex"] == b"z".hex()
    assert dec["empty"]["expect"] == {"has_bloom": False, "m": 0, "set_bits": [], "has_zone": False,
                                      "min_hex": None, "max_hex": None}
    assert dec["unknown_fields"]["expect"]["set_bits"] == [0, 2]
    return {"encode": enc, "decode": dec}


# ---- SSTable data files: independent Python restatement ---------------------------

def b64_std_decode(v: bytes):
    """base64 0.21.7 STANDARD.decode: canonical padded base64 only. Python's
    strict decoder plus a re-encode check is an independent statement of
    "canonical": it rejects missing padding and non-zero trailing bits."""
    import base64
    import binascii
    try:
        d = base64.b64decode(v, validate=True)
    except (binascii.Error, ValueError):
        return None
    return d if base64.b64encode(d) == v else None


def table_get_py(data: bytes, key: bytes):
    lines = [ln for ln in data.split(b"\n") if ln]
    lo, hi = 0, len(lines)
    while lo < hi:
        mid = (lo + hi) // 2
        line = lines[mid]
        pos = line.find(b"\t")
        if pos < 0:
            break
        k = line[:pos]
        if k < key:
            lo = mid + 1
        elif k > key:
            hi = mid
        else:
            return mid, line[pos + 1:]
    return -1, None


def db_get_py(tables_newest_first, key: bytes):
    for t, data in enumerate(tables_newest_first):
        ln, enc = table_get_py(data, key)
        if ln < 0:
            continue
        v = b64_std_decode(enc)
        if v is None:
            continue  # Err(..) is skipped
        return t, v
    return -1, None


def sstable_fixtures() -> dict:
    import base64

    def file_of(entries):  # SsTable::create (stable sort by key)
        return b"".join(k + b"\t" + base64.b64encode(v) + b"\n" for k, v in sorted(entries, key=lambda e: e[0]))

    ts0 = (0).to_bytes(8, "big")
    files = {
        "sstable_test": file_of([(b"b", b"2"), (b"a", b"1"), (b"c", b"3")]),
        "lsm_flush_test": file_of([(b"k1", ts0 + b"v1"), (b"k2", ts0 + b"v2")]),
        "sstable_local_test": file_of([(b"k", b"v")]),
        "empty": b"",
        "only_newlines": b"\n\n\n",
        "empty_lines": b"\n\na\tMQ==\n\n\nb\tMg==\n\n",
        "no_trailing_newline": b"a\tMQ==\nb\tMg==",
        "line_without_tab": b"a\tMQ==\nbroken\nc\tMw==\n",
        "unsorted": b"b\tMg==\na\tMQ==\n",
        "bad_base64": b"a\tM===\nb\tMR==\nc\tMw\nd\tQUJD\ne\t\nf\t====\n",
        "empty_key_and_tabs": b"\tMQ==\na\tMg==\tx\n",
        "duplicates": b"a\tMQ==\na\tMg==\na\tMw==\n",
        "utf8": "é\tMQ==\n✓\tMg==\n".encode(),
    }
    probes = [b"", b"a", b"b", b"c", b"d", b"e", b"f", b"k", b"k1", b"k2", b"missing", b"broken",
              "é".encode(), "✓".encode()]
    out = {"files_hex": {k: v.hex() for k, v in files.items()}, "probes_hex": [p.hex() for p in probes],
           "search": {}}
    for name, data in files.items():
        res = []
        for p in probes:
            ln, enc = table_get_py(data, p)
            dec = b64_std_decode(enc) if enc is not None else None
            res.append({"line": ln, "value_hex": None if enc is None else enc.hex(),
                        "decoded_hex": None if dec is None else dec.hex()})
        out["search"][name] = res
    s = out["search"]
    assert s["sstable_test"][1]["decoded_hex"] == b"1".hex()          # tests/sstable_test.rs:13
    assert s["sstable_test"][2]["decoded_hex"] == b"2".hex()          # tests/sstable_test.rs:14
    assert s["lsm_flush_test"][8]["decoded_hex"] == (ts0 + b"v1").hex()
    assert s["lsm_flush_test"][10]["line"] == -1                     # tests/lsm_flush_test.rs:23
    assert s["line_without_tab"][3]["line"] == -1                    # mid hits "broken": search ends
    assert s["unsorted"][2]["line"] == -1 and s["unsorted"][1]["line"] == 1
    assert s["bad_base64"][1]["line"] == 0 and s["bad_base64"][1]["decoded_hex"] is None
    # newest-first walk over 4 tables with overlaps and a bad newest value
    stack = [b"a\tM===\nb\tYg==\n", files["sstable_test"], b"a\tb2xk\nz\tZW5k\n", files["empty_lines"]]
    out["get_tables_hex"] = [t.hex() for t in stack]
    out["get"] = [{"which": w, "value_hex": None if v is None else v.hex()}
                  for w, v in (db_get_py(stack, p) for p in probes)]
    assert out["get"][1] == {"which": 1, "value_hex": b"1".hex()}   # newest has bad base64 for "a"
    assert out["get"][2] == {"which": 0, "value_hex": b"b".hex()}
    return out


def create_fixtures() -> dict:
    """Python's sorted() is stable and orders bytes as Rust orders &str."""
    import base64

    def create_py(entries):
        return b"".join(k + b"\t" + base64.b64encode(v) + b"\n" for k, v in sorted(entries, key=lambda e: e[0]))

    rng = np.random.default_rng(21)
    cases = {
        "sstable_test": [(b"b", b"2"), (b"a", b"1"), (b"c", b"3")],
        "lsm_flush_test": [(b"k1", (0).to_bytes(8, "big") + b"v1"), (b"k2", (0).to_bytes(8, "big") + b"v2")],
        "empty": [],
        "duplicates_stable": [(b"k", b"first"), (b"a", b""), (b"k", b"second"), (b"a", b"x"), (b"k", b"third")],
        "value_lengths": [(bytes([97 + i]), bytes(range(i))) for i in range(12)],
        "binary_values": [(b"v%03d" % i, rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8).tobytes())
                          for i in range(40)][::-1],
        "shared_prefixes": [(k, k[::-1]) for k in [b"abcdefghijklmnopq", b"abcdefghijklmnop", b"abcdefghijklmnopa",
                                                   b"abcdefghijklmnoo", b"abcdefgh", b"abcdefgh\x00", b"", b"\xff",
                                                   b"abcdefghijklmnop\x00", "é".encode()]],
        "long_value": [(b"big", bytes(range(256)) * 8), (b"a", b"z" * 1001)],
    }
    out = {}
    for name, entries in cases.items():
        f = create_py(entries)
        out[name] = {"keys_hex": [k.hex() for k, _ in entries], "values_hex": [v.hex() for _, v in entries],
                     "file_hex": f.hex(), "len": len(f)}
    assert bytes.fromhex(out["sstable_test"]["file_hex"]) == b"a\tMQ==\nb\tMg==\nc\tMw==\n"  # sstable_test.rs:20-25
    assert bytes.fromhex(out["duplicates_stable"]["file_hex"]).startswith(b"a\t\na\teA==\nk\tZmlyc3Q=\n")
    return out


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


# ---- C4 / C5 (BASELINE configs 4 and 5) --------------------------

def c4_fixture() -> dict:
    """C4: 64 filters of m = 2^25, filter f built from key(200 + f, i < 2^18):
    the SHA-256 and popcount of each byte-per-bit array."""
    nf, m, kpf = 64, 1 << 25, 1 << 18
    out = {"nf": nf, "m": m, "keys_per_filter": kpf, "seed_base": 200, "bools_sha256": [], "packed_sha256": [],
           "popcount": []}
    for f in range(nf):
        bits = np_build(np_keys(200 + f, np.arange(kpf, dtype=np.uint64)), m)
        out["bools_sha256"].append(sha(bits))
        out["packed_sha256"].append(sha(np.packbits(bits, bitorder="little")))
        out["popcount"].append(int(bits.sum()))
    return out


def c5_fixture() -> dict:
    """C5: 256 filters of m = 2^26 ("L0-L4"), filter f from key(1000 + f, i < 2^19);
    10M lookups (even i: key(1000 + j mod 256, (j div 256) mod 2^19), j = i/2;
    odd i: key(9999, i)). The hit map [256][156250] is recorded per 32-filter
    rank slice (rank r of 8 holds filters [32r, 32r+32)), as SHA-256 of the
    little-endian uint64 rows, plus per-filter hit counts."""
    nf, m, kpf, nl, per = 256, 1 << 26, 1 << 19, 10_000_000, 32
    lk = lookups(nl, nf, kpf, 1000, 9999)
    h1, h2 = np_raw_hashes(lk)
    a = (h1 % np.uint64(m)).astype(np.int64)
    b = (h2 % np.uint64(m)).astype(np.int64)
    del h1, h2
    slices, counts = [], []
    rows = []
    for f in range(nf):
        bits = np_build(np_keys(1000 + f, np.arange(kpf, dtype=np.uint64)), m)
        hit = (bits[a] & bits[b]).astype(bool)
        counts.append(int(hit.sum()))
        rows.append(_pack64(hit).astype("<u8"))
        if len(rows) == per:
            slices.append(sha(np.stack(rows)))
            rows = []
    return {"nf": nf, "m": m, "keys_per_filter": kpf, "n_lookups": nl, "seed_base": 1000, "absent_seed": 9999,
            "lookups_sha256": sha(lk), "filters_per_rank": per, "rank_slice_hits_sha256": slices,
            "hits_per_filter": counts, "hits_popcount": int(sum(counts))}


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "--only":
        # regenerate only the named large-config sections into the existing file
        path = os.path.join(HERE, "golden.json")
        with open(path) as fh:
            g = json.load(fh)
        for name in sys.argv[2:]:
            g[name] = {"c4": c4_fixture, "c5": c5_fixture}[name]()
            print("regenerated", name)
        with open(path, "w") as fh:
            json.dump(g, fh, indent=1, sort_keys=True)
    else:
        main()
