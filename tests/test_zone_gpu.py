"""GPU parity for SURVEY.md §8f row 1: the zone-map gate fused into the
FilterSet probe, and the device ZoneMap::update reduction. Bit-exact against
the C oracle (oracle.probe_gated / OracleZone) and the golden fixtures.

Reference semantics: src/zonemap.rs:21-42 (update / contains),
src/sstable.rs:62-65 (zone built next to the filter), src/sstable.rs:138
(the gate `zone_map.contains(key) && bloom.may_contain(key)`).
"""
import hashlib

import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def var_batch(gpu, keys):
    offs = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    data = np.frombuffer(b"".join(keys), np.uint8).copy() if offs[-1] else np.zeros(1, np.uint8)
    return gpu.KeyBatch(n=len(keys), data=data, offsets=offs), data, offs


def bit(hits, f, i):
    return bool(int(hits[f, i >> 6]) >> (i & 63) & 1)


def test_zone_scenarios(gpu, golden):
    # tests/sstable_test.rs, lsm_flush_test.rs, sstable_local_test.rs shapes
    for name, s in golden["zone"]["scenarios"].items():
        ins = [bytes.fromhex(k) for k in s["insert_hex"]]
        probes = [bytes.fromhex(k) for k in s["probe_hex"]]
        f = gpu.BloomFilter(s["m"])
        for k in ins:
            f.insert(k)
        fs = gpu.FilterSet(s["m"], width=32)
        fs.assign(0, f)
        fs.zone_from_keys(0, var_batch(gpu, ins)[0])
        z = fs.zone(0)
        assert (z.min, z.max) == (bytes.fromhex(s["min_hex"]), bytes.fromhex(s["max_hex"])), name
        assert [z.contains(k) for k in probes] == s["zone"], name  # host mirror agrees
        kb = var_batch(gpu, probes)[0]
        g = fs.probe(kb, gated=True)
        assert [bit(g, 0, i) for i in range(len(probes))] == s["gate"], name
        u = fs.probe(kb)
        assert [bit(u, 0, i) for i in range(len(probes))] == [f.may_contain(k) for k in probes], name


@pytest.mark.parametrize("width", [32, 64])
def test_zone_range_tables_golden(gpu, golden, width):
    g = golden["zone"]
    tables = workload.zone_tables(g["tables"], g["seed_base"], g["keys_per_seed"])
    lk = workload.zone_lookups(tables, g["n_lookups"])
    assert sha(lk) == g["lookups_sha256"]
    filters = []
    for t in tables:
        b = gpu.BloomFilter(g["m"])
        b.insert_batch(t)
        filters.append(b)
    s = gpu.FilterSet.from_filters(filters, width=width)
    for i, t in enumerate(tables):
        s.zone_from_keys(i, t)  # device ZoneMap::update over the table's keys
        z = s.zone(i)
        assert (z.min.hex(), z.max.hex()) == tuple(g["zones_hex"][i])
    assert sha(s.probe(lk).astype("<u8")) == g["hits_sha256"]
    gated = s.probe(lk, gated=True)
    assert sha(gated.astype("<u8")) == g["gated_sha256"]
    # the same zones given explicitly (TableMeta load path)
    s2 = gpu.FilterSet.from_filters(filters, width=width)
    for i, (lo, hi) in enumerate(g["zones_hex"]):
        s2.set_zone(i, (bytes.fromhex(lo), bytes.fromhex(hi)))
    assert sha(s2.probe(lk, gated=True).astype("<u8")) == g["gated_sha256"]


@pytest.mark.parametrize("m", [1000, (1 << 20) + 3, 1 << 22])
def test_zone_gate_var_keys_matches_oracle(gpu, m):
    rng = np.random.default_rng(31)
    nt = 40
    filters, refs, zones, ozones = [], [], [], []
    for f in range(nt):
        data, offs = workload.var_keys(rng, 3000, max_len=12)
        b = gpu.BloomFilter(m)
        b.insert_batch(gpu.KeyBatch(n=3000, data=data, offsets=offs))
        o = oracle.OracleFilter(m)
        o.insert_var(data, offs)
        filters.append(b)
        refs.append(o)
        keys = [data[offs[i]:offs[i + 1]].tobytes() for i in range(0, 3000, 97)]
        lo, hi = sorted(keys[:2])
        kind = f % 5
        if kind == 1:
            lo = lo[:1]  # a prefix bound
        elif kind == 2:
            lo = None  # half-open: accepts everything (zonemap.rs:40)
        elif kind == 3:
            lo, hi = b"", b"\xff"
        elif kind == 4:
            hi = lo  # single-key zone
        zones.append((lo, hi))
        ozones.append(oracle.OracleZone(lo, hi))
    s = gpu.FilterSet(m, width=64)
    s.assign_all(filters)
    for i, z in enumerate(zones):
        s.set_zone(i, z)
    data, offs = workload.var_keys(rng, 60_000, max_len=12)
    # mix in the exact bounds and their neighbours
    extra = []
    for lo, hi in zones:
        for b in (lo, hi):
            if b is not None:
                extra += [b, b + b"\x00", b[:-1]]
    keys = [data[offs[i]:offs[i + 1]].tobytes() for i in range(60_000)] + extra
    kb, d2, o2 = var_batch(gpu, keys)
    exp = oracle.probe_gated(refs, ozones, d2, o2)
    assert np.array_equal(s.probe(kb, gated=True), exp)
    assert np.array_equal(s.probe(kb), oracle.probe_var(refs, d2, o2))


def test_zone_reset_on_reassign(gpu):
    m = 1 << 16
    t = workload.zone_tables(2, 400, 20_000)
    fa, fb = gpu.BloomFilter(m), gpu.BloomFilter(m)
    fa.insert_batch(t[0])
    fb.insert_batch(t[1])
    s = gpu.FilterSet(m)
    s.assign(0, fa)
    s.zone_from_keys(0, t[0])
    lk = workload.zone_lookups(t, 20_000)
    assert not np.array_equal(s.probe(lk, gated=True), s.probe(lk))
    s.assign(0, fb)  # another table's filter: the old zone must not gate it
    z = s.zone(0)
    assert z.min is None and z.max is None
    assert np.array_equal(s.probe(lk, gated=True), s.probe(lk))
    s.zone_from_keys(0, t[1])
    s.clear_slot(0)
    assert s.zone(0).min is None


def test_zone_from_keys_merges(gpu):
    # ZoneMap::update keeps widening across batches
    s = gpu.FilterSet(1024)
    s.zone_from_keys(3, ["m", "n"])
    s.zone_from_keys(3, ["b", "c"])
    s.zone_from_keys(3, [])  # no keys: unchanged
    z = s.zone(3)
    assert (z.min, z.max) == (b"b", b"n")
    s.zone_from_keys(3, ["z", "a\x00"])
    assert (s.zone(3).min, s.zone(3).max) == (b"a\x00", b"z")


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 70_001, 1 << 20])
def test_zone_bounds_fixed(gpu, n):
    k = workload.key_range(77, n)
    k[n // 3] = k[n // 2]  # a duplicate pair: the first index wins on ties
    lo, hi = gpu.zone_bounds(k)
    # equal-length keys: byte order == order of the big-endian (hi, lo) u64 pair
    w = k.view(">u8").reshape(n, 2)
    idx = np.arange(n)
    exp_lo = np.lexsort((idx, w[:, 1], w[:, 0]))[0]
    exp_hi = np.lexsort((idx, ~w[:, 1], ~w[:, 0]))[0]
    assert (lo, hi) == (exp_lo, exp_hi)


def test_zone_bounds_var_and_empty(gpu):
    assert gpu.zone_bounds(np.zeros((0, 16), np.uint8)) is None
    keys = [b"k10", b"k1", b"k", b"", b"k2", b"k", b"\xff", b"\xff", b"j\xff\xff"]
    kb = var_batch(gpu, keys)[0]
    assert gpu.zone_bounds(kb) == (3, 6)
    rng = np.random.default_rng(4)
    data, offs = workload.var_keys(rng, 200_000, max_len=6)
    rows = [data[offs[i]:offs[i + 1]].tobytes() for i in range(200_000)]
    lo, hi = gpu.zone_bounds(gpu.KeyBatch(n=200_000, data=data, offsets=offs))
    assert rows[lo] == min(rows) and lo == rows.index(min(rows))
    assert rows[hi] == max(rows) and hi == rows.index(max(rows))


def test_zone_gate_device_resident(gpu):
    import torch
    g = workload.zone_tables(4, 500, 30_000)
    m = (1 << 20) + 11
    fs = []
    for t in g:
        b = gpu.BloomFilter(m)
        b.insert_batch(t)
        fs.append(b)
    s = gpu.FilterSet.from_filters(fs)
    for i, t in enumerate(g):
        s.zone_from_keys(i, torch.from_numpy(t).cuda())
    lk = workload.zone_lookups(g, 100_000)
    host = s.probe(lk, gated=True)
    dk = torch.from_numpy(lk).cuda()
    out = torch.zeros((4, (len(lk) + 63) // 64), dtype=torch.int64, device="cuda")
    s.probe(dk, out=out, gated=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), host)
    refs, zs = [], []
    for t in g:
        o = oracle.OracleFilter(m)
        o.insert_fixed(t)
        refs.append(o)
        zs.append(oracle.OracleZone(bytes(min(bytes(r) for r in t)), bytes(max(bytes(r) for r in t))))
    d = np.ascontiguousarray(lk.reshape(-1))
    offs = np.arange(0, 16 * (len(lk) + 1), 16, dtype=np.uint64)
    assert np.array_equal(host, oracle.probe_gated(refs, zs, d, offs))


@pytest.mark.parametrize("width", [32, 64])
def test_zone_gate_fixed16_bound_lengths(gpu, width):
    # 16-byte keys take the LDS word-compare path: bounds of every length
    # class (empty, inside one word, word-aligned, 16, longer than the key),
    # cut from the keys themselves so equal prefixes are common
    rng = np.random.default_rng(17)
    alpha = np.frombuffer(b"ab", np.uint8)
    m = 4099
    nt = width
    keys = [alpha[rng.integers(0, 2, (3000, 16))] for _ in range(nt)]
    filters, refs, zones = [], [], []
    lens = [0, 1, 3, 4, 5, 8, 11, 15, 16, 17, 20]
    for f in range(nt):
        b = gpu.BloomFilter(m)
        b.insert_batch(keys[f])
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys[f])
        filters.append(b)
        refs.append(o)
        r = [bytes(x) for x in keys[f][:2]]
        lo = r[0][: lens[f % len(lens)]]
        hi = (r[1] + b"ab")[: lens[(f * 7 + 3) % len(lens)]]
        if lo > hi:
            lo, hi = hi, lo
        zones.append((lo, hi))
    s = gpu.FilterSet(m, width=width)
    s.assign_all(filters)
    for i, z in enumerate(zones):
        s.set_zone(i, z)
    look = alpha[rng.integers(0, 2, (50_000, 16))]
    look[: len(zones)] = [np.frombuffer((z[0] + b"a" * 16)[:16], np.uint8) for z in zones]
    got = s.probe(look, gated=True)
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    exp = oracle.probe_gated(refs, [oracle.OracleZone(lo, hi) for lo, hi in zones], d, offs)
    assert np.array_equal(got, exp)
    assert int(np.unpackbits(exp.view(np.uint8)).sum()) > 0


def test_zone_update_waits_for_gated_probes_on_other_streams(gpu):
    """A zone update while gated probes (and the fused read path's gate) are
    still queued on other streams: the update waits for those streams' last
    readers (per-stream events, no device-wide sync), so the queued probes see
    the old zones and the probes after it the new ones, bit-exact."""
    import torch
    m = 1 << 22
    nt = 6
    g = workload.zone_tables(nt, 4000, 60_000)
    fs, refs = [], []
    for t in g:
        b = gpu.BloomFilter(m)
        b.insert_batch(t)
        fs.append(b)
        o = oracle.OracleFilter(m)
        o.insert_fixed(t)
        refs.append(o)
    s = gpu.FilterSet.from_filters(fs)
    full = [(bytes(min(bytes(r) for r in t)), bytes(max(bytes(r) for r in t))) for t in g]
    narrow = []
    for t in g:
        srt = sorted(bytes(r) for r in t)
        narrow.append((srt[len(srt) // 3], srt[2 * len(srt) // 3]))
    for i, z in enumerate(full):
        s.set_zone(i, z)
    lk = workload.zone_lookups(g, 1 << 20)
    dk = torch.from_numpy(lk).cuda()
    d = np.ascontiguousarray(lk.reshape(-1))
    offs = np.arange(0, 16 * (len(lk) + 1), 16, dtype=np.uint64)
    exp_full = oracle.probe_gated(refs, [oracle.OracleZone(lo, hi) for lo, hi in full], d, offs)
    exp_narrow = oracle.probe_gated(refs, [oracle.OracleZone(lo, hi) for lo, hi in narrow], d, offs)
    assert not np.array_equal(exp_full, exp_narrow)
    words = (len(lk) + 63) // 64
    streams = [torch.cuda.Stream() for _ in range(3)]
    before = [torch.zeros((nt, words), dtype=torch.int64, device="cuda") for _ in range(3 * 4)]
    for i, out in enumerate(before):  # queue a dozen gated probes on three other streams
        s.probe(gpu.DeviceKeys(dk), out=out, stream=streams[i % 3], gated=True)
    for i, z in enumerate(narrow):  # update while they are queued or running
        s.set_zone(i, z)
    after = s.probe(lk, gated=True)
    torch.cuda.synchronize()
    for out in before:
        assert np.array_equal(out.cpu().numpy().view(np.uint64), exp_full)
    assert np.array_equal(after, exp_narrow)
