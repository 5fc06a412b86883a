"""GPU parity for SURVEY.md §8f row 2: the SSTable `.meta` codec
(TableMeta{bloom, zone_map}) through the C ABI, against the golden fixtures
and the C oracle. Byte-exact on encode, field-exact on decode.

Reference: src/sstable.rs:31-37 (TableMeta), 74-81 (encode in create),
96-108 (decode in load, with BloomFilter::new(1024) / ZoneMap::default()
fallbacks), tests/sstable_local_test.rs:12-14 (round trip).
"""
import hashlib

import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def test_meta_encode_golden(gpu, golden):
    for name, e in golden["meta"]["encode"].items():
        keys = [bytes.fromhex(k) for k in e["keys_hex"]]
        b = gpu.BloomFilter(1024)
        z = gpu.ZoneMap()
        for k in keys:
            b.insert(k)
            z.update(k)
        data = gpu.TableMeta(b, z).encode()
        assert len(data) == e["len"] and hashlib.sha256(data).hexdigest() == e["sha256"], name
        # tests/sstable_local_test.rs:12-14: load() gives back the same filter and zone
        lb, lz = gpu.TableMeta.load(data)
        assert lb.to_bytes() == b.to_bytes(), name
        assert (lz.min, lz.max) == (z.min, z.max), name


def test_meta_decode_golden(gpu, golden):
    for name, c in golden["meta"]["decode"].items():
        data = bytes.fromhex(c["hex"])
        exp = c["expect"]
        if exp is None:
            with pytest.raises(ValueError):
                gpu.TableMeta.decode(data)
            continue
        t = gpu.TableMeta.decode(data)
        assert (t.bloom is not None) == exp["has_bloom"], name
        if t.bloom is not None:
            assert t.bloom.m == exp["m"], name
            assert list(np.flatnonzero(t.bloom.bools())) == exp["set_bits"], name
        assert (t.zone_map is not None) == exp["has_zone"], name
        if t.zone_map is not None:
            want = tuple(None if h is None else bytes.fromhex(h) for h in (exp["min_hex"], exp["max_hex"]))
            assert (t.zone_map.min, t.zone_map.max) == want, name


def test_meta_load_defaults(gpu):
    # src/sstable.rs:99-103: a meta without fields -> BloomFilter::new(1024), ZoneMap::default()
    b, z = gpu.TableMeta.load(b"")
    assert b.m == 1024 and not b.bools().any()
    assert z.min is None and z.max is None
    t = gpu.TableMeta.decode(b"")
    assert t.bloom is None and t.zone_map is None


@pytest.mark.parametrize("m", [1, 1000, (1 << 20) + 7, 1 << 24])
def test_meta_roundtrip_vs_oracle(gpu, m):
    keys = workload.key_range(41, 200_000)
    b = gpu.BloomFilter(m)
    b.insert_batch(keys)
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    lo, hi = bytes(keys[int(np.argmin(keys[:, 0]))]), b"\x7f" * 3
    data = gpu.TableMeta(b, gpu.ZoneMap(lo, hi)).encode()
    assert data == oracle.meta_encode(o, oracle.OracleZone(lo, hi))
    t = gpu.TableMeta.decode(data)
    assert np.array_equal(t.bloom.bools(), o.bools())
    assert (t.zone_map.min, t.zone_map.max) == (lo, hi)
    # only a filter / only a zone
    assert gpu.TableMeta(b, None).encode() == oracle.meta_encode(o, None)
    assert gpu.TableMeta(None, gpu.ZoneMap(lo, None)).encode() == oracle.meta_encode(None, oracle.OracleZone(lo, None))


def test_meta_pinned_to_the_protobuf_wire_format(gpu):
    """The device codec's TableMeta bytes against bytes written from the
    protobuf encoding spec (tests/test_oracle.py _meta_wire), and decoded
    back field by field."""
    from tests.test_oracle import _meta_wire, _wire
    for m, lo, hi in [(10, b"apple", b"pear"), (200, b"a" * 130, b"z"), (1, None, None), (64, b"k", None)]:
        rng = np.random.default_rng(m)
        bits = [int(x) for x in rng.integers(0, 2, m)]
        want = _meta_wire(bits, lo, hi)
        b = gpu.BloomFilter.from_bytes(_wire(bits))
        assert gpu.TableMeta(b, gpu.ZoneMap(lo, hi)).encode() == want, m
        t = gpu.TableMeta.decode(want)
        assert list(t.bloom.bools()) == bits and (t.zone_map.min, t.zone_map.max) == (lo, hi), m


def test_meta_encode_into_device_buffer(gpu):
    import ctypes

    import torch
    from lsmt_amd import _lib
    b = gpu.BloomFilter(100_003)
    b.insert_batch(workload.key_range(42, 5000))
    host = gpu.TableMeta(b, gpu.ZoneMap(b"a", b"b")).encode()
    dev = torch.zeros(len(host), dtype=torch.uint8, device="cuda")
    lb, hb = ctypes.create_string_buffer(b"a"), ctypes.create_string_buffer(b"b")
    zb = _lib.ZoneBounds(ctypes.cast(lb, ctypes.c_void_p), 1, 1, ctypes.cast(hb, ctypes.c_void_p), 1, 1)
    n = ctypes.c_uint64()
    rc = _lib.load().cb_meta_encode(b.handle, ctypes.byref(zb), dev.data_ptr(), len(host), ctypes.byref(n))
    assert rc == 0 and n.value == len(host)
    torch.cuda.synchronize()
    assert dev.cpu().numpy().tobytes() == host


def test_set_load_meta_restart_path(gpu, golden):
    # every table's .meta (written by the oracle, i.e. independently of the
    # product encoder) loaded straight into a FilterSet slot; the gated probe
    # then reproduces the zone fixture
    g = golden["zone"]
    tables = workload.zone_tables(g["tables"], g["seed_base"], g["keys_per_seed"])
    lk = workload.zone_lookups(tables, g["n_lookups"])
    s = gpu.FilterSet(g["m"])
    for i, t in enumerate(tables):
        o = oracle.OracleFilter(g["m"])
        o.insert_fixed(t)
        lo, hi = (bytes.fromhex(h) for h in g["zones_hex"][i])
        s.load_meta(i, oracle.meta_encode(o, oracle.OracleZone(lo, hi)))
    assert hashlib.sha256(s.probe(lk, gated=True).astype("<u8").tobytes()).hexdigest() == g["gated_sha256"]
    assert hashlib.sha256(s.probe(lk).astype("<u8").tobytes()).hexdigest() == g["hits_sha256"]
    before = s.probe(lk, gated=True)
    with pytest.raises(ValueError):
        s.load_meta(0, b"\x0a\x05\x0a\x03\x01")  # truncated: the slot is left untouched
    other = oracle.OracleFilter(1024)
    with pytest.raises(Exception):
        s.load_meta(0, oracle.meta_encode(other, None))  # m differs from the set's
    assert np.array_equal(s.probe(lk, gated=True), before)
