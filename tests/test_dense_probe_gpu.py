"""The dense FilterSet probe (lsmt_amd/csrc/densefs.hip: keys partitioned by
set region, each 64 KiB region of the set staged in LDS once) against the CPU
oracle, bit for bit.

Reference semantics: BloomFilter::may_contain (/root/reference/src/bloom.rs:
26-51) for every table of Database::get's fan-out (src/lib.rs:129-134); the
set answers all slots of a key with set[a] & set[b]. The dense path is chosen
by density (>= 2 keys per 128-B line of the set: the C5 shape); here it is
forced on (cb_set_dense(1)) at sizes the oracle finishes in seconds, and the
auto choice is checked at the BASELINE C5 rank-slice shape against its
golden SHA-256 (tests/golden/make_golden.py's numpy restatement).
"""
import hashlib

import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu

DENSE_PATH = 6
C = 12288  # keys per partition block (densefs.hip kDenseC)


@pytest.fixture
def dense(gpu):
    gpu.set_dense(1)
    yield gpu
    gpu.set_dense(0)


def build(gpu, m, nf, kpf, seed):
    filters, refs = [], []
    for f in range(nf):
        keys = workload.key_range(seed + f, kpf)
        g = gpu.BloomFilter(m)
        g.insert_batch(keys)
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        filters.append(g)
        refs.append(o)
    return filters, refs


@pytest.mark.parametrize("width,nf", [(32, 1), (32, 5), (32, 32), (64, 37), (64, 64)])
@pytest.mark.parametrize("n", [1, 63, 64, 4095, 4097, C - 1, C, C + 1, 50_001])
def test_dense_matches_oracle(dense, width, nf, n):
    m = 1 << 20
    filters, refs = build(dense, m, nf, 6000, 700)
    s = dense.FilterSet.from_filters(filters, width=width)
    look = workload.probe_lookups(n, nf, 6000, seed_base=700, absent_seed=995)
    got = s.probe(look)
    assert dense.last_path() == DENSE_PATH
    assert np.array_equal(got, oracle.probe_fixed(refs, look))


@pytest.mark.parametrize("m", [100_003, (1 << 21) + 3, 1 << 24, (1 << 26) - 5])
def test_dense_generic_m_and_region_tails(dense, m):
    # m not a multiple of the region (the last region's tail is partial) and
    # the exact 64-bit fastmod positions (MOD_GENERIC)
    filters, refs = build(dense, m, 7, 9000, 710)
    s = dense.FilterSet.from_filters(filters, width=32)
    look = workload.probe_lookups(120_000, 7, 9000, seed_base=710, absent_seed=994)
    got = s.probe(look)
    assert dense.last_path() == DENSE_PATH
    assert np.array_equal(got, oracle.probe_fixed(refs, look))


def test_dense_var_and_unaligned_keys(dense):
    m = (1 << 20) + 17
    filters, refs = build(dense, m, 6, 5000, 720)
    s = dense.FilterSet.from_filters(filters, width=32)
    rng = np.random.default_rng(12)
    data, offs = workload.var_keys(rng, 30_000, max_len=40)
    got = s.probe(dense.KeyBatch(n=30_000, data=data, offsets=offs))
    assert dense.last_path() == DENSE_PATH
    assert np.array_equal(got, oracle.probe_var(refs, data, offs))
    # fixed-length keys of other lengths (KEY_FIXED)
    for kl in (0, 7, 24):
        keys = rng.integers(0, 256, size=(9000, kl), dtype=np.uint8)
        exp = oracle.probe_fixed(refs, keys) if kl else oracle.probe_var(refs, np.zeros(1, np.uint8),
                                                                        np.zeros(9001, np.uint64))
        assert np.array_equal(s.probe(keys), exp), kl


def test_dense_duplicate_heavy_batch(dense):
    # every key the same (one region takes every entry: the probe's rounds
    # loop over 200k entries in one workgroup), plus a present key and an
    # absent one repeated in runs longer than a partition block
    m = 1 << 22
    filters, refs = build(dense, m, 9, 20_000, 730)
    s = dense.FilterSet.from_filters(filters, width=32)
    one = workload.key_range(733, 1)
    look = np.concatenate([np.repeat(one, 200_000, axis=0), np.repeat(workload.key_range(999_999, 1), 9000, axis=0),
                           workload.key_range(731, 3000)])
    got = s.probe(look)
    assert dense.last_path() == DENSE_PATH
    assert np.array_equal(got, oracle.probe_fixed(refs, look))


def test_dense_device_buffers_and_padding_words(dense):
    # device keys; a hit buffer with rows past the set's used slots, all
    # pre-filled with a pattern: the probe writes exactly the used rows'
    # ceil(n/64) words (its partition pass zeroes them, the probe ORs bits in)
    import torch
    m = 1 << 21
    filters, refs = build(dense, m, 11, 7000, 740)
    s = dense.FilterSet.from_filters(filters, width=32)
    n = 3 * C + 100
    look = workload.probe_lookups(n, 11, 7000, seed_base=740, absent_seed=993)
    nw = (n + 63) // 64
    out = torch.full((13, nw), -1, dtype=torch.int64, device="cuda")
    s.probe(dense.DeviceKeys(torch.from_numpy(look).cuda()), out=out)
    got = out.cpu().numpy().view(np.uint64)
    assert dense.last_path() == DENSE_PATH
    assert np.array_equal(got[:11], oracle.probe_fixed(refs, look))
    assert (got[11:] == np.uint64(0xFFFFFFFFFFFFFFFF)).all()


def test_dense_chunks(dense):
    # more keys than one launch pair takes (2048 partition blocks of C keys
    # = 25,165,824): two chunks, the second's key indices offset
    import torch
    m = 1 << 20
    filters, refs = build(dense, m, 3, 4000, 750)
    s = dense.FilterSet.from_filters(filters, width=32)
    n = 2048 * C + 70_001
    look = workload.probe_lookups(n, 3, 4000, seed_base=750, absent_seed=992)
    out = torch.zeros((3, (n + 63) // 64), dtype=torch.int64, device="cuda")
    s.probe(dense.DeviceKeys(torch.from_numpy(look).cuda()), out=out)
    assert dense.last_path() == DENSE_PATH
    exp = oracle.probe_fixed(refs, look, threads=8)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), exp)


def test_auto_choice_by_density(gpu):
    # C3's density (0.5 keys per set line) keeps k_set_probe; 4x the lines'
    # worth of keys takes the dense probe; -1 turns it off
    m = 1 << 20  # a 4 MiB set of 32768 lines
    filters, refs = build(gpu, m, 4, 3000, 760)
    s = gpu.FilterSet.from_filters(filters, width=32)
    sparse_look = workload.probe_lookups(16_384, 4, 3000, seed_base=760, absent_seed=991)
    dense_look = workload.probe_lookups(4 * 32768, 4, 3000, seed_base=760, absent_seed=991)
    assert np.array_equal(s.probe(sparse_look), oracle.probe_fixed(refs, sparse_look))
    assert gpu.last_path() == 3
    assert np.array_equal(s.probe(dense_look), oracle.probe_fixed(refs, dense_look))
    assert gpu.last_path() == DENSE_PATH
    gpu.set_dense(-1)
    try:
        assert np.array_equal(s.probe(dense_look), oracle.probe_fixed(refs, dense_look))
        assert gpu.last_path() == 3
    finally:
        gpu.set_dense(0)


def test_dense_gated_falls_back(dense):
    # the zone gate is not part of the dense path: a gated probe keeps k_set_probe
    m = 1 << 20
    filters, refs = build(dense, m, 4, 3000, 770)
    s = dense.FilterSet.from_filters(filters, width=32)
    for f in range(4):
        s.zone_from_keys(f, workload.key_range(770 + f, 3000))
    look = workload.probe_lookups(40_000, 4, 3000, seed_base=770, absent_seed=990)
    s.probe(look, gated=True)
    assert dense.last_path() == 3


@pytest.mark.slow
def test_dense_c5_rank_slice_golden(gpu, golden):
    # BASELINE C5, rank 0's slice: 10M lookups x filters 0..31 of m = 2^26;
    # the auto choice takes the dense probe at this density
    import torch
    g = golden["c5"]
    F, m, kpf, n, nf = 32, 1 << 26, 1 << 19, 10_000_000, 256
    filters = []
    for f in range(F):
        b = gpu.BloomFilter(m)
        b.insert_batch(gpu.DeviceKeys(torch.from_numpy(workload.c5_filter_keys(f, kpf)).cuda()))
        filters.append(b)
    s = gpu.FilterSet.from_filters(filters, width=32)
    look = workload.c5_lookups(n, nf, kpf)
    out = torch.zeros((F, (n + 63) // 64), dtype=torch.int64, device="cuda")
    s.probe(gpu.DeviceKeys(torch.from_numpy(look).cuda()), out=out)
    assert gpu.last_path() == DENSE_PATH
    got = out.cpu().numpy().view(np.uint64).astype("<u8")
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == g["rank_slice_hits_sha256"][0]
