"""BASELINE configs C1, C4 and C5 at full size through the HIP path (C ABI),
bit-exact against the golden SHA-256s of tests/golden/make_golden.py (the
independent numpy restatement of src/bloom.rs:26-51, itself checked against
the C oracle in tests/test_oracle.py).

- C1: 10k keys into m = 2^17 and m = 100003; the false-positive hit set of
  100k absent keys (the reference's tests/bloom_test.rs-style check).
- C4: 64 concurrent flush builds, 2^18 keys each into m = 2^25, through
  cb_filter_insert_fixed_many (SsTable::create's build, src/sstable.rs:62-65,
  64 flushes at once).
- C5: one rank's slice of the read fan-out (src/lib.rs:129-134 over 256
  tables): 32 filters of m = 2^26 against 10M lookups, through the FilterSet
  probe and the per-filter tiled probe.
"""
import hashlib

import numpy as np
import pytest

from lsmt_amd import workload

pytestmark = pytest.mark.gpu

DIRECT, TILED, AUTO = 1, 2, 0


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("path", [DIRECT, TILED], ids=["direct", "tiled"])
@pytest.mark.parametrize("m", ["131072", "100003"])
def test_c1_bits_and_fp_hits(gpu, golden, m, path):
    g = golden["c1"][m]
    gpu.set_path(path)
    try:
        b = gpu.BloomFilter(int(m))
        b.insert_batch(workload.key_range(1, g["n"]))
        bits = b.bools()
        assert sha(bits) == g["bools_sha256"] and int(bits.sum()) == g["popcount"]
        present = b.may_contain_batch(workload.key_range(1, g["n"]))
        assert present.all()  # tests/bloom_test.rs:5-7, at C1 scale
        hits = gpu.probe([b], workload.key_range(2, 100_000))
    finally:
        gpu.set_path(AUTO)
    assert sha(hits[0].astype("<u8")) == g["fp_hits_sha256"]
    assert int(np.unpackbits(hits[0].view(np.uint8)).sum()) == g["fp_absent_100k"]


@pytest.mark.parametrize("path", [AUTO, DIRECT, TILED], ids=["auto", "direct", "tiled"])
def test_c4_concurrent_builds_full(gpu, golden, path):
    g = golden["c4"]
    import torch
    keys = [torch.from_numpy(workload.c4_filter_keys(f, g["keys_per_filter"])).cuda() for f in range(g["nf"])]
    fs = [gpu.BloomFilter(g["m"]) for _ in range(g["nf"])]
    gpu.set_path(path)
    try:
        gpu.insert_many(fs, [gpu.DeviceKeys(k) for k in keys])
    finally:
        gpu.set_path(AUTO)
    for f, b in enumerate(fs):
        words = b.packed()
        assert sha(words.view(np.uint8)) == g["packed_sha256"][f], f
        assert int(np.unpackbits(words.view(np.uint8)).sum()) == g["popcount"][f], f
    # the bench's step: clear, then rebuild all 64 in one call; same bits again
    for b in fs:
        b.clear()
    gpu.insert_many(fs, [gpu.DeviceKeys(k) for k in keys])
    assert [sha(b.packed().view(np.uint8)) for b in fs] == g["packed_sha256"]


@pytest.fixture(scope="module")
def c5_lookups_dev(golden):
    import torch
    g = golden["c5"]
    look = workload.c5_lookups(g["n_lookups"], g["nf"], g["keys_per_filter"])
    assert sha(look) == g["lookups_sha256"]
    return torch.from_numpy(look).cuda()


@pytest.mark.parametrize("rank", [0, 7])
def test_c5_rank_slice(gpu, golden, c5_lookups_dev, rank):
    import torch
    g = golden["c5"]
    per, m, kpf = g["filters_per_rank"], g["m"], g["keys_per_filter"]
    filters = []
    for f in range(rank * per, (rank + 1) * per):
        b = gpu.BloomFilter(m)
        b.insert_batch(gpu.DeviceKeys(torch.from_numpy(workload.c5_filter_keys(f, kpf)).cuda()))
        filters.append(b)
    n = g["n_lookups"]
    words = (n + 63) // 64
    keys = gpu.DeviceKeys(c5_lookups_dev)
    out = torch.zeros((per, words), dtype=torch.int64, device="cuda")
    # FilterSet probe (the bench's headline path)
    s = gpu.FilterSet.from_filters(filters)
    s.probe(keys, out=out)
    hits = out.cpu().numpy().view(np.uint64)
    assert sha(hits.astype("<u8")) == g["rank_slice_hits_sha256"][rank]
    counts = np.unpackbits(hits.view(np.uint8), axis=1).sum(axis=1)
    assert counts.tolist() == g["hits_per_filter"][rank * per:(rank + 1) * per]
    # per-filter tiled probe (cb_probe_fixed)
    out.zero_()
    gpu.probe(filters, keys, out=out)
    assert sha(out.cpu().numpy().view(np.uint64).astype("<u8")) == g["rank_slice_hits_sha256"][rank]


def test_c5_all_ranks_exchanged(gpu, golden, c5_lookups_dev):
    """C5 end to end on one GPU: eight 'ranks' (FilterSets of 32 filters of
    m = 2^26, 256 tables in all) each probe the 10M lookups writing their
    sparse exchange pack (cb_set_probe_pack_fixed, the probe of
    cb_set_probe_allgather_fixed), the eight packs are expanded into the
    [256][156250] map the all-gather would leave on every rank
    (cb_hits_expand_set), and every rank's rows match the golden SHA-256s
    (src/lib.rs:129-134 over 256 tables)."""
    import torch

    from lsmt_amd.shard import shard_range, sparse_cap
    g = golden["c5"]
    per, m, kpf, n, nf = g["filters_per_rank"], g["m"], g["keys_per_filter"], g["n_lookups"], g["nf"]
    world = nf // per
    words = (n + 63) // 64
    cap = sparse_cap(n, nf, world)
    stride = gpu.FilterSet.pack_words(n, cap)
    packs = torch.zeros(world * stride, dtype=torch.int32, device="cuda")
    hits = torch.empty((per, words), dtype=torch.int64, device="cuda")
    sets = []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        s = gpu.FilterSet(m, 32)
        for slot, f in enumerate(range(lo, hi)):
            b = gpu.BloomFilter(m)
            b.insert_batch(gpu.DeviceKeys(torch.from_numpy(workload.c5_filter_keys(f, kpf)).cuda()))
            s.assign(slot, b)
            del b
        s.probe_pack(c5_lookups_dev, hits, packs[r * stride:(r + 1) * stride], cap=cap)
        assert sha(hits.cpu().numpy().view(np.uint64).astype("<u8")) == g["rank_slice_hits_sha256"][r], r
        sets.append(s)
    counts = packs.view(world, stride)[:, 0].cpu().numpy()
    assert (counts <= cap).all() and int(counts.sum()) == g["hits_popcount"]
    full = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
    ok = torch.ones(1, dtype=torch.int32, device="cuda")
    gpu.hits_expand_set(packs, world, [shard_range(nf, world, r)[0] for r in range(world)], n, full, cap, ok=ok)
    assert int(ok.item()) == 1
    got = full.cpu().numpy().view(np.uint64)
    for r in range(world):
        assert sha(got[r * per:(r + 1) * per].astype("<u8")) == g["rank_slice_hits_sha256"][r], r
    del full, got, packs

    # The same C5 exchange as the N = 8 product path runs it: eight ranks of
    # the C ABI's communicator (loopback transport: one thread and one stream
    # per rank, all on this GPU), each calling cb_set_probe_allgather_fixed
    # with its own FilterSet; ranks 0 and 7 check every slice of their map.
    import threading

    from lsmt_amd.shard import Comm
    comms = Comm.loopback(world, 0)
    fulls = {r: torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for r in (0, 7)}
    errs = []

    def rank(r):
        try:
            st = torch.cuda.Stream()
            loc = torch.empty((per, words), dtype=torch.int64, device="cuda")
            out = fulls.get(r, None)
            if out is None:
                out = torch.empty((nf, words), dtype=torch.int64, device="cuda")
            ok = torch.ones(1, dtype=torch.int32, device="cuda")
            comms[r].probe_allgather(sets[r], c5_lookups_dev, nf, loc, out, sparse=True, cap=cap, ok=ok, stream=st)
            st.synchronize()
            assert int(ok.item()) == 1
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    try:
        assert not any(t.is_alive() for t in ts) and not errs, errs
        for r0, fm in fulls.items():
            got = fm.cpu().numpy().view(np.uint64)
            for r in range(world):
                assert sha(got[r * per:(r + 1) * per].astype("<u8")) == g["rank_slice_hits_sha256"][r], (r0, r)
    finally:
        for c in comms:
            c.close()
