"""The multi-GPU hit-map exchange on the device (the fan-out it
shards is /root/reference/src/lib.rs:129-134):

- cb_hits_compress (one launch; blocks claim their slots atomically and
  record them in the pack's directory) against a numpy restatement of "the
  set-bit positions of every 2048-word block, in order", at sizes from one
  word to a C5 rank slice (32 x 156250 words, ~4900 blocks), repeated so the
  alternating counter pairs are exercised;
- cb_hits_expand of uneven rank slices (one empty), with an overflowed rank;
- the C-ABI communicator (cb_comm over RCCL) at world size 1: dense, sparse,
  sparse with the synchronous overflow fallback and with the asynchronous ok
  flag, on hit rows from a real probe, bit-exact against the oracle's probe.
"""
import numpy as np
import pytest

from lsmt_amd import workload
from lsmt_amd.shard import PACK_BLOCK_WORDS

pytestmark = pytest.mark.gpu


def positions(h):
    return np.flatnonzero(np.unpackbits(np.ascontiguousarray(h).reshape(-1).view(np.uint8),
                                        bitorder="little")).astype(np.uint32)


def check_pack(pk, h, cap):
    """pk (uint32) against the positions of h: count, and through the
    directory every 2048-word block's positions in order, in disjoint slot
    ranges that tile [0, count)."""
    want = positions(h)
    nw = h.size
    nblk = -(-nw // PACK_BLOCK_WORDS)
    assert pk[0] == len(want) and pk[1] == 0
    assert len(pk) >= 2 + cap + 2 * nblk
    dirs = pk[2 + cap:2 + cap + 2 * nblk].reshape(nblk, 2).astype(np.int64)
    blk = (want >> 6) // PACK_BLOCK_WORDS
    assert np.array_equal(dirs[:, 1], np.bincount(blk, minlength=nblk)[:nblk])
    if len(want) <= cap:
        used = dirs[dirs[:, 1] > 0]  # empty blocks claim no slots
        used = used[np.argsort(used[:, 0], kind="stable")]
        ends = np.cumsum(used[:, 1])
        assert np.array_equal(used[:, 0], ends - used[:, 1])  # the blocks tile the slots
        for b in range(nblk):
            f, c = dirs[b]
            assert np.array_equal(pk[2 + f:2 + f + c], want[blk == b]), b


@pytest.mark.parametrize("rows,words,density", [
    (1, 1, 0.3), (1, 1023, 0.02), (1, 1025, 0.02), (3, 1000, 0.0), (7, 3079, 0.05),
    (32, 16384, 0.0005), (32, 156250, 0.00025), (2, 4096, 1.0)])
def test_compress_matches_numpy(gpu, rows, words, density):
    import torch
    rng = np.random.default_rng(rows * 7919 + words)
    for rep in range(3):  # successive launches on one stream: the counter pairs alternate
        bits = (rng.random(rows * words * 64) < density).astype(np.uint8)
        if rep == 1 and bits.size >= 4096:
            bits[1024:4096] = 1  # a dense run inside one block
        h = np.packbits(bits, bitorder="little").view(np.uint64).reshape(rows, words)
        cap = int(bits.sum()) + 5
        pack = torch.full((2 + cap + 2 * (-(-h.size // PACK_BLOCK_WORDS)),), -1, dtype=torch.int32, device="cuda")
        gpu.hits_compress(torch.from_numpy(h.view(np.int64).copy()).cuda(), pack, cap)
        check_pack(pack.cpu().numpy().view(np.uint32), h, cap)


def test_compress_overflow_reports_count(gpu):
    import torch
    rng = np.random.default_rng(3)
    h = np.packbits((rng.random(64 * 50_000) < 0.01).astype(np.uint8), bitorder="little").view(np.uint64)
    pack = torch.zeros(2 + 1000 + 2 * 49, dtype=torch.int32, device="cuda")
    gpu.hits_compress(torch.from_numpy(h.view(np.int64).reshape(1, -1).copy()).cuda(), pack, cap=1000)
    pk = pack.cpu().numpy().view(np.uint32)
    assert pk[0] == len(positions(h)) > 1000
    check_pack(pk, h, 1000)  # count and per-block counts still exact


def test_compress_rejects_oversized(gpu):
    import torch
    h = torch.zeros((1 << 13, 1 << 13), dtype=torch.int64, device="cuda")  # 2^26 words: 2^32 positions
    pack = torch.zeros(2 + 16 + 2 * 65536, dtype=torch.int32, device="cuda")
    with pytest.raises(Exception):
        gpu.hits_compress(h, pack, cap=16)


@pytest.mark.parametrize("sizes", [[3, 2, 2], [1, 2, 1, 1, 2, 2, 1, 1, 2, 1], [5, 0, 4]])
def test_expand_rebuilds_map(gpu, sizes):
    """Packs of uneven rank slices (one with no rows), gathered at the largest
    shard's stride, expand to the dense concatenation; an overflowed rank
    clears ok and leaves zeros."""
    import torch
    rng = np.random.default_rng(len(sizes))
    words = 1500
    parts = [np.packbits((rng.random((r, words * 64)) < 0.02).astype(np.uint8), axis=1,
                         bitorder="little").view(np.uint64).reshape(r, words) for r in sizes]
    parts[0][0, :3] = ~np.uint64(0)  # all-ones words
    cap = max(int(np.unpackbits(p.view(np.uint8)).sum()) for p in parts) + 10
    stride = 2 + cap + 2 * (-(-max(sizes) * words // PACK_BLOCK_WORDS))
    packs = torch.zeros(len(sizes) * stride, dtype=torch.int32, device="cuda")
    for r, p in enumerate(parts):
        if p.size:
            gpu.hits_compress(torch.from_numpy(p.view(np.int64).copy()).cuda(),
                              packs[r * stride:(r + 1) * stride], cap=cap)
    dense = np.concatenate(parts, 0)
    row_off = list(np.cumsum([0] + sizes[:-1]))
    full = torch.full(dense.shape, -1, dtype=torch.int64, device="cuda")
    ok = torch.ones(1, dtype=torch.int32, device="cuda")
    gpu.hits_expand(packs, len(sizes), row_off, full, cap, ok=ok)
    assert np.array_equal(full.cpu().numpy().view(np.uint64), dense) and int(ok.item()) == 1
    # rank 0's count beyond cap: ok cleared, its rows zero, the others intact
    bad = packs.clone()
    bad[0] = cap + 1
    gpu.hits_expand(bad, len(sizes), row_off, full, cap, ok=ok)
    got = full.cpu().numpy().view(np.uint64)
    assert int(ok.item()) == 0 and not got[:sizes[0]].any()
    assert np.array_equal(got[sizes[0]:], dense[sizes[0]:])


@pytest.fixture(scope="module")
def probed_rows():
    """Hit rows of 6 filters probed on the GPU, and the oracle's rows."""
    import torch

    import lsmt_amd
    from oracle import oracle
    m, kpf, n, nf = 1 << 18, 3000, 40_000, 6
    look = workload.probe_lookups(n, nf, kpf, seed_base=100, absent_seed=999)
    gf, of = [], []
    for f in range(nf):
        keys = workload.key_range(100 + f, kpf)
        b = lsmt_amd.BloomFilter(m)
        b.insert_batch(keys)
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        gf.append(b)
        of.append(o)
    out = torch.zeros((nf, (n + 63) // 64), dtype=torch.int64, device="cuda")
    lsmt_amd.FilterSet.from_filters(gf).probe(lsmt_amd.DeviceKeys(torch.from_numpy(look).cuda()), out=out)
    expect = oracle.probe_fixed(of, look)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), expect)
    return out, expect


@pytest.fixture(scope="module")
def comm1():
    from lsmt_amd.shard import Comm
    c = Comm(0, 1, 0, Comm.unique_id())
    yield c
    c.close()


@pytest.mark.parametrize("mode", ["dense", "sparse", "sparse_async", "overflow_sync", "overflow_async"])
def test_comm_allgather_world1(gpu, comm1, probed_rows, mode):
    import torch
    local, expect = probed_rows
    nf, words = local.shape
    full = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
    nbits = int(np.unpackbits(expect.view(np.uint8)).sum())
    cap = 7 if mode.startswith("overflow") else nbits + 100
    ok = torch.ones(1, dtype=torch.int32, device="cuda") if mode.endswith("async") else None
    used = comm1.allgather(local, nf, full, sparse=mode != "dense", cap=cap, ok=ok)
    torch.cuda.synchronize()
    if mode == "overflow_async":
        assert int(ok.item()) == 0 and used  # reported, not repaired: the caller redoes it densely
        comm1.allgather(local, nf, full, sparse=False)
        torch.cuda.synchronize()
    else:
        assert used == (mode in ("sparse", "sparse_async"))
        if ok is not None:
            assert int(ok.item()) == 1
    assert np.array_equal(full.cpu().numpy().view(np.uint64), expect)


def test_comm_checks_shapes(gpu, comm1, probed_rows):
    import torch
    local, _ = probed_rows
    nf, words = local.shape
    full = torch.zeros((nf + 1, words), dtype=torch.int64, device="cuda")
    with pytest.raises(Exception):  # rows must equal this rank's shard of total_rows
        comm1.allgather(local, nf + 1, full)
    with pytest.raises(Exception):  # sparse needs a capacity
        comm1.allgather(local, nf, full[:nf], sparse=True, cap=0)


# ---- the probe writing the pack itself (cb_set_probe_pack_fixed / cb_hits_expand_set) ----

@pytest.fixture(scope="module")
def rank_sets():
    """Four 'ranks' on one GPU: FilterSets of 3, 2, 0 and 2 slots over 7
    filters, the same lookup batch, and the oracle's hit rows."""
    import torch

    import lsmt_amd
    from oracle import oracle
    m, kpf, n = 1 << 18, 3000, 70_001
    look = workload.probe_lookups(n, 7, kpf, seed_base=100, absent_seed=999)
    gf, of = [], []
    for f in range(7):
        keys = workload.key_range(100 + f, kpf)
        b = lsmt_amd.BloomFilter(m)
        b.insert_batch(keys)
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        gf.append(b)
        of.append(o)
    sizes = [3, 2, 0, 2]
    sets, lo = [], 0
    for sz in sizes:
        s = lsmt_amd.FilterSet(m, 32)
        if sz:
            s.assign_all(gf[lo:lo + sz])
        sets.append(s)
        lo += sz
    expect = oracle.probe_fixed(of, look)
    return sets, sizes, torch.from_numpy(look).cuda(), expect


@pytest.mark.parametrize("overflow_rank", [None, 1])
def test_probe_pack_expand_ranks(gpu, rank_sets, overflow_rank):
    import torch
    sets, sizes, keys, expect = rank_sets
    n = keys.shape[0]
    words = (n + 63) // 64
    nbits = int(np.unpackbits(expect.view(np.uint8)).sum())
    cap = nbits + 10
    stride = gpu.FilterSet.pack_words(n, cap)
    packs = torch.full((len(sizes) * stride,), -1, dtype=torch.int32, device="cuda")
    for r, (s, sz) in enumerate(zip(sets, sizes)):
        hits = torch.full((max(sz, 1), words), -1, dtype=torch.int64, device="cuda")
        s.probe_pack(keys, hits, packs[r * stride:(r + 1) * stride], cap=cap)
        if sz:
            lo = sum(sizes[:r])
            assert np.array_equal(hits.cpu().numpy().view(np.uint64), expect[lo:lo + sz])
            pk = packs[r * stride:(r + 1) * stride].cpu().numpy().view(np.uint32)
            assert pk[0] == int(np.unpackbits(expect[lo:lo + sz].view(np.uint8)).sum())
    if overflow_rank is not None:
        packs[overflow_rank * stride] = cap + 1
    full = torch.full((sum(sizes), words), -1, dtype=torch.int64, device="cuda")
    ok = torch.ones(1, dtype=torch.int32, device="cuda")
    row_off = list(np.cumsum([0] + sizes[:-1]))
    gpu.hits_expand_set(packs, len(sizes), row_off, n, full, cap, ok=ok)
    got = full.cpu().numpy().view(np.uint64)
    if overflow_rank is None:
        assert int(ok.item()) == 1 and np.array_equal(got, expect)
    else:
        lo = row_off[overflow_rank]
        hi = lo + sizes[overflow_rank]
        assert int(ok.item()) == 0 and not got[lo:hi].any()
        keep = np.r_[0:lo, hi:len(got)]
        assert np.array_equal(got[keep], expect[keep])


@pytest.mark.parametrize("mode", ["dense", "sparse", "sparse_async", "overflow_sync", "overflow_async", "gated"])
def test_comm_probe_allgather_world1(gpu, comm1, mode):
    """cb_set_probe_allgather_fixed at world size 1: the probe (writing the
    pack itself in sparse mode) and the exchange in one call, against the
    oracle's probe (and, gated, its zone && bloom gate)."""
    import torch

    import lsmt_amd
    from oracle import oracle
    m, kpf, n, nf = 1 << 18, 3000, 40_001, 5
    look = workload.probe_lookups(n, nf, kpf, seed_base=300, absent_seed=998)
    gf, of, zones = [], [], []
    for f in range(nf):
        keys = workload.key_range(300 + f, kpf)
        b = lsmt_amd.BloomFilter(m)
        b.insert_batch(keys)
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        gf.append(b)
        of.append(o)
        srt = workload.sort_keys16(keys)
        zones.append((bytes(srt[kpf // 4]), bytes(srt[3 * kpf // 4])))  # half-width zones: the gate rejects
    s = lsmt_amd.FilterSet.from_filters(gf)
    if mode == "gated":
        for f, (lo, hi) in enumerate(zones):
            s.set_zone(f, (lo, hi))
        d = np.ascontiguousarray(look.reshape(-1))
        offs = np.arange(0, 16 * (n + 1), 16, dtype=np.uint64)
        expect = oracle.probe_gated(of, [oracle.OracleZone(lo, hi) for lo, hi in zones], d, offs)
    else:
        expect = oracle.probe_fixed(of, look)
    words = (n + 63) // 64
    keys = torch.from_numpy(look).cuda()
    local = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
    full = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
    nbits = int(np.unpackbits(expect.view(np.uint8)).sum())
    cap = 7 if mode.startswith("overflow") else nbits + 100
    ok = torch.ones(1, dtype=torch.int32, device="cuda") if mode.endswith("async") else None
    used = comm1.probe_allgather(s, keys, nf, local, full, sparse=mode != "dense", cap=cap, ok=ok,
                                 gated=mode == "gated")
    torch.cuda.synchronize()
    assert np.array_equal(local.cpu().numpy().view(np.uint64), expect)
    if mode == "overflow_async":
        assert int(ok.item()) == 0 and used
        comm1.allgather(local, nf, full, sparse=False)
        torch.cuda.synchronize()
    else:
        assert used == (mode in ("sparse", "sparse_async", "gated"))
    assert np.array_equal(full.cpu().numpy().view(np.uint64), expect)
