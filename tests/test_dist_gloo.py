"""World-size-2 (and 3) gloo runs of the multi-GPU logic on CPU: filters
sharded per rank, local probes (the CPU oracle stands in for the per-rank GPU
probe here), one all-gather of the hit bitmaps; rank 0 checks the gathered
bitmap against the unsharded probe."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lsmt_amd.shard import PACK_BLOCK_WORDS, shard_range, sparse_cap


def test_shard_range_covers_exactly():
    for n in (1, 7, 32, 33, 256):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def np_compress(h, pack, cap):
    """CPU stand-in for lsmt_amd.hits_compress (the kernel is covered on the
    GPU by tests/test_exchange_gpu.py): {count, 0, positions[cap], directory
    of {first slot, number} per PACK_BLOCK_WORDS words}, positions grouped by block."""
    a = np.ascontiguousarray(h.numpy()).view(np.uint64).reshape(-1)
    pos = np.flatnonzero(np.unpackbits(a.view(np.uint8), bitorder="little")).astype(np.uint32)
    pk = pack.numpy().view(np.uint32)
    pk[:] = 0
    pk[0] = len(pos)
    k = min(len(pos), cap)
    pk[2:2 + k] = pos[:k]
    nblk = -(-a.size // PACK_BLOCK_WORDS)
    blk = (pos >> 6) // PACK_BLOCK_WORDS
    first = np.searchsorted(blk, np.arange(nblk))
    cnt = np.bincount(blk, minlength=nblk)[:nblk]
    pk[2 + cap:2 + cap + 2 * nblk:2] = first
    pk[3 + cap:3 + cap + 2 * nblk:2] = cnt


def np_expand(packs, world, row_off, full, ok, cap):
    """CPU stand-in for lsmt_amd.hits_expand, reading through the directory."""
    words = full.shape[1]
    fw = full.numpy().view(np.uint64).reshape(-1)
    fw[:] = 0
    pk = packs.numpy().view(np.uint32).reshape(world, -1)
    bounds = list(row_off) + [full.shape[0]]
    for r in range(world):
        if int(pk[r, 0]) > cap:  # as k_hits_expand: the rank contributes zeros, ok cleared
            if ok is not None:
                ok[0] = 0
            continue
        nblk = -(-(bounds[r + 1] - bounds[r]) * words // PACK_BLOCK_WORDS)
        for b in range(nblk):
            e0, ne = int(pk[r, 2 + cap + 2 * b]), int(pk[r, 3 + cap + 2 * b])
            pos = pk[r, 2 + e0:2 + e0 + ne].astype(np.uint64)
            assert ((pos >> np.uint64(6)) // np.uint64(PACK_BLOCK_WORDS) == b).all()
            np.bitwise_or.at(fw, bounds[r] * words + (pos >> np.uint64(6)),
                             np.left_shift(np.uint64(1), pos & np.uint64(63)))


def _worker(rank, world, port, n_filters, result_q, mode="dense"):
    import torch
    import torch.distributed as dist

    from lsmt_amd import workload
    from lsmt_amd.shard import gather_hits, shard_range
    from oracle import oracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m, kpf, n = 1 << 16, 800, 70_000  # 1094 hit words per row: several 2048-word pack blocks per shard
        lo, hi = shard_range(n_filters, world, rank)
        local = []
        for f in range(lo, hi):
            o = oracle.OracleFilter(m)
            o.insert_fixed(workload.key_range(100 + f, kpf))
            local.append(o)
        look = workload.probe_lookups(n, n_filters, kpf, seed_base=100, absent_seed=999)
        words = (n + 63) // 64
        lh = oracle.probe_fixed(local, look) if local else np.zeros((0, words), np.uint64)
        t = torch.from_numpy(lh.view(np.int64).copy()).reshape(hi - lo, words)
        if mode == "dense":
            full = gather_hits(t, n_filters)
        else:
            from lsmt_amd.shard import gather_hits_sparse, sparse_cap
            # "overflow": a pack too small for one rank -> every rank takes the dense path
            cap = 3 if mode == "overflow" else sparse_cap(n, n_filters, world)
            if mode.startswith("async"):
                # no host round trip: the overflow comes back in ok, and the
                # caller redoes that batch with the dense exchange
                cap = 3 if mode == "async_overflow" else cap
                ok = torch.ones(1, dtype=torch.int32)
                full = gather_hits_sparse(t, n_filters, cap, np_compress, np_expand, ok=ok)
                assert int(ok[0]) == (0 if mode == "async_overflow" else 1)
                if not int(ok[0]):
                    full = gather_hits(t, n_filters)
            else:
                st = {}
                full = gather_hits_sparse(t, n_filters, cap, np_compress, np_expand, stats=st)
                assert st["sparse"] == (mode == "sparse")
        if rank == 0:
            ref = []
            for f in range(n_filters):
                o = oracle.OracleFilter(m)
                o.insert_fixed(workload.key_range(100 + f, kpf))
                ref.append(o)
            expect = oracle.probe_fixed(ref, look)
            result_q.put(bool(np.array_equal(full.numpy().view(np.uint64), expect)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_filters,mode", [(2, 6, "dense"), (2, 5, "dense"), (3, 7, "dense"),
                                                  (2, 6, "sparse"), (3, 7, "sparse"), (3, 7, "overflow"),
                                                  (3, 7, "async"), (2, 5, "async_overflow"), (8, 19, "sparse"),
                                                  (8, 19, "dense")])
def test_sharded_probe_allgather_gloo(world, n_filters, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_filters, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("n_keys,f_total", [(1 << 20, 256), (10_000_000, 256), (4096, 3)])
def test_sparse_cap_covers_every_shard(n_keys, f_total):
    """The pack capacity covers the largest shard's present keys (half of the
    lookups, key j = i/2 in table j mod f_total, lsmt_amd/workload.py) plus
    four times the expected false positives (2.4e-4 per pair at 10 bits/key)."""
    for world in range(1, 9):
        cap = sparse_cap(n_keys, f_total, world)
        for r in range(world):
            lo, hi = shard_range(f_total, world, r)
            j = np.arange(n_keys // 2)
            present = int(((j % f_total >= lo) & (j % f_total < hi)).sum())
            assert cap >= present + 4 * 2.4e-4 * n_keys * (hi - lo), (world, r)


def test_comm_shard_matches_shard_range():
    # the C ABI's split (cb_comm_shard, lsmt_amd/csrc/comm.cpp) is the one the
    # orchestration above uses; host-only, no GPU call
    from lsmt_amd.shard import comm_shard
    for n in (0, 1, 7, 32, 33, 256, 257):
        for world in (1, 2, 3, 8, 64):
            for r in range(world):
                assert comm_shard(n, world, r) == shard_range(n, world, r), (n, world, r)


def test_pack_words_matches_c_abi():
    import ctypes

    from lsmt_amd import _lib
    from lsmt_amd.shard import pack_words
    out = ctypes.c_uint64()
    for rows, words, cap in ((0, 5, 7), (1, 1, 0), (32, 16384, 119570), (3, 1025, 10), (32, 156250, 10 ** 6)):
        _lib.check(_lib.load().cb_hits_pack_words(rows, words, cap, ctypes.byref(out)))
        assert out.value == pack_words(rows * words, cap)
