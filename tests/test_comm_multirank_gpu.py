"""The C-ABI exchange at world size > 1 on one GPU (the fan-out
it shards is /root/reference/src/lib.rs:129-134).

Every host and device step of the product's exchange — shard split, pack
strides, the probe writing its pack, the sparse and dense all-gathers, the
uneven-shard padding and placement (comm.cpp allgather_dense), the
synchronous overflow redo and the asynchronous ok flag, and the collective
ordering across streams — runs here unchanged; only the transport that moves
the bytes differs from RCCL:

- loopback (cb_comm_init_loopback): every rank in this process, one host
  thread per rank, each on its own HIP stream;
- host (cb_comm_init_host): separate processes sharing the GPU, the bytes
  moved by a gloo all-gather of host buffers (test_host_transport_processes).

Each rank holds a contiguous shard of the filters (uneven: 7 over 3 ranks,
19 over 8, 5 over 2) and every rank's gathered map is compared with the
oracle's unsharded probe.
"""
import os
import socket
import threading

import numpy as np
import pytest

from lsmt_amd import workload
from lsmt_amd.shard import shard_range, sparse_cap

pytestmark = pytest.mark.gpu

M, KPF, N = 1 << 17, 1500, 30_001


def _run_ranks(world, fn):
    """fn(rank) on `world` threads at once; re-raises the first failure."""
    errs = [None] * world
    out = [None] * world

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    assert not any(t.is_alive() for t in ts), "a rank's collective never completed"
    for e in errs:
        if e is not None:
            raise e
    return out


_cache = {}


def _filters(nf):
    """nf GPU filters of M bits (filter f from key(500 + f, i)), the oracle's
    hit rows for the lookup batch, and the lookups themselves."""
    if nf in _cache:
        return _cache[nf]
    import lsmt_amd
    from oracle import oracle
    look = workload.probe_lookups(N, nf, KPF, seed_base=500, absent_seed=997)
    gf, of = [], []
    for f in range(nf):
        keys = workload.key_range(500 + f, KPF)
        b = lsmt_amd.BloomFilter(M)
        b.insert_batch(keys)
        o = oracle.OracleFilter(M)
        o.insert_fixed(keys)
        gf.append(b)
        of.append(o)
    _cache[nf] = (gf, oracle.probe_fixed(of, look), look)
    return _cache[nf]


CASES = [(2, 5), (3, 7), (8, 19), (2, 6)]


@pytest.mark.parametrize("mode", ["dense", "sparse", "overflow_sync", "probe"])
def test_rccl_single_rank(gpu, mode):
    """The RCCL transport itself (cb_comm_unique_id's ncclGetUniqueId and its
    socket bootstrap, ncclCommInitRank, ncclAllGather on the caller's stream,
    ncclCommDestroy) at world 1 on this box's one GPU: the calls every
    multi-GPU line makes, here with one rank (RCCL refuses two ranks on one
    device, so world > 1 runs only on the driver's 8-GPU node)."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    nf = 5
    gf, expect, look = _filters(nf)
    keys = torch.from_numpy(look).cuda()
    words = (N + 63) // 64
    s = lsmt_amd.FilterSet(M, 32)
    s.assign_all(gf)
    st = torch.cuda.Stream()
    full = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
    c = Comm(0, 1, 0, Comm.unique_id())
    try:
        if mode == "probe":
            local = torch.zeros((nf, words), dtype=torch.int64, device="cuda")
            c.probe_allgather(s, keys, nf, local, full, sparse=True,
                              cap=sparse_cap(N, nf, 1), stream=st)
        else:
            local = torch.zeros((nf, words), dtype=torch.int64, device="cuda")
            s.probe(lsmt_amd.DeviceKeys(keys), out=local)
            torch.cuda.synchronize()
            cap = 5 if mode == "overflow_sync" else sparse_cap(N, nf, 1)
            used = c.allgather(local, nf, full, sparse=mode != "dense", cap=cap, stream=st)
            assert used == (mode == "sparse")
        st.synchronize()
        assert np.array_equal(full.cpu().numpy().view(np.uint64), expect)
    finally:
        c.close()


@pytest.mark.parametrize("world,nf", CASES)
@pytest.mark.parametrize("mode", ["dense", "sparse", "sparse_async", "overflow_sync", "overflow_async"])
def test_loopback_hits_allgather(gpu, world, nf, mode):
    """cb_hits_allgather at world > 1: each rank's rows from its own FilterSet
    probe, gathered into every rank's [nf][words] map."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    gf, expect, look = _filters(nf)
    keys = torch.from_numpy(look).cuda()
    words = (N + 63) // 64
    comms = Comm.loopback(world, 0)
    sets, locals_ = [], []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        s = lsmt_amd.FilterSet(M, 32)
        s.assign_all(gf[lo:hi])
        loc = torch.zeros((hi - lo, words), dtype=torch.int64, device="cuda")
        if hi > lo:
            s.probe(lsmt_amd.DeviceKeys(keys), out=loc)
        sets.append(s)
        locals_.append(loc)
    torch.cuda.synchronize()
    cap = 5 if mode.startswith("overflow") else sparse_cap(N, nf, world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    fulls = [torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for _ in range(world)]
    oks = [torch.ones(1, dtype=torch.int32, device="cuda") for _ in range(world)]

    def rank(r):
        ok = oks[r] if mode.endswith("async") else None
        used = comms[r].allgather(locals_[r], nf, fulls[r], sparse=mode != "dense", cap=cap, ok=ok,
                                  stream=streams[r])
        streams[r].synchronize()
        if mode == "overflow_async":
            assert used and int(oks[r].item()) == 0  # reported, not repaired: redo densely
            comms[r].allgather(locals_[r], nf, fulls[r], stream=streams[r])
            streams[r].synchronize()
        return used

    try:
        used = _run_ranks(world, rank)
        assert all(u == (mode in ("sparse", "sparse_async", "overflow_async")) for u in used), used
        for r in range(world):
            assert np.array_equal(fulls[r].cpu().numpy().view(np.uint64), expect), f"rank {r}"
            if mode == "sparse_async":
                assert int(oks[r].item()) == 1
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("world,nf", CASES)
@pytest.mark.parametrize("mode", ["dense", "sparse", "sparse_async", "overflow_sync", "gated"])
def test_loopback_probe_allgather(gpu, world, nf, mode):
    """cb_set_probe_allgather_fixed at world > 1: the probe (writing the pack
    itself in sparse mode) and the exchange in one call per rank."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    from oracle import oracle
    gf, expect, look = _filters(nf)
    keys = torch.from_numpy(look).cuda()
    words = (N + 63) // 64
    zones = None
    if mode == "gated":  # half-width zones, so the gate rejects
        zones = []
        for f in range(nf):
            srt = workload.sort_keys16(workload.key_range(500 + f, KPF))
            zones.append((bytes(srt[KPF // 4]), bytes(srt[3 * KPF // 4])))
        of = []
        for f in range(nf):
            o = oracle.OracleFilter(M)
            o.insert_fixed(workload.key_range(500 + f, KPF))
            of.append(o)
        d = np.ascontiguousarray(look.reshape(-1))
        offs = np.arange(0, 16 * (N + 1), 16, dtype=np.uint64)
        expect = oracle.probe_gated(of, [oracle.OracleZone(lo, hi) for lo, hi in zones], d, offs)
    comms = Comm.loopback(world, 0)
    sets = []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        s = lsmt_amd.FilterSet(M, 32)
        s.assign_all(gf[lo:hi])
        if zones:
            for i, f in enumerate(range(lo, hi)):
                s.set_zone(i, zones[f])
        sets.append(s)
    torch.cuda.synchronize()
    cap = 5 if mode.startswith("overflow") else sparse_cap(N, nf, world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    fulls = [torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for _ in range(world)]
    locs = [torch.full((max(1, shard_range(nf, world, r)[1] - shard_range(nf, world, r)[0]), words), -1,
                       dtype=torch.int64, device="cuda") for r in range(world)]
    oks = [torch.ones(1, dtype=torch.int32, device="cuda") for _ in range(world)]

    def rank(r):
        ok = oks[r] if mode.endswith("async") else None
        used = comms[r].probe_allgather(sets[r], keys, nf, locs[r], fulls[r], sparse=mode != "dense", cap=cap,
                                        ok=ok, gated=mode == "gated", stream=streams[r])
        streams[r].synchronize()
        return used

    try:
        used = _run_ranks(world, rank)
        assert all(u == (mode in ("sparse", "sparse_async", "gated")) for u in used), used
        for r in range(world):
            lo, hi = shard_range(nf, world, r)
            if hi > lo:
                assert np.array_equal(locs[r].cpu().numpy().view(np.uint64), expect[lo:hi]), f"rank {r} rows"
            assert np.array_equal(fulls[r].cpu().numpy().view(np.uint64), expect), f"rank {r} map"
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("world,nf", [(2, 5), (3, 7)])
@pytest.mark.parametrize("gated", [0, 1])
def test_loopback_probe_allgather_uneven_sets(gpu, world, nf, gated):
    """The ranks' sets differ in what the caller cannot see: rank 0's slots
    carry zone bounds and the others' do not, and the last rank's set is 64
    wide instead of 32, on a batch dense enough for the region-partitioned
    probe (N = 30001 against m = 2^17). Every rank must still take the same
    pack format (comm.cpp sparse_separate reads only shared values; ADVICE
    r5: a choice read from the rank's own zone state split the ranks into
    different all-gather sizes and hung them). The map: rank 0's rows gated
    by its zones, the others' plain."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    from oracle import oracle
    gf, plain, look = _filters(nf)
    keys = torch.from_numpy(look).cuda()
    words = (N + 63) // 64
    expect = plain.copy()
    lo0, hi0 = shard_range(nf, world, 0)
    zones = []
    for f in range(lo0, hi0):
        srt = workload.sort_keys16(workload.key_range(500 + f, KPF))
        zones.append((bytes(srt[KPF // 4]), bytes(srt[3 * KPF // 4])))
    if gated:
        of = []
        for f in range(lo0, hi0):
            o = oracle.OracleFilter(M)
            o.insert_fixed(workload.key_range(500 + f, KPF))
            of.append(o)
        d = np.ascontiguousarray(look.reshape(-1))
        offs = np.arange(0, 16 * (N + 1), 16, dtype=np.uint64)
        expect[lo0:hi0] = oracle.probe_gated(of, [oracle.OracleZone(a, b) for a, b in zones], d, offs)
    comms = Comm.loopback(world, 0)
    sets = []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        s = lsmt_amd.FilterSet(M, 64 if r == world - 1 else 32)
        s.assign_all(gf[lo:hi])
        if r == 0:
            for i, z in enumerate(zones):
                s.set_zone(i, z)
        sets.append(s)
    torch.cuda.synchronize()
    cap = sparse_cap(N, nf, world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    fulls = [torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for _ in range(world)]
    locs = [torch.full((shard_range(nf, world, r)[1] - shard_range(nf, world, r)[0], words), -1,
                       dtype=torch.int64, device="cuda") for r in range(world)]

    def rank(r):
        used = comms[r].probe_allgather(sets[r], keys, nf, locs[r], fulls[r], sparse=True, cap=cap,
                                        gated=bool(gated), stream=streams[r])
        streams[r].synchronize()
        return used

    try:
        used = _run_ranks(world, rank)
        assert all(used), used
        for r in range(world):
            lo, hi = shard_range(nf, world, r)
            assert np.array_equal(locs[r].cpu().numpy().view(np.uint64), expect[lo:hi]), f"rank {r} rows"
            assert np.array_equal(fulls[r].cpu().numpy().view(np.uint64), expect), f"rank {r} map"
    finally:
        for c in comms:
            c.close()


def test_loopback_pipelined_lanes(gpu):
    """Three lanes per rank (streams) sharing one communicator, several
    batches in flight: each lane keeps its own packs and the collectives run
    in issue order, so every lane's map is the right one for its batch."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    world, nf, lanes, steps = 3, 7, 3, 6
    gf, _, _ = _filters(nf)
    batches = [workload.probe_lookups(N, nf, KPF, seed_base=500, absent_seed=900 + b) for b in range(lanes)]
    from oracle import oracle
    of = []
    for f in range(nf):
        o = oracle.OracleFilter(M)
        o.insert_fixed(workload.key_range(500 + f, KPF))
        of.append(o)
    expects = [oracle.probe_fixed(of, b) for b in batches]
    dkeys = [torch.from_numpy(b).cuda() for b in batches]
    comms = Comm.loopback(world, 0)
    sets = []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        s = lsmt_amd.FilterSet(M, 32)
        s.assign_all(gf[lo:hi])
        sets.append(s)
    torch.cuda.synchronize()
    words = (N + 63) // 64
    cap = sparse_cap(N, nf, world)
    fulls = [[torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for _ in range(lanes)]
             for _ in range(world)]

    def rank(r):
        lo, hi = shard_range(nf, world, r)
        sts = [torch.cuda.Stream() for _ in range(lanes)]
        locs = [torch.empty((hi - lo, words), dtype=torch.int64, device="cuda") for _ in range(lanes)]
        ok = torch.ones(1, dtype=torch.int32, device="cuda")
        for step in range(steps):
            ln = step % lanes
            comms[r].probe_allgather(sets[r], dkeys[ln], nf, locs[ln], fulls[r][ln], sparse=step % 2 == 0,
                                     cap=cap, ok=ok, stream=sts[ln])
        for st in sts:
            st.synchronize()
        return int(ok.item())

    try:
        oks = _run_ranks(world, rank)
        assert oks == [1] * world
        for r in range(world):
            for ln in range(lanes):
                assert np.array_equal(fulls[r][ln].cpu().numpy().view(np.uint64), expects[ln]), (r, ln)
    finally:
        for c in comms:
            c.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_worker(rank, world, port, nf, q):
    """One process per rank on the same GPU; the communicator's bytes move
    through gloo (cb_comm_init_host), everything else is the product path."""
    import torch
    import torch.distributed as dist

    import lsmt_amd
    from lsmt_amd.shard import Comm
    from oracle import oracle
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        def gloo_allgather(send, recv):
            n = send.size
            parts = [torch.empty(n, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(send.copy()))
            for r, p in enumerate(parts):
                recv[r * n:(r + 1) * n] = p.numpy()

        comm = Comm.host(rank, world, 0, gloo_allgather)
        look = workload.probe_lookups(N, nf, KPF, seed_base=500, absent_seed=997)
        lo, hi = shard_range(nf, world, rank)
        fl = []
        for f in range(lo, hi):
            b = lsmt_amd.BloomFilter(M)
            b.insert_batch(workload.key_range(500 + f, KPF))
            fl.append(b)
        s = lsmt_amd.FilterSet(M, 32)
        s.assign_all(fl)
        words = (N + 63) // 64
        keys = torch.from_numpy(look).cuda()
        ok_all = True
        of = []
        for f in range(nf):
            o = oracle.OracleFilter(M)
            o.insert_fixed(workload.key_range(500 + f, KPF))
            of.append(o)
        expect = oracle.probe_fixed(of, look)
        for sparse in (False, True):
            loc = torch.empty((hi - lo, words), dtype=torch.int64, device="cuda")
            full = torch.full((nf, words), -1, dtype=torch.int64, device="cuda")
            comm.probe_allgather(s, keys, nf, loc, full, sparse=sparse, cap=sparse_cap(N, nf, world))
            torch.cuda.synchronize()
            ok_all &= bool(np.array_equal(full.cpu().numpy().view(np.uint64), expect))
        comm.close()
        q.put((rank, ok_all))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nf", [(2, 5), (3, 7)])
def test_host_transport_processes(gpu, world, nf):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, nf, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=110)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive and all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=5) for _ in range(world))
    assert all(got[r] for r in range(world)), got


@pytest.mark.parametrize("world,nf", [(2, 150), (3, 200)])
@pytest.mark.parametrize("mode", ["dense", "sparse", "sparse_async"])
def test_loopback_probe_allgather_wide(gpu, world, nf, mode):
    """Shards past 64 tables per rank (wide FilterSets of 128 slots): the
    probe and the exchange in one call per rank — the sparse form probing
    first and compressing the rows separately — equal to the oracle's
    unsharded probe on every rank."""
    import torch

    import lsmt_amd
    from lsmt_amd.shard import Comm
    gf, expect, look = _filters(nf)
    keys = torch.from_numpy(look).cuda()
    words = (N + 63) // 64
    comms = Comm.loopback(world, 0)
    sets = []
    for r in range(world):
        lo, hi = shard_range(nf, world, r)
        assert hi - lo > 64
        s = lsmt_amd.FilterSet(M, 128)
        s.assign_all(gf[lo:hi])
        sets.append(s)
    torch.cuda.synchronize()
    cap = sparse_cap(N, nf, world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    fulls = [torch.full((nf, words), -1, dtype=torch.int64, device="cuda") for _ in range(world)]
    locs = [torch.full((shard_range(nf, world, r)[1] - shard_range(nf, world, r)[0], words), -1,
                       dtype=torch.int64, device="cuda") for r in range(world)]
    oks = [torch.ones(1, dtype=torch.int32, device="cuda") for _ in range(world)]

    def rank(r):
        ok = oks[r] if mode.endswith("async") else None
        used = comms[r].probe_allgather(sets[r], keys, nf, locs[r], fulls[r], sparse=mode != "dense", cap=cap,
                                        ok=ok, stream=streams[r])
        streams[r].synchronize()
        return used

    try:
        used = _run_ranks(world, rank)
        assert all(u == (mode != "dense") for u in used), used
        for r in range(world):
            lo, hi = shard_range(nf, world, r)
            assert np.array_equal(locs[r].cpu().numpy().view(np.uint64), expect[lo:hi]), f"rank {r} rows"
            assert np.array_equal(fulls[r].cpu().numpy().view(np.uint64), expect), f"rank {r} map"
            if mode == "sparse_async":
                assert int(oks[r].item()) == 1
    finally:
        for c in comms:
            c.close()
