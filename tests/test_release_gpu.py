"""Stream-ordered release of filter, table and set memory (Next 4).

The reference drops an SsTable (and its BloomFilter) while other tokio tasks
keep reading under `sstables.read()` (/root/reference/src/lib.rs:21,129). Round
5's pool_release ran hipDeviceSynchronize on every destroy, so one Drop
stalled every stream of the process. Now a destroyed handle's block is
retired behind an event on each stream the library has seen and handed out
again only once those events have completed (capi.cpp pool_release / reap):

- a probe loop on one stream keeps its device step time while another
  thread's handles are destroyed between its launches;
- a block whose last reader is still queued is never handed to a new
  filter before that reader has run (its hits are the old filter's, checked
  against the oracle);
- cb_stream_release frees a stream's buffers and later destroys no longer
  record on it.
"""
import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu

M = 1 << 26
F, KPF, N = 32, 1 << 17, 1 << 21


def _loop_ms(torch, gpu, fset, keys, hits, st, steps, between=None):
    """HIP-event time of `steps` FilterSet probes queued on st behind a ~5 ms
    spin (so the device never waits for the host's issue); between(i) runs on
    the host after step i is issued."""
    with torch.cuda.stream(st):
        torch.cuda._sleep(10_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(steps):
        fset.probe(keys, out=hits, stream=st.cuda_stream)
        if between is not None:
            between(i)
    e1.record(st)
    st.synchronize()
    return e0.elapsed_time(e1) / steps


def test_destroy_does_not_stall_a_probe_loop(gpu):
    """200 probe steps on stream A (each ~70 us on the device) with 20
    filters and 20 SSTables destroyed from the host between launches: the
    device step time stays within 5 % of the same loop without destroys.
    With a device-wide sync per destroy the host would drain A's queue 40
    times, and A would idle while Python issued the next steps."""
    import torch
    filters = []
    for f in range(F):
        b = gpu.BloomFilter(M)
        b.insert_batch(workload.key_range(300 + f, KPF))
        filters.append(b)
    fset = gpu.FilterSet.from_filters(filters)
    look = workload.probe_lookups(N, F, KPF, seed_base=300, absent_seed=399)
    keys = gpu.DeviceKeys(torch.from_numpy(look).cuda())
    hits = torch.zeros((F, (N + 63) // 64), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    other = torch.cuda.Stream()

    def victims():
        vf, vt = [], []
        for i in range(20):
            b = gpu.BloomFilter(1 << 22)
            b.insert_batch(workload.key_range(800 + i, 4096), stream=other.cuda_stream)
            vf.append(b)
            ks = workload.sort_keys16(workload.key_range(900 + i, 2048))
            t, _, _ = gpu.sstable_create([(bytes(k), bytes(k)) for k in ks], m=1024, stream=other.cuda_stream)
            vt.append(t)
        other.synchronize()
        return vf, vt

    for _ in range(3):
        _loop_ms(torch, gpu, fset, keys, hits, st, 20)  # warm-up (clocks, workspaces)
    base, rel = [], []
    for rep in range(3):
        base.append(_loop_ms(torch, gpu, fset, keys, hits, st, 200))
        vf, vt = victims()

        def drop(i, vf=vf, vt=vt):
            if i % 10 == 5 and vf:
                vf.pop().close()
                vt.pop().close()

        rel.append(_loop_ms(torch, gpu, fset, keys, hits, st, 200, drop))
        assert not vf and not vt
    b, r = float(np.median(base)), float(np.median(rel))
    assert r <= 1.05 * b, f"probe step {r:.4f} ms with destroys vs {b:.4f} ms without"
    # and the loop's answer is still the oracle's (filter 0's row)
    o = oracle.OracleFilter(M)
    o.insert_fixed(workload.key_range(300, KPF))
    assert np.array_equal(hits.cpu().numpy().view(np.uint64)[0], oracle.probe_fixed([o], look)[0])


def test_retired_block_not_reused_under_a_queued_reader(gpu):
    """A probe of filter A is queued behind a long spin on stream S; A is
    destroyed right away and a same-size filter B is created and built with
    other keys on stream T while S still waits. B must not get A's block
    before the probe has read it: the probe's hits are A's (oracle), and B's
    bits are B's."""
    import torch
    m = 1 << 24
    ka, kb = workload.key_range(31, 200_000), workload.key_range(32, 200_000)
    look = np.concatenate([ka[:5000], kb[:5000], workload.key_range(33, 5000)])
    a = gpu.BloomFilter(m)
    a.insert_batch(ka)
    torch.cuda.synchronize()
    s, t = torch.cuda.Stream(), torch.cuda.Stream()
    dkeys = torch.from_numpy(look).cuda()
    hits = torch.zeros((1, (len(look) + 63) // 64), dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        torch.cuda._sleep(400_000_000)  # ~0.2 s
    gpu.probe([a], gpu.DeviceKeys(dkeys), out=hits, stream=s.cuda_stream)
    a.close()  # returns at once: the block is retired behind s's event
    b = gpu.BloomFilter(m)
    b.insert_batch(gpu.DeviceKeys(torch.from_numpy(kb).cuda()), stream=t.cuda_stream)
    t.synchronize()
    s.synchronize()
    oa, ob = oracle.OracleFilter(m), oracle.OracleFilter(m)
    oa.insert_fixed(ka)
    ob.insert_fixed(kb)
    assert np.array_equal(hits.cpu().numpy().view(np.uint64), oracle.probe_fixed([oa], look))
    assert np.array_equal(b.bools(), ob.bools())


def test_stream_release(gpu):
    """cb_stream_release on a stream the library has used: its buffers go,
    later destroys do not touch it (the stream is then destroyed), and a
    later call on a new stream works as before."""
    import ctypes

    from lsmt_amd import _lib
    L = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
    keys = workload.key_range(41, 50_000)
    b = gpu.BloomFilter(1 << 20)
    b.insert_batch(keys, stream=st.value)
    got = b.may_contain_batch(keys[:1000], stream=st.value)
    assert L.cb_stream_release(st) == 0
    assert L.cb_stream_release(st) == 0  # unknown now: nothing to do
    assert hip.hipStreamDestroy(st) == 0
    b.close()  # records on the streams still known; the destroyed one is not among them
    c = gpu.BloomFilter(1 << 20)
    c.insert_batch(keys)
    o = oracle.OracleFilter(1 << 20)
    o.insert_fixed(keys)
    assert np.array_equal(c.bools(), o.bools())
    assert np.asarray(got).all()


def test_set_destroy_is_stream_ordered(gpu):
    """A FilterSet's words come from the same pool: destroying a set whose
    probe is still queued, then making a new set of the same shape, leaves
    the queued probe's answer intact."""
    import torch
    m = 1 << 22
    fs = []
    for f in range(8):
        b = gpu.BloomFilter(m)
        b.insert_batch(workload.key_range(60 + f, 20_000))
        fs.append(b)
    look = workload.probe_lookups(50_000, 8, 20_000, seed_base=60, absent_seed=69)
    s1 = gpu.FilterSet.from_filters(fs)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    hits = torch.zeros((8, (len(look) + 63) // 64), dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        torch.cuda._sleep(400_000_000)
    s1.probe(gpu.DeviceKeys(torch.from_numpy(look).cuda()), out=hits, stream=s.cuda_stream)
    s1.close()
    s2 = gpu.FilterSet(m, 32)
    s2.assign_all(fs[::-1])
    s.synchronize()
    ofs = []
    for f in range(8):
        o = oracle.OracleFilter(m)
        o.insert_fixed(workload.key_range(60 + f, 20_000))
        ofs.append(o)
    assert np.array_equal(hits.cpu().numpy().view(np.uint64), oracle.probe_fixed(ofs, look))
    h2 = s2.probe(look)
    assert np.array_equal(h2, oracle.probe_fixed(ofs[::-1], look))


def test_small_block_not_reused_under_a_queued_reader(gpu):
    """The same as above for a filter small enough to come from a slab
    (m = 2^16: 8 KiB, capi.cpp pool_alloc's small blocks): the queued probe
    reads A's bits, B's build gets another block or A's after the probe."""
    import torch
    m = 1 << 16
    ka, kb = workload.key_range(34, 3000), workload.key_range(35, 3000)
    look = np.concatenate([ka[:2000], kb[:2000], workload.key_range(36, 2000)])
    a = gpu.BloomFilter(m)
    a.insert_batch(ka)
    torch.cuda.synchronize()
    s, t = torch.cuda.Stream(), torch.cuda.Stream()
    dkeys = torch.from_numpy(look).cuda()
    hits = torch.zeros((1, (len(look) + 63) // 64), dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        torch.cuda._sleep(400_000_000)  # ~0.2 s
    gpu.probe([a], gpu.DeviceKeys(dkeys), out=hits, stream=s.cuda_stream)
    a.close()
    b = gpu.BloomFilter(m)
    b.insert_batch(gpu.DeviceKeys(torch.from_numpy(kb).cuda()), stream=t.cuda_stream)
    t.synchronize()
    s.synchronize()
    oa, ob = oracle.OracleFilter(m), oracle.OracleFilter(m)
    oa.insert_fixed(ka)
    ob.insert_fixed(kb)
    assert np.array_equal(hits.cpu().numpy().view(np.uint64), oracle.probe_fixed([oa], look))
    assert np.array_equal(b.bools(), ob.bools())


def test_small_blocks_are_reused(gpu):
    """Tables of the reference's auto-flush shape (1024 entries, m = 1024)
    made and dropped in rounds: once a round's blocks are retired and their
    events done, the next round's tables take them again (no new slabs: the
    device's free memory does not fall round over round), and every table
    answers its own keys."""
    import torch

    def round_(seed):
        ts = []
        for i in range(60):
            ks = workload.sort_keys16(workload.key_range(seed + i, 1024))
            t, bloom, _ = gpu.sstable_create([(bytes(k), bytes(k)) for k in ks], m=1024)
            ts.append((t, bloom, ks))
        torch.cuda.synchronize()
        for t, bloom, ks in ts[::17]:
            assert bloom.may_contain_batch(ks[:64]).all()
        for t, bloom, _ in ts:
            t.close()
            bloom.close()
        torch.cuda.synchronize()

    round_(5000)
    free1 = torch.cuda.mem_get_info()[0]
    for r in range(3):
        round_(6000 + 100 * r)
    free2 = torch.cuda.mem_get_info()[0]
    assert free2 >= free1 - (8 << 20), f"device free memory fell by {(free1 - free2) >> 20} MiB over 3 rounds"
