"""Single-key may_contain at the drop-in surface (row (b) of SURVEY.md §8):
SsTable::get calls `bloom.may_contain(key)` once per key per table
(/root/reference/src/sstable.rs:138; BloomFilter::may_contain,
src/bloom.rs:48-51). cb_may_contain answers it from a host mirror of the
filter's words (refreshed by one copy after each write) or, with the mirror
off, from a one-key GPU probe. Both are checked against the oracle and the
golden scenarios, the mirror's refresh after every kind of write (batched
build, per-key inserts, clear, import, decode), concurrent readers racing the
refresh, and the C-ABI latency tool (tests/cpp/may_contain_latency.c).
"""
import json
import os
import subprocess
import threading

import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _forget_streams(torch):
    """cb_stream_release on every stream earlier tests may have handed to the
    library (torch's pool streams, which rotate, and the null stream), so a
    refresh waits only on the streams the test itself uses. HIP multiplexes
    streams onto GPU_MAX_HW_QUEUES (4) hardware queues in creation order: an
    event on any stream sharing the busy stream's queue completes only after
    the busy kernel, so the busy stream must share a queue with no stream the
    library knows (the tests create the writer's stream right before it)."""
    from lsmt_amd import _lib
    L = _lib.load()
    for _ in range(64):
        assert L.cb_stream_release(torch.cuda.Stream().cuda_stream) == 0
    assert L.cb_stream_release(torch.cuda.current_stream().cuda_stream) == 0
    assert L.cb_stream_release(None) == 0


def _raw_stream():
    import ctypes
    raw = ctypes.c_void_p()
    assert ctypes.CDLL("libamdhip64.so").hipStreamCreateWithFlags(ctypes.byref(raw), 1) == 0
    return raw


def _busy_stream(torch):
    """A fresh HIP stream the library has never seen, running ~1 s of spin;
    (stream, event recorded after the spin, raw handle)."""
    raw = _raw_stream()
    st = torch.cuda.ExternalStream(raw.value)
    with torch.cuda.stream(st):
        torch.cuda._sleep(2_000_000_000)
        done = torch.cuda.Event()
        done.record(st)
    return st, done, raw


def _release(raw):
    import ctypes
    ctypes.CDLL("libamdhip64.so").hipStreamDestroy(raw)


def _lib_release(raw):
    from lsmt_amd import _lib
    assert _lib.load().cb_stream_release(raw) == 0
    _release(raw)


def oracle_hits(o, keys):
    h = oracle.probe_fixed([o], keys)
    return np.unpackbits(h.view(np.uint8), bitorder="little")[:len(keys)].astype(bool)


@pytest.mark.parametrize("mode", [1, 0])
def test_scenarios_both_sources(gpu, golden, mode):
    for name, s in golden["scenarios"].items():
        b = gpu.BloomFilter(s["m"])
        b.host_mirror(mode)
        for k in s["insert_hex"]:
            b.insert(bytes.fromhex(k))
        assert [b.may_contain(bytes.fromhex(k)) for k in s["probe_hex"]] == s["probe"], (name, mode)
        assert gpu.last_path() == (5 if mode else 1)


@pytest.mark.parametrize("m", [1 << 17, 100003, 1024, 1 << 26])
def test_c1_per_key_matches_oracle(gpu, m):
    """BASELINE C1 (10k keys; 100k absent keys probed) key by key through the
    mirror, and a slice of the same keys through the GPU probe."""
    keys = workload.key_range(1, 10_000)
    absent = workload.key_range(2, 100_000)
    b = gpu.BloomFilter(m)
    b.insert_batch(keys)
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    b.host_mirror(1)
    look = np.concatenate([keys, absent])
    got = np.array([b.may_contain(bytes(k)) for k in look])
    assert got[:len(keys)].all()
    assert np.array_equal(got, oracle_hits(o, look))
    b.host_mirror(0)
    sl = look[::37]
    assert np.array_equal(np.array([b.may_contain(bytes(k)) for k in sl]), oracle_hits(o, sl))


def test_mirror_follows_every_write(gpu):
    m = 1 << 16
    a, c = workload.key_range(31, 3000), workload.key_range(32, 3000)
    probe = np.concatenate([a, c, workload.key_range(33, 3000)])
    b = gpu.BloomFilter(m)
    b.host_mirror(1)
    o = oracle.OracleFilter(m)

    def check(tag):
        assert np.array_equal(np.array([b.may_contain(bytes(k)) for k in probe]), oracle_hits(o, probe)), tag
        assert b.host_mirror_info() == (True, True), tag

    check("empty")
    b.insert_batch(a)
    assert b.host_mirror_info() == (True, False)  # stale until the next read
    o.insert_fixed(a)
    check("batch")
    for k in c[:50]:
        b.insert(bytes(k))  # queued per-key inserts, flushed by the next read
    o.insert_fixed(c[:50])
    check("per-key inserts")
    b.clear()
    o = oracle.OracleFilter(m)
    check("clear")
    b.insert_batch(c)
    o.insert_fixed(c)
    check("rebuild after clear")
    bools = o.bools().copy()
    b2 = gpu.BloomFilter(m)
    b2.host_mirror(1)
    b2.may_contain(b"x")  # mirror taken of the empty filter
    b2.load_packed(np.packbits(bools, bitorder="little").view(np.uint32))  # cb_filter_import_packed
    assert np.array_equal(np.array([b2.may_contain(bytes(k)) for k in probe]), oracle_hits(o, probe))
    b3 = gpu.BloomFilter.from_bytes(b.to_bytes())
    b3.host_mirror(1)
    assert np.array_equal(np.array([b3.may_contain(bytes(k)) for k in probe]), oracle_hits(o, probe))


def test_concurrent_readers_race_the_refresh(gpu):
    """&self readers from many threads right after a build (on a side
    stream): every answer is the oracle's."""
    import torch
    m = 1 << 20
    keys = workload.key_range(41, 20_000)
    probe = np.concatenate([keys[:4000], workload.key_range(42, 4000)])
    expect = None
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    expect = oracle_hits(o, probe)
    for rep in range(3):
        b = gpu.BloomFilter(m)
        b.host_mirror(1)
        st = torch.cuda.Stream()
        b.insert_batch(gpu.DeviceKeys(torch.from_numpy(keys).cuda()), stream=st)  # async on st
        res = [None] * 8

        def reader(t):
            res[t] = np.array([b.may_contain(bytes(k)) for k in probe[t::8]])

        ts = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        for t in range(8):
            assert np.array_equal(res[t], expect[t::8]), (rep, t)


def test_mirror_turned_on_after_unrecorded_writes(gpu):
    """m = 2^26 is past the auto mirror (m <= 2^24), so builds record no
    write event; turning the mirror on afterwards, while a build on a side
    stream may still run, must still give the oracle's answers (the first
    refresh syncs the device), and so must a batched build of two filters."""
    import torch
    m = 1 << 26
    keys = workload.key_range(51, 200_000)
    probe = np.concatenate([keys[:3000], workload.key_range(52, 3000)])
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    expect = oracle_hits(o, probe)
    b = gpu.BloomFilter(m)
    assert b.host_mirror_info()[0] is False  # auto: off past 2^24
    st = torch.cuda.Stream()
    b.insert_batch(gpu.DeviceKeys(torch.from_numpy(keys).cuda()), stream=st)  # async on st
    b.host_mirror(1)
    assert np.array_equal(np.array([b.may_contain(bytes(k)) for k in probe]), expect)
    # on, a write (marked), off, a write (unrecorded), on again
    more = workload.key_range(53, 50_000)
    b.insert_batch(more)
    b.host_mirror(0)
    extra = workload.key_range(54, 50_000)
    b.insert_batch(gpu.DeviceKeys(torch.from_numpy(extra).cuda()), stream=st)
    b.host_mirror(1)
    o.insert_fixed(more)
    o.insert_fixed(extra)
    assert np.array_equal(np.array([b.may_contain(bytes(k)) for k in probe]), oracle_hits(o, probe))
    # a batched build (one launch pair for both filters), then the mirror
    fs = [gpu.BloomFilter(m) for _ in range(2)]
    dk = [torch.from_numpy(keys).cuda(), torch.from_numpy(extra).cuda()]
    gpu.insert_many(fs, dk, stream=st)
    for f, ks in zip(fs, (keys, extra)):
        f.host_mirror(1)
        of = oracle.OracleFilter(m)
        of.insert_fixed(ks)
        assert np.array_equal(np.array([f.may_contain(bytes(k)) for k in probe]), oracle_hits(of, probe))


def test_unrecorded_refresh_waits_for_its_stream_only(gpu):
    """A write made while the mirror was off records nothing; the first
    refresh after the mirror comes on waits, by events, for the streams the
    library has enqueued on, not for the whole device: a long kernel on a
    stream the library never saw (a ~1 s spin) is still running when the
    refresh has returned the oracle's answers (the refresh used to
    call hipDeviceSynchronize)."""
    import torch
    m = 1 << 26
    keys = workload.key_range(61, 100_000)
    probe = np.concatenate([keys[:500], workload.key_range(62, 500)])
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    b = gpu.BloomFilter(m)
    b.host_mirror(0)
    _forget_streams(torch)
    wr = _raw_stream()  # (created right before the busy stream: the next hardware queue)
    dkeys = torch.from_numpy(keys).cuda()
    torch.cuda.synchronize()
    b.insert_batch(gpu.DeviceKeys(dkeys), stream=wr.value)  # unrecorded
    busy, done, raw = _busy_stream(torch)
    b.host_mirror(1)
    got = np.array([b.may_contain(bytes(k)) for k in probe])
    still_busy = not done.query()
    busy.synchronize()
    _release(raw)
    _lib_release(wr)
    assert np.array_equal(got, oracle_hits(o, probe))
    assert still_busy, "the mirror refresh waited for an unrelated stream"


def test_unrecorded_write_on_a_destroyed_stream(gpu):
    """A write made while the mirror was off, on a stream the caller then
    releases (cb_stream_release: it synchronises that stream and forgets it)
    and destroys: the refresh keeps no stream handle (it used to
    synchronise a stored raw handle, falling back to the whole device for a
    dead one) and waits only on the streams the library still knows, so the
    mirror holds the write with no device-wide sync in the path: a ~1 s
    kernel on another stream is still running when the answers are back."""
    import ctypes

    import torch
    from lsmt_amd import _lib
    m = 1 << 26
    keys = workload.key_range(71, 100_000)
    probe = np.concatenate([keys[:500], workload.key_range(72, 500)])
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    b = gpu.BloomFilter(m)
    b.host_mirror(0)
    hip = ctypes.CDLL("libamdhip64.so")
    _forget_streams(torch)
    st = _raw_stream()
    b.insert_batch(keys, stream=st.value)  # on the raw stream, mirror off
    assert _lib.load().cb_stream_release(st) == 0
    assert hip.hipStreamDestroy(st) == 0
    busy, done, raw = _busy_stream(torch)
    b.host_mirror(1)
    got = np.array([b.may_contain(bytes(k)) for k in probe])
    still_busy = not done.query()
    busy.synchronize()
    _release(raw)
    assert np.array_equal(got, oracle_hits(o, probe))
    assert still_busy, "the mirror refresh waited for an unrelated stream"


def test_latency_tool_mirror_under_1us(gpu):
    """The C-ABI per-key call (no Python in the loop) at the product's m =
    1024 and at the C3 filter size: the mirror agrees with the GPU probe on
    every key and answers in well under a microsecond."""
    exe = os.path.join(ROOT, "build", "tests", "may_contain_latency")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    for m, n in ((1024, 100), (1 << 26, 1 << 19)):
        r = subprocess.run([exe, str(m), str(n), "200000"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["agree"] is True and d["hits"] >= d["probe_keys"] // 2
        assert d["mirror_ns_per_call"] < 1000.0, d
