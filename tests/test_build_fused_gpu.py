"""The one-launch single build (kernels.hip k_build_fused: partition and tile
workgroups in one grid, the tiles waiting on the partition's arrival counters)
against the CPU oracle and against the two-launch build, bit for bit.

Reference semantics: BloomFilter::insert (/root/reference/src/bloom.rs:40-44)
over a flush's keys (src/sstable.rs:59-65). The fused launch is the default
for every single tiled build (m >= 2^20 bits, >= 2^15 keys); cb_set_build_fused(-1)
restores k_build_part + k_build_tile. Besides the bits, these tests check that
the fused kernel is the one that ran (the library's per-launch profile), that
its counters are reused correctly by many builds on one stream (their two
sets alternate per launch), and that concurrent builds on several streams
keep apart (each stream has its own counters).
"""
import ctypes
import hashlib

import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def launches(gpu, name):
    from lsmt_amd import _lib
    tot, cnt = ctypes.c_double(0), ctypes.c_uint64(0)
    assert _lib.load().cb_profile_read(name.encode(), ctypes.byref(tot), ctypes.byref(cnt)) == 0
    return int(cnt.value)


@pytest.fixture
def prof(gpu):
    from lsmt_amd import _lib
    L = _lib.load()
    L.cb_profile_reset()
    L.cb_profile_enable(1)
    yield gpu
    L.cb_profile_enable(0)
    L.cb_profile_reset()


@pytest.fixture
def unfused(gpu):
    gpu.set_build_fused(-1)
    yield gpu
    gpu.set_build_fused(0)


@pytest.mark.parametrize("m", [1 << 20, (1 << 20) + 3, 1 << 24, 1 << 27])
@pytest.mark.parametrize("n", [1 << 15, 70_001, 1 << 20, (1 << 20) + 4097])
def test_fused_build_matches_oracle(prof, m, n):
    gpu = prof
    keys = workload.key_range(900 + n % 97, n)
    f = gpu.BloomFilter(m)
    f.insert_batch(keys)
    o = oracle.OracleFilter(m)
    o.insert_fixed(keys)
    assert np.array_equal(f.bools(), o.bools())
    assert gpu.last_path() == 2
    assert launches(gpu, "k_build_fused") == 1 and launches(gpu, "k_build_part") == 0


def test_fused_equals_two_launch_build(gpu):
    m, n = 1 << 27, 1 << 20
    keys = workload.c2_build_keys(n)
    a = gpu.BloomFilter(m)
    a.insert_batch(keys)
    gpu.set_build_fused(-1)
    try:
        b = gpu.BloomFilter(m)
        b.insert_batch(keys)
    finally:
        gpu.set_build_fused(0)
    assert np.array_equal(a.packed(), b.packed())


def test_unfused_path_still_builds(unfused, golden):
    g = golden["c2"]
    f = unfused.BloomFilter(g["m"])
    f.insert_batch(workload.c2_build_keys(g["n"]))
    assert sha(f.bools()) == g["bools_sha256"]


def test_fused_into_existing_filter_and_var_keys(prof):
    # a second batch ORed into a built filter (the tile blocks load the
    # filter's words instead of clearing), then variable-length keys
    gpu = prof
    m = (1 << 21) + 11
    rng = np.random.default_rng(5)
    k1 = workload.key_range(1201, 200_000)
    data, offs = workload.var_keys(rng, 150_000, max_len=40)
    f = gpu.BloomFilter(m)
    f.insert_batch(k1)
    f.insert_batch(gpu.KeyBatch(n=150_000, data=data, offsets=offs))
    o = oracle.OracleFilter(m)
    o.insert_fixed(k1)
    for i in range(150_000):
        o.insert(data[offs[i]:offs[i + 1]].tobytes())
    assert np.array_equal(f.bools(), o.bools())
    assert launches(gpu, "k_build_fused") == 2


def test_fused_many_builds_one_stream(gpu):
    # 40 builds back to back on one stream, every one checked: the counter
    # sets alternate per launch and each launch clears the other set
    import torch
    m = 1 << 22
    s = torch.cuda.Stream()
    made = []
    for i in range(40):
        keys = workload.key_range(1300 + i, 40_000 + 997 * i)
        dk = torch.from_numpy(keys).cuda()
        torch.cuda.synchronize()
        f = gpu.BloomFilter(m)
        f.insert_batch(gpu.DeviceKeys(dk), stream=s.cuda_stream)
        made.append((f, keys, dk))  # dk held until the stream is done with it
    s.synchronize()
    for f, keys, _ in made:
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        assert np.array_equal(f.bools(), o.bools())


def test_fused_concurrent_streams(gpu):
    # four streams building at once (the bench's C2 lanes), each stream with
    # its own counters, repeated so builds of different streams overlap
    import torch
    m, n = 1 << 27, 1 << 20
    keys = torch.from_numpy(workload.c2_build_keys(n)).cuda()
    streams = [torch.cuda.Stream() for _ in range(4)]
    fs = [gpu.BloomFilter(m) for _ in range(4)]
    torch.cuda.synchronize()
    for rep in range(6):
        for f, st in zip(fs, streams):
            f.clear(stream=st.cuda_stream)
            f.insert_batch(gpu.DeviceKeys(keys), stream=st.cuda_stream)
    torch.cuda.synchronize()
    o = oracle.OracleFilter(m)
    o.insert_fixed(workload.c2_build_keys(n))
    ref = o.bools()
    for f in fs:
        assert np.array_equal(f.bools(), ref)


def test_fused_uneven_load(gpu):
    # builds running beside streaming kernels of another stream that hold
    # CUs on every XCD: partition and tile workgroups are dispatched among
    # the other kernel's, the tiles wait unevenly, and must still see every
    # entry (the hand-off under uneven load)
    import torch
    m = 1 << 24
    other, s = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.ones(1 << 27, device="cuda")
    work = [(workload.key_range(1400 + i, 300_000 + 50_021 * i), gpu.BloomFilter(m)) for i in range(6)]
    dks = [torch.from_numpy(k).cuda() for k, _ in work]
    torch.cuda.synchronize()
    with torch.cuda.stream(other):
        for _ in range(12):
            x.mul_(1.0000001)
    for (keys, f), dk in zip(work, dks):
        f.insert_batch(gpu.DeviceKeys(dk), stream=s.cuda_stream)
    torch.cuda.synchronize()
    for keys, f in work:
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        assert np.array_equal(f.bools(), o.bools())
