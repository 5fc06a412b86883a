"""Tiled builds against the oracle when many are in flight: builds queued
back to back on one stream with no host sync (each reuses the stream's
partition workspace), the same spread over four streams at once (each
stream's own workspace), and plans with many more tiles than partition
blocks and the reverse. Reference: /root/reference/src/bloom.rs:40-44 via
src/sstable.rs:62-65."""
import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu
TILED = 2


def _bits_equal(g, o):
    return np.array_equal(g.bools(), o.bools())


def _cases(seed, count):
    rng = np.random.default_rng(seed)
    ms = [1 << 20, 1 << 22, 100003 * 17, 1 << 27, (1 << 24) + 5]
    out = []
    for i in range(count):
        m = ms[i % len(ms)]
        n = int(rng.integers(3000, 300_000))
        out.append((m, workload.key_range(1000 * seed + i, n)))
    return out


def test_builds_back_to_back_one_stream(gpu):
    import torch
    gpu.set_path(TILED)
    try:
        dev = torch.device("cuda", 0)
        cases = _cases(1, 24)
        filters = []
        for m, keys in cases:
            f = gpu.BloomFilter(m)
            f.insert_batch(gpu.DeviceKeys(torch.from_numpy(keys).to(dev)))  # device keys: no host sync
            filters.append(f)
        torch.cuda.synchronize(dev)
        for (m, keys), f in zip(cases, filters):
            o = oracle.OracleFilter(m)
            o.insert_fixed(keys)
            assert _bits_equal(f, o), (m, len(keys))
    finally:
        gpu.set_path(0)


def test_builds_four_streams(gpu):
    import torch
    gpu.set_path(TILED)
    try:
        dev = torch.device("cuda", 0)
        streams = [torch.cuda.Stream(device=dev) for _ in range(4)]
        cases = _cases(2, 24)
        dk = [torch.from_numpy(k).to(dev) for _, k in cases]
        torch.cuda.synchronize(dev)
        filters = []
        for i, (m, _) in enumerate(cases):
            f = gpu.BloomFilter(m)
            f.insert_batch(gpu.DeviceKeys(dk[i]), stream=streams[i % 4])
            filters.append(f)
        torch.cuda.synchronize(dev)
        for (m, keys), f in zip(cases, filters):
            o = oracle.OracleFilter(m)
            o.insert_fixed(keys)
            assert _bits_equal(f, o), (m, len(keys))
    finally:
        gpu.set_path(0)


@pytest.mark.parametrize("m,n", [(1 << 27, 5000),       # 256 tiles, 2 partition blocks
                                 (1 << 16, 1 << 20),    # few tiles, 256 blocks
                                 (1 << 21, 1)])
def test_build_tile_block_balance(gpu, m, n):
    gpu.set_path(TILED)
    try:
        keys = workload.key_range(77, n)
        g = gpu.BloomFilter(m)
        g.insert_batch(keys)
        g.insert_batch(keys[: max(1, n // 3)])  # again into the non-empty filter
        o = oracle.OracleFilter(m)
        o.insert_fixed(keys)
        assert _bits_equal(g, o)
    finally:
        gpu.set_path(0)


@pytest.mark.parametrize("m", [1 << 25, (1 << 25) + 12345, 3 << 23, 1 << 22, 1 << 26])
def test_batched_long_run_builds(gpu, m):
    """Batched builds of long runs take 16-bit entries in 2^16-bit sub-tiles
    (kernels.hip plan_build: C4's shape): 12 filters, ragged counts around
    2^18 keys, one of them a few keys repeated 60K times (super-runs past the
    two waves a tile workgroup loads at once), one already holding bits (the
    tile loaded, not cleared), m a power of two or not. The m's take every
    tile-kernel instantiation: 2^18-bit tiles of 4 sub-tiles (2^25, 3 2^23),
    2^17-bit tiles of 2 (2^22) and 2^19-bit tiles of 8 (2^26). Filters of 0,
    1 and 5000 keys leave partition blocks with no keys of theirs (the
    partition pass's clamped loads and discard word). Each against the
    oracle."""
    counts = [1 << 18, (1 << 18) - 1, 200_000, 150_000, 0, 1, 5000] + [240_000 + 997 * i for i in range(5)]
    keys = [workload.key_range(5000 + i, c) for i, c in enumerate(counts)]
    base = workload.key_range(77, 40)
    keys[2] = np.concatenate([keys[2], np.repeat(base[:3], 60_000, axis=0)])
    fs = [gpu.BloomFilter(m) for _ in counts]
    fs[7].insert_batch(workload.key_range(7, 1000))
    gpu.insert_many(fs, keys)
    for i, (f, k) in enumerate(zip(fs, keys)):
        o = oracle.OracleFilter(m)
        if i == 7:
            o.insert_fixed(workload.key_range(7, 1000))
        o.insert_fixed(k)
        assert _bits_equal(f, o), i
