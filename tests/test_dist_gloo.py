"""Host-side pieces of the multi-GPU path on CPU (no GPU): the shard split
and the pack sizes agree between Python and the C ABI, the sparse pack
capacity covers every shard, and `bench.py --gpus N` starts N ranks itself
(world-size 2 and 3 gloo dry runs). The exchange itself — the C ABI's
compress, all-gather and expand — runs at world > 1 in the GPU suite
(tests/test_comm_multirank_gpu.py: loopback and host transports)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from lsmt_amd.shard import shard_range, sparse_cap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_covers_exactly():
    for n in (1, 7, 32, 33, 256):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


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


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_n_ranks(world):
    """`python bench.py --gpus N` with no WORLD_SIZE starts N rank processes
    itself (torch.distributed.run) and relays rank 0's single JSON line; the
    dry run joins a gloo group and reports every rank's RANK / LOCAL_RANK /
    WORLD_SIZE without touching a GPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # exactly one JSON line on stdout
    d = json.loads(lines[0])
    assert d["dry_run"] is True and d["n_gpus"] == world and d["launcher"] == "bench.py"
    ranks = d["ranks"]
    assert sorted(r["rank"] for r in ranks) == list(range(world))
    assert sorted(r["local_rank"] for r in ranks) == list(range(world))
    assert all(r["world_size"] == world for r in ranks)


def test_bench_rank_refuses_wrong_world():
    """Inside a rank, --gpus must equal WORLD_SIZE (an error, not a note)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
    assert not p.stdout.strip()


def _bench_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "CB_BENCH_STALL")}


def test_stalled_rank_ends_the_job_within_the_bound():
    """A rank that stalls inside a guarded phase (CB_BENCH_STALL="1:dry_run":
    rank 1 never joins the all-gather, as a rank hung at RCCL init or in a
    collective would) passes its --phase-deadline; so does rank 0, blocked
    in the same all-gather: the first to fire prints one JSON diagnostic line
    and exits 4, torch.distributed.run ends the other, and the `--gpus 2`
    parent exits non-zero
    well inside the bound, with no result line (Next 3)."""
    import time
    env = dict(_bench_env(), CB_BENCH_STALL="1:dry_run")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--phase-deadline", "8", "--job-deadline", "200"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert p.returncode != 0, p.stderr[-3000:]
    assert not p.stdout.strip()
    diag = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith('{"error": "deadline"')]
    # the stalled rank, or its peer blocked in the same all-gather: whichever
    # watchdog fires first ends the job
    assert diag and diag[0]["phase"] == "dry_run" and diag[0]["seconds"] >= 8, p.stderr[-3000:]
    assert took < 120, took


def test_job_deadline_kills_every_rank():
    """The parent's backstop: with the ranks' own bound out of reach
    (--phase-deadline 1000) a stalled rank holds the job until the parent's
    --job-deadline, which kills the launcher's process group and exits 5
    with a JSON diagnostic line."""
    import time
    env = dict(_bench_env(), CB_BENCH_STALL="0:dry_run")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--phase-deadline", "1000", "--job-deadline", "25"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert p.returncode == 5, (p.returncode, p.stderr[-3000:])
    assert any(ln.startswith('{"error": "job deadline"') for ln in p.stderr.splitlines()), p.stderr[-3000:]
    assert took < 90, took
