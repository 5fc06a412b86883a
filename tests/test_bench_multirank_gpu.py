"""bench.py's N-rank path on one GPU (the driver's scaling runs use N GPUs,
which this box does not have): `bench.py --gpus N --rehearse-one-gpu`
starts N rank processes itself, puts every rank on GPU 0 and moves the
exchange's bytes with the C ABI's host transport over gloo instead of RCCL.
Everything else — the launcher, the per-rank filter shards, the pipelined
lanes sharing one communicator, the sparse and dense exchanges, the timing
reductions and the single result line — is the N-GPU code, and --check
compares every rank's rows and its neighbour's rows in the exchanged map with
the oracle (the fan-out it shards: /root/reference/src/lib.rs:129-134).
The C4 workload (64 concurrent flush builds split over the ranks,
src/lib.rs:96-109,195-210) and the C5 workload (10M-key fan-out over 32
filters per rank) run through the same N-rank code at world 2 and 3."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "4", "--warmup", "2", "--filters", "5", "--m-bits", str(1 << 22), "--keys-per-filter",
         str(1 << 15), "--n-keys", "100000", "--build-keys", str(1 << 16), "--build-m-bits", str(1 << 20),
         "--no-cpu", "--no-e2e", "--no-cold", "--no-read", "--no-flush", "--no-c4", "--no-c5", "--check"]


def _run(world, args, sparse=None, timeout=170):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    if sparse is not None:
        env["CB_SPARSE_EXCHANGE"] = sparse
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                        "--rehearse-one-gpu"] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world
    assert d["valid"] is False and "rehearsal" in d  # never a scaling number
    return d, p.stderr


@pytest.mark.parametrize("world,sparse", [(2, "1"), (3, "0")])
def test_bench_rehearsal_ranks(gpu, world, sparse):
    d, err = _run(world, SMALL, sparse)
    assert d["config"]["filters_total"] == 5 * world
    assert d["exchange"]["mode"] == ("sparse" if sparse == "1" else "dense")
    if sparse == "1":
        assert d["exchange"]["all_fit"] is True
    assert "[check] hits bit-exact vs oracle" in err


@pytest.mark.parametrize("world", [2, 3])
def test_bench_rehearsal_c4(gpu, world):
    """--workload c4 at world > 1: each rank builds its contiguous share of
    the 64 filters (32/32, or 22/21/21) on its lanes; every filter of every
    rank is checked against the golden SHA-256s and 4 per rank against the C
    oracle, the verdicts combined over the ranks."""
    d, _ = _run(world, ["--workload", "c4", "--steps", "4", "--warmup", "1", "--no-cpu", "--check"])
    leg = d["c4"]
    assert leg["filters_total"] == 64 and leg["filters_this_gpu"] == (64 + world - 1) // world
    assert leg["golden_all_filters_bit_exact"] is True and leg["oracle_sample_bit_exact"] is True
    assert d["scaling"] == "strong" and d["roofline"]["algorithmic_bytes"] > 0


@pytest.mark.parametrize("world,sparse", [(2, "1"), (3, "0")])
def test_bench_rehearsal_c5(gpu, world, sparse):
    """--workload c5 at world > 1 in a small shape (C5's filters and seeds,
    200K lookups): each rank's 32-filter slice and the exchanged map against
    the oracle."""
    d, err = _run(world, ["--workload", "c5", "--n-keys", "200000", "--steps", "4", "--warmup", "1",
                          "--no-cpu", "--no-e2e", "--no-cold", "--no-read", "--no-flush", "--no-zone", "--check"],
                  sparse)
    assert d["config"]["filters_total"] == 32 * world and d["config"]["m_bits"] == 1 << 26
    assert "[check] hits bit-exact vs oracle" in err
