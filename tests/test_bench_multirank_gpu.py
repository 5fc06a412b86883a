"""bench.py's N-rank path on one GPU (the driver's scaling runs use N GPUs,
which this box does not have): `bench.py --gpus N --rehearse-one-gpu`
starts N rank processes itself, puts every rank on GPU 0 and moves the
exchange's bytes with the C ABI's host transport over gloo instead of RCCL.
Everything else — the launcher, the per-rank filter shards, the pipelined
lanes sharing one communicator, the sparse and dense exchanges, the timing
reductions and the single result line — is the N-GPU code, and --check
compares every rank's rows and its neighbour's rows in the exchanged map with
the oracle (the fan-out it shards: /root/reference/src/lib.rs:129-134)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "4", "--warmup", "2", "--filters", "5", "--m-bits", str(1 << 22), "--keys-per-filter",
         str(1 << 15), "--n-keys", "100000", "--build-keys", str(1 << 16), "--build-m-bits", str(1 << 20),
         "--no-cpu", "--no-e2e", "--no-cold", "--no-read", "--no-flush", "--check"]


@pytest.mark.parametrize("world,sparse", [(2, "1"), (3, "0")])
def test_bench_rehearsal_ranks(gpu, world, sparse):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["CB_SPARSE_EXCHANGE"] = sparse
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu"]
                       + SMALL, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["config"]["filters_total"] == 5 * world
    assert d["valid"] is False and "rehearsal" in d  # never a scaling number
    assert d["exchange"]["mode"] == ("sparse" if sparse == "1" else "dense")
    if sparse == "1":
        assert d["exchange"]["all_fit"] is True
    assert "[check] hits bit-exact vs oracle" in p.stderr
