"""Time the pieces of the sparse hit-bitmap exchange (lsmt_amd/shard.py
cb_hits_allgather) on one GPU at the per-rank shape of C3 on 8 GPUs: a
[32][16384] rank slice holding ~66K set bits, 8 packs of that size to expand
into the [256][16384] global map. Prints one JSON line of microseconds per
piece (HIP events, median of 50), and the whole C-ABI exchange
(cb_hits_allgather) at world size 1. Diagnostic only."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd.shard import pack_words, sparse_cap  # noqa: E402


def timed(fn, reps=50):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(float(np.median(ts)), 2)


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    rows, words, world = 32, 16384, 8
    rng = np.random.default_rng(1)
    bits = np.zeros(rows * words * 64, np.uint8)
    bits[rng.choice(bits.size, 66_000, replace=False)] = 1
    h = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64).reshape(rows, words).copy()).to(dev)
    cap = sparse_cap(1 << 20, rows * world, world)
    stride = pack_words(rows * words, cap)
    pack = torch.empty(stride, dtype=torch.int32, device=dev)
    packs = torch.empty(world * stride, dtype=torch.int32, device=dev)
    full = torch.empty((rows * world, words), dtype=torch.int64, device=dev)
    lsmt_amd.hits_compress(h, pack, cap)
    for r in range(world):
        packs[r * stride:(r + 1) * stride] = pack
    row_off = [r * rows for r in range(world)]
    out = {"cap": cap, "bits_per_rank": int(bits.sum())}
    out["compress_us"] = timed(lambda: lsmt_amd.hits_compress(h, pack, cap))
    out["expand_8_ranks_us"] = timed(lambda: lsmt_amd.hits_expand(packs, world, row_off, full, cap))
    out["memset_full_us"] = timed(lambda: full.zero_())
    out["counts_to_host_us"] = timed(lambda: packs.view(world, stride)[:, 0].cpu())
    one = torch.empty(stride, dtype=torch.int32, device=dev)
    out["allgather_pack_world1_us"] = timed(lambda: dist.all_gather_into_tensor(one, pack))
    dense = torch.empty((rows, words), dtype=torch.int64, device=dev)
    out["allgather_dense_world1_us"] = timed(lambda: dist.all_gather_into_tensor(dense, h))
    # the whole exchange through the C ABI (cb_hits_allgather on the library's
    # own RCCL communicator), world size 1, on torch's current stream
    from lsmt_amd.shard import Comm
    c = Comm(0, 1, 0, Comm.unique_id())
    s = torch.cuda.current_stream(dev).cuda_stream
    full1 = torch.empty((rows, words), dtype=torch.int64, device=dev)
    ok = torch.ones(1, dtype=torch.int32, device=dev)
    out["capi_dense_world1_us"] = timed(lambda: c.allgather(h, rows, full1, stream=s))
    out["capi_sparse_world1_us"] = timed(lambda: c.allgather(h, rows, full1, sparse=True, cap=cap, ok=ok, stream=s))
    assert int(ok.item()) == 1 and torch.equal(full1, h)
    c.close()
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
