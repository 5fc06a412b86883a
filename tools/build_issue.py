"""Host issue time of bench.py's C2 build step (clear + insert_batch on a
lane) against its GPU time: is the pipelined build leg host-bound? Prints
one JSON line. Diagnostic only."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

dev = torch.device("cuda:0")
P = 3
lanes = [torch.cuda.Stream(device=dev) for _ in range(P)]
bk = torch.from_numpy(workload.c2_build_keys(1 << 20)).to(dev)
bfs = [lsmt_amd.BloomFilter(1 << 27, device=0) for _ in range(P)]
bkb = lsmt_amd.DeviceKeys(bk)
no = [0]


def step():
    i = no[0] % P
    no[0] += 1
    bfs[i].clear(stream=lanes[i].cuda_stream)
    bfs[i].insert_batch(bkb, stream=lanes[i].cuda_stream)


for _ in range(20):
    step()
torch.cuda.synchronize()
out = {}
for k in (200, 1000):
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f"k{k}"] = {"issue_us_per_step": round((t1 - t0) / k * 1e6, 2), "wall_us_per_step": round((t2 - t0) / k * 1e6, 2)}
# the pieces
t0 = time.perf_counter()
for _ in range(300):
    bfs[0].clear(stream=lanes[0].cuda_stream)
t1 = time.perf_counter()
torch.cuda.synchronize()
out["clear_us"] = round((t1 - t0) / 300 * 1e6, 2)
# the raw C call (no Python wrapper): lsmt_amd's own ctypes handle
from lsmt_amd._lib import load as _L  # noqa: E402
L = _L()
h = bfs[0]._h
kp = bk.data_ptr()
sp = lanes[0].cuda_stream
t0 = time.perf_counter()
for _ in range(300):
    L.cb_filter_insert_fixed(h, kp, 16, 1 << 20, sp)
t1 = time.perf_counter()
torch.cuda.synchronize()
out["raw_c_insert_us"] = round((t1 - t0) / 300 * 1e6, 2)
t0 = time.perf_counter()
for _ in range(300):
    bfs[0].insert_batch(bkb, stream=sp)
t1 = time.perf_counter()
torch.cuda.synchronize()
out["py_insert_us"] = round((t1 - t0) / 300 * 1e6, 2)
print(json.dumps(out))
