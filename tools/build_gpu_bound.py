"""Is the pipelined C2 build leg GPU-bound or host-bound? Queues K build
steps (clear + insert_batch, round-robin over P lanes) behind a ~5 ms spin
kernel, so the host has issued every step before the GPU starts any: the
time from the spin's end to the last step's end is then the GPU's own rate.
Beside it, the same K steps issued live (bench.py's leg) and the host's issue
time alone. Prints one JSON line. Diagnostic only."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

dev = torch.device("cuda:0")
K = 200
bk = torch.from_numpy(workload.c2_build_keys(1 << 20)).to(dev)
bkb = lsmt_amd.DeviceKeys(bk)
out = {}
for P in (1, 2, 3, 4):
    main = torch.cuda.current_stream(dev)
    lanes = [main] + [torch.cuda.Stream(device=dev) for _ in range(P - 1)]
    bfs = [lsmt_amd.BloomFilter(1 << 27, device=0) for _ in range(P)]
    no = [0]

    def step():
        i = no[0] % P
        no[0] += 1
        bfs[i].clear(stream=lanes[i].cuda_stream)
        bfs[i].insert_batch(bkb, stream=lanes[i].cuda_stream)

    for _ in range(3 * P):
        step()
    torch.cuda.synchronize()
    res = {}
    # live: the bench leg's form
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(main)
    for _ in range(K):
        step()
    t1 = time.perf_counter()
    for st in lanes[1:]:
        main.wait_stream(st)
    e1.record(main)
    torch.cuda.synchronize()
    res["live_us_per_step"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
    res["issue_us_per_step"] = round((t1 - t0) * 1e6 / K, 2)
    # queued behind a spin: the GPU's own rate
    torch.cuda._sleep(int(5e6 * 2.1))  # ~5 ms at ~2.1 GHz
    g0 = torch.cuda.Event(enable_timing=True)
    g0.record(main)
    for st in lanes[1:]:
        st.wait_stream(main)
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    t1 = time.perf_counter()
    for st in lanes[1:]:
        main.wait_stream(st)
    g1 = torch.cuda.Event(enable_timing=True)
    g1.record(main)
    torch.cuda.synchronize()
    res["queued_us_per_step"] = round(g0.elapsed_time(g1) * 1e3 / K, 2)
    res["queued_issue_us_per_step"] = round((t1 - t0) * 1e6 / K, 2)
    out[f"lanes{P}"] = res
print(json.dumps(out))
