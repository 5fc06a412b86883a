"""Is bench.py's C4 step (64 builds of 256K keys, m = 2^25, three lanes)
host-bound? Host issue time per step beside the GPU's rate with every step
queued behind a spin kernel first (as tools/build_gpu_bound.py). Diagnostic."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

dev = torch.device("cuda:0")
nf, kpf, m, P, K = 64, 1 << 18, 1 << 25, 3, 30
main = torch.cuda.current_stream(dev)
lanes = [main] + [torch.cuda.Stream(device=dev) for _ in range(P - 1)]
batches = [lsmt_amd.DeviceKeys(torch.from_numpy(workload.c4_filter_keys(f, kpf)).to(dev)) for f in range(nf)]
fsets = [[lsmt_amd.BloomFilter(m, device=0) for _ in range(nf)] for _ in range(P)]
no = [0]
t_clear, t_ins = [0.0], [0.0]


def step():
    i = no[0] % P
    no[0] += 1
    sh = lanes[i].cuda_stream
    a = time.perf_counter()
    for f in fsets[i]:
        f.clear(stream=sh)
    b = time.perf_counter()
    lsmt_amd.insert_many(fsets[i], batches, stream=sh)
    c = time.perf_counter()
    t_clear[0] += b - a
    t_ins[0] += c - b


for _ in range(6):
    step()
torch.cuda.synchronize()
out = {}
t_clear[0] = t_ins[0] = 0.0
t0 = time.perf_counter()
for _ in range(K):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
out["live_us_per_step"] = round((t2 - t0) / K * 1e6, 1)
out["issue_us_per_step"] = round((t1 - t0) / K * 1e6, 1)
out["clear_loop_us"] = round(t_clear[0] / K * 1e6, 1)
out["insert_many_us"] = round(t_ins[0] / K * 1e6, 1)
torch.cuda._sleep(int(20e6 * 2.1))  # ~20 ms
g0 = torch.cuda.Event(enable_timing=True)
g0.record(main)
for st in lanes[1:]:
    st.wait_stream(main)
for _ in range(K):
    step()
for st in lanes[1:]:
    main.wait_stream(st)
g1 = torch.cuda.Event(enable_timing=True)
g1.record(main)
torch.cuda.synchronize()
out["queued_us_per_step"] = round(g0.elapsed_time(g1) * 1e3 / K, 1)
print(json.dumps(out))
