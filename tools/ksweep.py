"""The C3 FilterSet step timed the way bench.py times it, at several K:
where the per-step cost at small K (the driver runs K = 20) goes. Per-step
HIP events on each lane show whether the first steps of a region run slower
than the steady state, or whether the region's ends (fill, drain) cost it."""
import json
import os
import sys
import time

if os.environ.get("SPIN") == "1":  # hipDeviceScheduleSpin before the runtime creates its context
    import ctypes
    ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(1)
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

dev = torch.device("cuda:0")
import os
F, m, kpf, n = 32, 1 << 26, 1 << 19, 1 << 20
P = int(os.environ.get("LANES", "3"))
stream = torch.cuda.current_stream(dev)
filters = []
for f in range(F):
    keys = torch.from_numpy(workload.key_range(11 + f, kpf)).to(dev)
    b = lsmt_amd.BloomFilter(m, device=0)
    b.insert_batch(lsmt_amd.DeviceKeys(keys), stream=stream.cuda_stream)
    filters.append(b)
look = torch.from_numpy(workload.probe_lookups(n, F, kpf, seed_base=11, absent_seed=999)).to(dev)
kb = lsmt_amd.DeviceKeys(look)
fset = lsmt_amd.FilterSet(m, width=32, device=0)
fset.assign_all(filters, stream=stream.cuda_stream)
lanes = [stream] + [torch.cuda.Stream(device=dev) for _ in range(P - 1)]
hits = [torch.zeros((F, n // 64), dtype=torch.int64, device=dev) for _ in range(P)]
no = [0]


def step(ev=None):
    i = no[0] % P
    no[0] += 1
    if ev is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record(lanes[i])
        ev.append((i, e))
    fset.probe(kb, out=hits[i], stream=lanes[i].cuda_stream)
    if ev is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record(lanes[i])
        ev.append((i, e))


def region(k, warm, per_step=False, waits=True):
    for _ in range(warm):
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev = [] if per_step else None
    t0 = time.perf_counter()
    e0.record(stream)
    if waits:
        for st in lanes[1:]:
            st.wait_stream(stream)
    t_issue0 = time.perf_counter()
    for _ in range(k):
        step(ev)
    t_issue = time.perf_counter() - t_issue0
    for st in lanes[1:]:
        stream.wait_stream(st)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    out = {"spin": os.environ.get("SPIN") == "1", "lanes": P, "k": k, "waits": waits, "wall_us_per_step": round(wall / k * 1e6, 2),
           "region_us_per_step": round(e0.elapsed_time(e1) * 1e3 / k, 2),
           "issue_us_per_step": round(t_issue / k * 1e6, 2)}
    if per_step:
        out["step_us"] = [round(ev[2 * j][1].elapsed_time(ev[2 * j + 1][1]) * 1e3, 1) for j in range(k)]
        out["start_us"] = [round(e0.elapsed_time(ev[2 * j][1]) * 1e3, 1) for j in range(k)]
    return out


res = []
for k in (20, 200, 20, 20, 20):
    res.append(region(k, 5, waits=False))
res.append(region(20, 5, per_step=True, waits=False))
for r in res:
    print(json.dumps(r))
