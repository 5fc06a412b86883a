"""Headline line-refetch experiment: does ordering the
lookup batch by set region, so that each region's probes run on one XCD
(workgroup b runs on XCD b mod 8), cut k_set_probe's line fills enough to
pay for itself? The C3 set (32 filters of m = 2^26) probed with the same 1M
keys in three orders, each timed as the bench times the headline (HIP events
around K launches on one stream, and on three lanes):
  - given: the SURVEY.md §8d batch as generated (what the bench probes);
  - xcd: keys bucketed by the top 3 bits of a = h1 % m (8 regions of 32 MB of
    the set) and laid out so 1024-key block b holds keys of region b mod 8:
    every a-read of a block stays in its XCD's region (the b-read is
    independent of a, so it cannot be routed too);
  - sorted_a: keys sorted by a, the best case for a-line reuse (any on-device
    routing is a partition pass, ~5 us, on top of the probe).
The reorder happens on the host before the timed region: this measures the
probe only, i.e. an upper bound on what routing could gain. Usage:
python tools/xcd_order.py [K]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import lsmt_amd
    from lsmt_amd import workload
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    F, m, kpf, n = 32, 1 << 26, 1 << 19, 1 << 20
    filters = []
    for f in range(F):
        b = lsmt_amd.BloomFilter(m)
        b.insert_batch(lsmt_amd.DeviceKeys(torch.from_numpy(workload.c3_filter_keys(f, kpf)).to(dev)))
        filters.append(b)
    fset = lsmt_amd.FilterSet.from_filters(filters)
    look = workload.c3_lookups(n, F, kpf)
    h1 = np.full(n, 5381, np.uint64)
    with np.errstate(over="ignore"):
        for j in range(16):
            h1 = (h1 << np.uint64(5)) + h1 + look[:, j].astype(np.uint64)
    a = (h1 % np.uint64(m)).astype(np.int64)
    region = a >> 23  # 8 regions of 2^23 positions (32 MB of the 32-slot set)
    buckets = [np.flatnonzero(region == r) for r in range(8)]
    per = 1024
    order, ptr = [], [0] * 8
    blk = 0
    while len(order) < n:  # block b takes its keys from region b mod 8 while it lasts
        r = blk % 8
        for rr in [r] + [x for x in range(8) if x != r]:
            if ptr[rr] < len(buckets[rr]):
                take = buckets[rr][ptr[rr]:ptr[rr] + per]
                ptr[rr] += len(take)
                order.extend(take.tolist())
                break
        blk += 1
    xcd = np.asarray(order[:n])
    orders = {"given": np.arange(n), "xcd": xcd, "sorted_a": np.argsort(a, kind="stable")}
    out = {"K": K, "config": "C3: 1M 16-B keys x 32 filters of m=2^26 (FilterSet)", "results": {}}
    lanes = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(2)]
    for name, o in orders.items():
        keys = lsmt_amd.DeviceKeys(torch.from_numpy(np.ascontiguousarray(look[o])).to(dev))
        hits = [torch.zeros((F, n // 64), dtype=torch.int64, device=dev) for _ in lanes]
        res = {}
        for nl in (1, 3):
            step = [0]

            def go():
                i = step[0] % nl
                step[0] += 1
                fset.probe(keys, out=hits[i], stream=lanes[i].cuda_stream)
            for _ in range(10):
                go()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(lanes[0])
            for _ in range(K):
                go()
            for st in lanes[1:nl]:
                lanes[0].wait_stream(st)
            e1.record(lanes[0])
            torch.cuda.synchronize(dev)
            res[f"us_per_step_{nl}_lane"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
        out["results"][name] = res
        print(name, res, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
