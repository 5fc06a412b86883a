"""The product's flush shape: SsTable::create of an auto-flush memtable
(src/lib.rs:72,105: every 1024 inserts; src/sstable.rs:44,59: m = 1024),
16-byte keys and values in HBM, sorted as MemTable::scan hands them over.
Times K enqueue-only creates on one stream (HIP events: the GPU time per
flush) and the host time per call, for n = 1024 and a few other sizes.
Usage: python tools/small_flush.py [K] > out.json"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import lsmt_amd
    from lsmt_amd import workload
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    out = {"K": K, "what": "enqueue-only cb_sstable_create on one stream, sorted 16-B keys and values in HBM",
           "rows": []}
    for n in (1024, 4096, 16384):
        fk = workload.sort_keys16(workload.key_range(7100, n))
        fv = workload.table_value(fk, 1)
        kd = torch.from_numpy(np.ascontiguousarray(fk.reshape(-1))).to(dev)
        vd = torch.from_numpy(np.ascontiguousarray(fv.reshape(-1))).to(dev)
        ko = torch.from_numpy(np.arange(0, 16 * (n + 1), 16, dtype=np.int64)).to(dev)
        kb = lsmt_amd.KeyBatch(n=n, data=kd, offsets=ko)
        vb = lsmt_amd.KeyBatch(n=n, data=vd, offsets=ko)
        made = []
        for _ in range(20):
            made.append(lsmt_amd.sstable_create((kb, vb), m=1024, stream=st, wait=False))
        for t, _, _ in made:
            t.wait()
        made.clear()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        h0 = time.perf_counter()
        for _ in range(K):
            made.append(lsmt_amd.sstable_create((kb, vb), m=1024, stream=st, wait=False))
        h1 = time.perf_counter()
        e1.record(st)
        torch.cuda.synchronize(dev)
        for t, _, _ in made:
            t.wait()
        # one create followed by its wait: the latency a flush thread sees
        lat = []
        for _ in range(20):
            a = time.perf_counter()
            t, _, _ = lsmt_amd.sstable_create((kb, vb), m=1024, stream=st, wait=True)
            lat.append(time.perf_counter() - a)
        row = {"n": n, "gpu_us_per_flush": round(e0.elapsed_time(e1) * 1e3 / K, 2),
               "host_us_per_enqueue": round((h1 - h0) * 1e6 / K, 2),
               "us_create_and_wait_median": round(sorted(lat)[len(lat) // 2] * 1e6, 1)}
        out["rows"].append(row)
        print(row, file=sys.stderr, flush=True)
        made.clear()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
