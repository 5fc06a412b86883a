"""Where a device SsTable::create's time goes (bench.py's flush leg, sorted
1M-entry input): the C call alone, the zone-bound key fetch, and the release
of an older table. Host perf_counter around each piece, median of 20, after
a stream sync. Diagnostic only; prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402
from lsmt_amd._lib import load as _L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n = 1 << 20
    fk = workload.sort_keys16(workload.key_range(7000, n))
    fv = workload.table_value(fk, 1)
    kd = torch.from_numpy(np.ascontiguousarray(fk.reshape(-1))).to(dev)
    vd = torch.from_numpy(np.ascontiguousarray(fv.reshape(-1))).to(dev)
    ko = torch.from_numpy(np.arange(0, 16 * (n + 1), 16, dtype=np.int64)).to(dev)
    kb = lsmt_amd.KeyBatch(n=n, data=kd, offsets=ko)
    vb = lsmt_amd.KeyBatch(n=n, data=vd, offsets=ko)
    torch.cuda.synchronize()
    L = _L()
    res = {}

    def med(xs):
        return round(float(np.median(xs)) * 1e6, 1)

    # 1. the C call alone, tables kept alive
    keep, t_c = [], []
    for _ in range(25):
        th, fh = ctypes.c_void_p(), ctypes.c_void_p()
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        t0 = time.perf_counter()
        rc = L.cb_sstable_create(kd.data_ptr(), ko.data_ptr(), vd.data_ptr(), ko.data_ptr(), n, 1 << 26, 0, None,
                                 ctypes.byref(th), ctypes.byref(fh), ctypes.byref(lo), ctypes.byref(hi))
        t_c.append(time.perf_counter() - t0)
        assert rc == 0
        keep.append((th.value, fh.value))
    res["c_call_us"] = med(t_c[5:])
    # 2. the Python wrapper (C call + zone key fetch), tables kept
    made, t_py = [], []
    for _ in range(25):
        t0 = time.perf_counter()
        made.append(lsmt_amd.sstable_create((kb, vb), m=1 << 26))
        t_py.append(time.perf_counter() - t0)
    res["python_create_us"] = med(t_py[5:])
    # 3. releasing one table + filter
    t_rel = []
    for th, fh in keep[:20]:
        t0 = time.perf_counter()
        L.cb_table_destroy(ctypes.c_void_p(th))
        L.cb_filter_destroy(ctypes.c_void_p(fh))
        t_rel.append(time.perf_counter() - t0)
    res["release_us"] = med(t_rel)
    # 4. one empty device sync, for scale
    t_s = []
    for _ in range(20):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t_s.append(time.perf_counter() - t0)
    res["sync_us"] = med(t_s)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
