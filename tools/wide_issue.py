"""Host issue cost of the wide fan-out step (bench.py wide_fanout_leg: 300
tables of m = 1024 in one wide set, 2^18 lookups, enqueue-only get_many):
per-call host time of lsmt_amd.get_many from Python, of the bare C call
(cb_set_get_many_fixed with its arguments built once), and the device time
per step, so the leg's step time can be read as host- or device-bound.
Diagnostic only: `timeout -k 10 300 python tools/wide_issue.py` on the box."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import lsmt_amd  # noqa: E402
from lsmt_amd import _lib, workload  # noqa: E402
from lsmt_amd.bloom import _ptr_of  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    nt, per, n = 300, 1024, 1 << 18
    rng = np.random.default_rng(300)
    pool = workload.key_range(4242, 120_000)
    tables, blooms, zones = [], [], []
    for t in range(nt):
        idx = np.unique(rng.choice(len(pool), per, replace=False))
        ks = np.ascontiguousarray(pool[idx])
        vs = workload.table_value(ks, t)
        off = np.arange(0, 16 * (len(idx) + 1), 16, dtype=np.uint64)
        kb = lsmt_amd.KeyBatch(n=len(idx), data=ks.reshape(-1), offsets=off)
        vb = lsmt_amd.KeyBatch(n=len(idx), data=np.ascontiguousarray(vs).reshape(-1), offsets=off)
        tb, bloom, zone = lsmt_amd.sstable_create((kb, vb), m=1024, device=0)
        tables.append(tb)
        blooms.append(bloom)
        zones.append(zone)
    fset = lsmt_amd.FilterSet(1024, width=320, device=0)
    for t in range(nt):
        fset.assign(t, blooms[t])
        fset.set_zone(t, zones[t])
    present = pool[rng.integers(0, len(pool), 3 * n // 4)]
    look = np.concatenate([present, workload.key_range(4343, n - len(present))])[rng.permutation(n)]
    keys_t = torch.from_numpy(look).to(dev)
    keys = lsmt_amd.DeviceKeys(keys_t)
    newest = tables[::-1]
    slots = np.arange(nt, dtype=np.uint32)[::-1].copy()
    which = torch.empty(n, dtype=torch.int32, device=dev)
    voff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    vals = torch.empty(n * 16, dtype=torch.uint8, device=dev)

    def py_step():
        lsmt_amd.get_many(newest, keys, filterset=fset, hit_rows=slots, out=(which, voff, vals), stream=sh,
                          wait=False)

    L = _lib.load()
    arr = (ctypes.c_void_p * nt)(*[t.handle.value for t in newest])
    rp = slots.ctypes.data
    kp = _ptr_of(keys_t)[0]
    wp, vo, vp = _ptr_of(which)[0], _ptr_of(voff)[0], _ptr_of(vals)[0]
    cap = int(vals.numel())

    def c_step():
        rc = L.cb_set_get_many_fixed(fset._h, ctypes.cast(arr, ctypes.c_void_p), nt, rp, kp, 16, n, wp, vo, vp,
                                     cap, None, ctypes.c_void_p(sh))
        assert rc == 0

    out = {}
    for label, fn in (("python", py_step), ("c_call", c_step)):
        for _ in range(50):
            fn()
        torch.cuda.synchronize(dev)
        reps = []
        for _ in range(3):
            k = 200
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2100 * 60000)  # a 60 ms gate: the host issues all k calls before the device starts
            e0.record(st)
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            host = (time.perf_counter() - t0) / k * 1e6
            e1.record(st)
            torch.cuda.synchronize(dev)
            reps.append({"host_us_per_call": round(host, 2), "device_us_per_step": round(e0.elapsed_time(e1) * 1e3 / k, 2)})
        out[label] = reps
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
