"""Which registered stream makes the mirror refresh wait for an unrelated
busy stream? (round-6 debugging of wait_known_streams)."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import lsmt_amd as gpu  # noqa: E402
from lsmt_amd import workload  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def busy_stream():
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(raw), 1) == 0
    st = torch.cuda.ExternalStream(raw.value)
    with torch.cuda.stream(st):
        torch.cuda._sleep(2_000_000_000)
        done = torch.cuda.Event()
        done.record(st)
    return st, done, raw


def trial(tag, pre):
    m = 1 << 26
    keys = workload.key_range(61, 100_000)
    b = gpu.BloomFilter(m)
    b.host_mirror(0)
    pre()
    wr = torch.cuda.Stream()
    b.insert_batch(gpu.DeviceKeys(torch.from_numpy(keys).cuda()), stream=wr)
    torch.cuda.synchronize()
    st, done, raw = busy_stream()
    b.host_mirror(1)
    t0 = time.perf_counter()
    b.may_contain(bytes(keys[0]))
    t1 = time.perf_counter()
    sb = not done.query()
    st.synchronize()
    t2 = time.perf_counter()
    print(f"{tag}: refresh {1e3 * (t1 - t0):.1f} ms, busy still running {sb}, spin left {1e3 * (t2 - t1):.0f} ms",
          flush=True)
    hip.hipStreamDestroy(raw)


trial("fresh", lambda: None)
trial("after null-stream call", lambda: gpu.BloomFilter(1 << 20).insert_batch(workload.key_range(1, 1000)))
ts = torch.cuda.Stream()
trial("after a pool-stream call", lambda: gpu.BloomFilter(1 << 20).insert_batch(workload.key_range(1, 1000),
                                                                               stream=ts.cuda_stream))
