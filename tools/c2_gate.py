"""How the C2 one-lane device time depends on what the GPU did just before
(bench.py gated_steps: K builds queued behind a spin kernel). Three gates,
alternating: (spin) a ~11.7 ms one-wave spin kernel, as the bench does;
(warm) W real builds queued first, the K timed builds issued while the device
still works through them; (warm+spin) a 0.3 s warm-up, then the spin gate.
Prints device us per build for each, and whether the K builds were all queued
before the device reached them. Diagnostic only: `timeout -k 10 300 python tools/c2_gate.py` on the box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

SPIN_CYCLES_PER_US = 2100


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    keys = torch.from_numpy(workload.c2_build_keys(1 << 20)).to(dev)
    kb = lsmt_amd.DeviceKeys(keys)
    f = lsmt_amd.BloomFilter(1 << 27)

    def build():
        f.clear(stream=sh)
        f.insert_batch(kb, stream=sh)

    def spin_gate(k):
        spin_us = 4000 + 120 * k
        e0, e1, es = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        es.record(st)
        torch.cuda._sleep(SPIN_CYCLES_PER_US * spin_us)
        e0.record(st)
        t0 = time.perf_counter()
        for _ in range(k):
            build()
        issue = time.perf_counter() - t0
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e3 / k, issue * 1e3 < es.elapsed_time(e0)

    def warm_gate(k, w):
        e0, e1, es = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        es.record(st)
        for _ in range(w):
            build()
        e0.record(st)
        for _ in range(k):
            build()
        host = time.perf_counter() - t0
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e3 / k, host * 1e3 < es.elapsed_time(e0)

    def warm_up(seconds):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(32):
                build()
            torch.cuda.synchronize(dev)

    warm_up(0.3)
    for rep in range(3):
        print("spin", *spin_gate(64), flush=True)
        print("warm", *warm_gate(64, 600), flush=True)
        warm_up(0.3)
        print("warm+spin", *spin_gate(64), flush=True)
        print("warm(2000)", *warm_gate(64, 2000), flush=True)


if __name__ == "__main__":
    main()
