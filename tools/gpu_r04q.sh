#!/bin/bash
# Round 4: persistent partition pass (k_build_part_loop) for batched builds
# (k_build_part_loop was removed after this A/B: profiles/part_loop_ab_r04.json)
# with more partition blocks than fit at once — build parity, then C4 A/B
# (CB_BUILD_LOOP=0: k_build_part) with every filter's golden check.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_build_streams_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_loop.log 2>&1 || { tail -30 gpurun_out/pytest_loop.log; exit 1; }
tail -1 gpurun_out/pytest_loop.log
C4_SWEEP_CHECK=1 timeout -k 10 600 python tools/c4_sweep.py 100 '[{"CB_BUILD_LOOP": "0"}, {}, {"CB_BUILD_LOOP": "0"}, {}]' > gpurun_out/c4_loop.jsonl 2> gpurun_out/c4_loop.err || { tail -5 gpurun_out/c4_loop.err; exit 1; }
cat gpurun_out/c4_loop.jsonl
