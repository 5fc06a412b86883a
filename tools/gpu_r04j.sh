#!/bin/bash
# Round 4: 16-bit partition entries for batched long-run builds (C4) —
# parity first, phase stamps, then the C4 A/B (experiment library).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_gpu_parity.py tests/test_build_streams_gpu.py -k "c4 or insert_many or build" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1 || { tail -40 gpurun_out/pytest_sub.log; exit 1; }
tail -2 gpurun_out/pytest_sub.log
timeout -k 10 60 ./build/ubench_build c4 > gpurun_out/ub_c4_sub.json && cat gpurun_out/ub_c4_sub.json
timeout -k 10 600 python tools/c4_sweep.py 60 '[{}, {"CB_BUILD_SUB":"0"}, {}, {"CB_BUILD_SUB":"0"}]' > gpurun_out/c4_sub.jsonl 2> gpurun_out/c4_sub.err || { tail -5 gpurun_out/c4_sub.err; exit 1; }
cut -c1-330 gpurun_out/c4_sub.jsonl
