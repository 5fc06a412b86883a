#!/bin/bash
# Round 5: the multi-rank / exchange / config suites after the dense probe
# joined the fused exchange path.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 1000 python -u -m pytest tests/test_configs_gpu.py tests/test_comm_multirank_gpu.py tests/test_exchange_gpu.py tests/test_bench_multirank_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest_x.log 2>&1 || { tail -40 $O/pytest_x.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest_x.log | tail -60 | cut -c1-150
tail -2 $O/pytest_x.log
