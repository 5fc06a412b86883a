#!/bin/bash
# Round-3 check on one box: the new world>1 / may_contain / zone-update tests
# first, then the whole GPU suite, then one default bench line.
# Usage: bash tools/gpu_r03.sh [new|all|bench]...   (default: new all bench)
set -o pipefail
mkdir -p gpurun_out
steps=${*:-new all bench}
for st in $steps; do
  case $st in
    new)
      timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
        tests/test_may_contain_gpu.py tests/test_comm_multirank_gpu.py tests/test_zone_gpu.py \
        tests/test_exchange_gpu.py > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
      tail -2 gpurun_out/pytest_new.log ;;
    all)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
      tail -2 gpurun_out/pytest_gpu.log ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
      cat gpurun_out/bench.json | head -c 600; echo ;;
  esac
done
