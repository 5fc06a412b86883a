#!/bin/bash
# The flush sort tests, then the bench's flush leg with group targets T.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flush_gpu.py \
  > gpurun_out/pytest_flush.log 2>&1 || { tail -60 gpurun_out/pytest_flush.log; exit 1; }
tail -2 gpurun_out/pytest_flush.log
for T in ${TS:-2048 3840 0}; do
  CB_BIN_T=$T timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone --steps 40 > gpurun_out/bench_sort_$T.json 2> gpurun_out/bench_sort_$T.err || { tail -30 gpurun_out/bench_sort_$T.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_sort_$T.json'));f=d['flush']
print('T=$T', 'sorted', f['sorted_input']['ms_per_flush'], 'unsorted', f['unsorted_input']['ms_per_flush'], f['unsorted_input']['kernels_us'])"
done
