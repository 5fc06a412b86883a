#!/bin/bash
# Flush sort tests, then the flush leg at the default group target and at CB_BIN_T values in TS.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flush_gpu.py \
  > gpurun_out/pytest_flush.log 2>&1 || { tail -60 gpurun_out/pytest_flush.log; exit 1; }
tail -1 gpurun_out/pytest_flush.log
for T in auto ${TS}; do
  if [ "$T" = auto ]; then unset CB_BIN_T; else export CB_BIN_T=$T; fi
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone --no-read --steps 40 > gpurun_out/fl_$T.json 2> gpurun_out/fl_$T.err || { tail -30 gpurun_out/fl_$T.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/fl_$T.json'));f=d['flush']
print('T=$T', 'sorted', f['sorted_input']['ms_per_flush'], 'unsorted', f['unsorted_input']['ms_per_flush'], f['unsorted_input']['kernels_us'])"
done
