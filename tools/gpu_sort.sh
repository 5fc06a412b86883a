#!/bin/bash
# Unsorted flush on one GPU: the flush parity tests (hand-written sort), then
# the bench's flush leg with the hand-written sort and with rocPRIM's.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flush_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_flush.log 2>&1 || { tail -30 gpurun_out/pytest_flush.log; exit 1; }
tail -1 gpurun_out/pytest_flush.log
for srt in hand rocprim; do
  CB_SORT=$srt timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone --steps 8 > gpurun_out/bench_sort.json 2> gpurun_out/bench_sort.err || { tail -20 gpurun_out/bench_sort.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_sort.json'));f=d['flush'];print('$srt','sorted',f['sorted_input']['ms_per_flush'],'unsorted',f['unsorted_input']['ms_per_flush'],f['unsorted_input']['kernels_us'])"
done
