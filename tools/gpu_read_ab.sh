#!/bin/bash
# Read path A/B on one GPU: parity tests with the staged get_many (default),
# then the bench read leg with the staged and the lane-per-search forms.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_flush_gpu.py tests/test_meta_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "get_many or search or sstable or create or table" > gpurun_out/pytest_read.log 2>&1 || { tail -30 gpurun_out/pytest_read.log; exit 1; }
tail -1 gpurun_out/pytest_read.log
for form in staged lane; do
  CB_GET=$form timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush > gpurun_out/bench_read_$form.json 2> gpurun_out/bench_read_$form.err || { tail -20 gpurun_out/bench_read_$form.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_read_$form.json'));r=d['read_path'];print('$form',round(r['value']/1e9,2),r['ms_per_step'],r['kernels_us'])"
done
