#!/bin/bash
# Read path on one GPU: the SSTable/flush parity tests, then the bench's read
# leg (hash index vs fence index).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_flush_gpu.py tests/test_meta_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_read.log 2>&1 || { tail -30 gpurun_out/pytest_read.log; exit 1; }
tail -1 gpurun_out/pytest_read.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold > gpurun_out/bench_read.json 2> gpurun_out/bench_read.err || { tail -20 gpurun_out/bench_read.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_read.json'));r=d['read_path'];print('read',round(r['value']/1e9,2),r['ms_per_step'],r['kernels_us']);f=d['flush'];print('flush',f['sorted_input']['ms_per_flush'],f['unsorted_input']['ms_per_flush'],f['sorted_input']['kernels_us'])"
