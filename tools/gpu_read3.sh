#!/bin/bash
# SSTable / read-path parity, then the bench's read leg and flush leg.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sstable_gpu.py \
  tests/test_flush_gpu.py tests/test_meta_gpu.py > gpurun_out/pytest_read.log 2>&1 || { tail -60 gpurun_out/pytest_read.log; exit 1; }
tail -2 gpurun_out/pytest_read.log
timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold --steps 100 > gpurun_out/bench_read.json 2> gpurun_out/bench_read.err || { tail -30 gpurun_out/bench_read.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_read.json'));r=d['read_path']
print('probe',d['value'],'read',r['value'],r['form'],r['kernels_us'],r['fused_equals_two_step'])
print({k:(v['value'],v['kernels_us']) for k,v in r['forms'].items()})
f=d['flush'];print('flush',f['sorted_input']['ms_per_flush'],f['unsorted_input']['ms_per_flush'],f['sorted_input']['kernels_us'])"
