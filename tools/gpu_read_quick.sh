#!/bin/bash
# Read path quick loop: SSTable parity tests, then the gated probe + get_many leg.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py tests/test_zone_gpu.py tests/test_flush_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sst.log 2>&1 || { tail -30 gpurun_out/pytest_sst.log; exit 1; }
tail -1 gpurun_out/pytest_sst.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold > gpurun_out/read.json 2> gpurun_out/read.err || { tail -20 gpurun_out/read.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/read.json'));print(d['read_path']['value']/1e9, d['read_path']['kernels_us'], d['zone_gate']['kernels_us'], d['kernels_us'], d['flush']['sorted_input']['entries_per_s']/1e9, d['flush']['sorted_input']['kernels_us'])"
