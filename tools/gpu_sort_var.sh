#!/bin/bash
# Unsorted flush over prebuilt library variants (variants/*.so): flush parity
# tests, then the bench's flush leg, per variant.
set -o pipefail
mkdir -p gpurun_out
for v in variants/*.so; do
  cp "$v" lsmt_amd/libcassbloom.so
  timeout -k 10 300 python -u -m pytest tests/test_flush_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sv_test.log 2>&1 || { tail -30 gpurun_out/sv_test.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/sv_test.log)"
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone --steps 8 > gpurun_out/sv.json 2> gpurun_out/sv.err || { tail -20 gpurun_out/sv.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv.json'));f=d['flush'];print('$v','sorted',f['sorted_input']['ms_per_flush'],'unsorted',f['unsorted_input']['ms_per_flush'],f['unsorted_input']['kernels_us'])"
done
