#!/bin/bash
# Read-leg A/B over prebuilt library variants (variants/*.so), with 1 and 2
# pipeline lanes; the library is swapped in the box's copy of the tree.
set -o pipefail
mkdir -p gpurun_out
for v in variants/*.so; do
  cp "$v" lsmt_amd/libcassbloom.so
  timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread  > gpurun_out/rv_test.log 2>&1 || { tail -30 gpurun_out/rv_test.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/rv_test.log)"
  for lanes in ${LANES:-1 2}; do
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush --probe-streams $lanes > gpurun_out/rv.json 2> gpurun_out/rv.err || { tail -20 gpurun_out/rv.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/rv.json'));r=d['read_path'];print('$v lanes=$lanes',round(r['value']/1e9,2),r['ms_per_step'],r['kernels_us'])"
  done
done
