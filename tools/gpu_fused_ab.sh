#!/bin/bash
# A/B of k_set_get_many variants (env CB_FUSED_VAR) on the read leg.
# Usage: bash tools/gpu_fused_ab.sh "v1 v2 ..." [reps] [lanes]
set -o pipefail
mkdir -p gpurun_out/fab
VALS=$1; R=${2:-2}; LN=${3:-1}
for v in $VALS; do
  CB_FUSED_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py -m gpu -x -q -k set_get_many --timeout 120 --timeout-method thread > gpurun_out/fab/pytest_$v.log 2>&1 || { echo "tests var=$v failed"; tail -30 gpurun_out/fab/pytest_$v.log; exit 1; }
  echo "var=$v $(tail -1 gpurun_out/fab/pytest_$v.log)"
done
for r in $(seq $R); do for v in $VALS; do
  CB_FUSED_VAR=$v timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush --steps 100 --probe-streams $LN > gpurun_out/fab/b_$v.json 2> gpurun_out/fab/b_$v.err || { tail -20 gpurun_out/fab/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fab/b_$v.json'))['read_path'];f=d['forms']['fused'];print('var=$v rep $r', round(f['value']/1e9,3), f['kernels_us'], d['fused_equals_two_step'])"
done; done
