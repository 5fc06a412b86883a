#!/bin/bash
# A/B of a kernel variant chosen by an environment variable, on the read leg:
# the fused-path parity tests under each value, then alternating bench runs.
# Usage: bash tools/gpu_env_ab.sh ENVNAME "v1 v2 ..." [reps] [lanes]
set -o pipefail
mkdir -p gpurun_out/ab
E=$1; VALS=$2; R=${3:-2}; LN=${4:-1}
for v in $VALS; do
  env $E=$v timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py -m gpu -x -q -k "set_get_many or get_many_golden" --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { echo "tests $E=$v failed"; tail -30 gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "$E=$v $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
for r in $(seq $R); do for v in $VALS; do
  env $E=$v timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush --steps 100 --probe-streams $LN > gpurun_out/ab/b_$v.json 2> gpurun_out/ab/b_$v.err || { tail -20 gpurun_out/ab/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/b_$v.json'))['read_path'];f=d['forms']['fused'];print('$E=$v rep $r', round(f['value']/1e9,3), f['kernels_us'], d['fused_equals_two_step'])"
done; done
