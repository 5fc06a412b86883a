#!/bin/bash
# A/B of k_get_many variants (env CB_GM_VAR_NAME=values) on the read leg, one lane.
# Usage: bash tools/gpu_gm_ab.sh ENVNAME "v1 v2 ..." [reps]
set -o pipefail
mkdir -p gpurun_out/ab
E=$1; VALS=$2; R=${3:-2}
for v in $VALS; do
  env $E=$v timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py tests/test_flush_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { echo "tests $E=$v failed"; tail -30 gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "$E=$v $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
for r in $(seq $R); do for v in $VALS; do
  env $E=$v timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush --steps 100 --probe-streams ${LANES:-1} > gpurun_out/ab/b_$v.json 2> gpurun_out/ab/b_$v.err || { tail -20 gpurun_out/ab/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/b_$v.json'))['read_path'];print('$E=$v rep $r', round(d['value']/1e9,3), d['ms_per_step'], d['kernels_us'], d['oracle_sample_bit_exact'])"
done; done
