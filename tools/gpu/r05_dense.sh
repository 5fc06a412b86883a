#!/bin/bash
# Round 5: the dense FilterSet probe (densefs.hip): its parity tests, the C5
# tests, then the C5 leg A/B (k_set_probe vs dense), alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_dense_probe_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_dense.log 2>&1 || { tail -40 $O/pytest_dense.log; exit 1; }
tail -3 $O/pytest_dense.log
for rep in 1 2; do
  for mode in off on; do
    timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 --set-dense $mode > $O/c5_${mode}_$rep.json 2> $O/c5_${mode}_$rep.err || { tail -20 $O/c5_${mode}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/c5_${mode}_$rep.json'))['c5'];r=d['roofline']
print('$mode', d['path'][:20], 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
  done
done
