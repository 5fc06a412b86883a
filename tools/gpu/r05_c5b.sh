#!/bin/bash
# Round 5: dense probe with the run table transposed between the passes:
# tests, then the C5 leg dense vs k_set_probe, alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_dense_probe_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dense3.log 2>&1 || { tail -40 $O/pytest_dense3.log; exit 1; }
tail -1 $O/pytest_dense3.log
show() {
python -c "
import json;d=json.load(open('$1'))['c5'];r=d['roofline']
print('$2', 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
}
for rep in 1 2; do
  for mode in on off; do
    timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 --set-dense $mode > $O/c5c_${mode}_$rep.json 2> $O/c5c_${mode}_$rep.err || { tail -20 $O/c5c_${mode}_$rep.err; exit 1; }
    show $O/c5c_${mode}_$rep.json "$mode"
  done
done
for x in 2 3; do
  CB_DENSE_X=$x EXPBENCH_LIB=build/expr5/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5c_x$x.json 2> $O/c5c_x$x.err || { tail -20 $O/c5c_x$x.err; exit 1; }
  show $O/c5c_x$x.json "x$x(timing only)"
done
