#!/bin/bash
# Round 5: the dense partition pass at two workgroups per CU (eight waves per
# SIMD: fewer keys per thread so it fits 64 VGPRs) against one per CU,
# experiment builds build/xk*w*, alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.load(open('$1'))['c5'];r=d['roofline']
print('$2', 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
}
for rep in 1 2; do
  for v in k7w1 k5w8 k6w8 k4w8; do
    EXPBENCH_LIB=build/x$v/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5p_${v}_$rep.json 2> $O/c5p_${v}_$rep.err || { tail -20 $O/c5p_${v}_$rep.err; exit 1; }
    show $O/c5p_${v}_$rep.json "$v"
  done
done
