#!/bin/bash
# Round 5: the dense probe's run table written straight from the partition
# pass (XCD-dealt blocks, experiment build CB_DENSE_DIRECT=1) against the
# transpose kernel (product), alternating; then the C5 rocprofv3 evidence.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.load(open('$1'))['c5'];r=d['roofline']
print('$2', 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
}
for rep in 1 2; do
  timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5d_prod_$rep.json 2> $O/c5d_prod_$rep.err || { tail -20 $O/c5d_prod_$rep.err; exit 1; }
  show $O/c5d_prod_$rep.json "segT-kernel"
  CB_DENSE_DIRECT=1 EXPBENCH_LIB=build/expr5/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5d_direct_$rep.json 2> $O/c5d_direct_$rep.err || { tail -20 $O/c5d_direct_$rep.err; exit 1; }
  show $O/c5d_direct_$rep.json "direct"
done
PROF_OUT=$O/prof_c5 bash tools/profile_round.sh c5 > $O/prof_c5.log 2>&1 || { tail -20 $O/prof_c5.log; exit 1; }
tail -12 $O/prof_c5.log
