#!/bin/bash
# Round 5: the wide walk at four waves per SIMD without spill (experiment
# build CB_WIDE_LB4, 109 VGPRs) against the product's five waves (96 VGPRs,
# 56 B of spill per lane), alternating, three reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --leg wide --no-cpu --steps 20 --warmup 2 > $O/w4_prod_$rep.json 2> $O/w4_prod_$rep.err || { tail -20 $O/w4_prod_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/w4_prod_$rep.json'))['wide_fanout'];print('5 waves', round(d['value']/1e6,1), d['kernels_us'])"
  EXPBENCH_LIB=build/expr5w4/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --no-cpu --steps 20 --warmup 2 > $O/w4_exp_$rep.json 2> $O/w4_exp_$rep.err || { tail -20 $O/w4_exp_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/w4_exp_$rep.json'))['wide_fanout'];print('4 waves', round(d['value']/1e6,1), d['kernels_us'])"
done
