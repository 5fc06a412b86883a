#!/bin/bash
# Round 5: the dense probe after the partition-pass rework (block scan, block-
# major run table): its tests, then the C5 leg for the product library, the
# eight-wave partition build (CB_DENSE_PART_LB8), and timing-only variants of
# the experiment build (CB_DENSE_X=1 no set[b] gathers, 2 no hit atomics).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_dense_probe_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dense2.log 2>&1 || { tail -40 $O/pytest_dense2.log; exit 1; }
tail -1 $O/pytest_dense2.log
show() {
python -c "
import json;d=json.load(open('$1'))['c5'];r=d['roofline']
print('$2', 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'))"
}
for rep in 1 2; do
  timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5b_prod_$rep.json 2> $O/c5b_prod_$rep.err || { tail -20 $O/c5b_prod_$rep.err; exit 1; }
  show $O/c5b_prod_$rep.json "product"
  EXPBENCH_LIB=build/expr5lb8/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5b_lb8_$rep.json 2> $O/c5b_lb8_$rep.err || { tail -20 $O/c5b_lb8_$rep.err; exit 1; }
  show $O/c5b_lb8_$rep.json "lb8"
done
for x in 1 2 3; do
  CB_DENSE_X=$x EXPBENCH_LIB=build/expr5/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5b_x$x.json 2> $O/c5b_x$x.err || { tail -20 $O/c5b_x$x.err; exit 1; }
  show $O/c5b_x$x.json "x$x(timing only)"
done
