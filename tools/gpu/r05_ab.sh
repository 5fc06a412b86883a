#!/bin/bash
# Round 5: the dense FilterSet probe (densefs.hip) and the wide walk's screen:
# their parity tests, then the C5 leg A/B (k_set_probe vs dense) and the wide
# fan-out A/B (experiment build with CB_NO_SCREEN=1 vs the product), alternating.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_dense_probe_gpu.py tests/test_wide_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
tail -3 $O/pytest_ab.log
for rep in 1 2; do
  for mode in off on; do
    timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 --set-dense $mode > $O/c5_${mode}_$rep.json 2> $O/c5_${mode}_$rep.err || { tail -20 $O/c5_${mode}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/c5_${mode}_$rep.json'))['c5'];r=d['roofline']
print('c5 $mode', d['path'][:20], 'region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
  done
  for v in noscreen screen; do
    if [ $v = noscreen ]; then
      CB_NO_SCREEN=1 EXPBENCH_LIB=build/expr5/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --steps 10 --warmup 2 > $O/wide_${v}_$rep.json 2> $O/wide_${v}_$rep.err || { tail -20 $O/wide_${v}_$rep.err; exit 1; }
    else
      timeout -k 10 300 python bench.py --leg wide --steps 10 --warmup 2 > $O/wide_${v}_$rep.json 2> $O/wide_${v}_$rep.err || { tail -20 $O/wide_${v}_$rep.err; exit 1; }
    fi
    python -c "
import json;d=json.load(open('$O/wide_${v}_$rep.json'))['wide_fanout']
print('wide $v', round(d['value']/1e6,1), 'M gets/s', d['kernels_us'], 'oracle', d.get('oracle_sample_bit_exact'))"
  done
done
