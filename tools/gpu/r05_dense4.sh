#!/bin/bash
# Round 5: the dense probe with three batches of four keys per partition
# thread (C = 12288): its tests, the C5 exchange tests, then the C5 leg twice.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_dense_probe_gpu.py tests/test_comm_multirank_gpu.py tests/test_bench_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dense4.log 2>&1 || { tail -40 $O/pytest_dense4.log; exit 1; }
tail -1 $O/pytest_dense4.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5d4_$rep.json 2> $O/c5d4_$rep.err || { tail -20 $O/c5d4_$rep.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/c5d4_$rep.json'))['c5'];r=d['roofline']
print('region', d['region_us_per_step'], 'one-lane', d['one_lane_us_per_step'], 'frac', r['frac'], d.get('kernels_us'), 'golden', d.get('golden_slice_bit_exact'), 'oracle', d.get('oracle_row_bit_exact'))"
done
