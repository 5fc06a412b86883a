#!/bin/bash
# Round 4: the partition-pass load fix (k_build_part, scan unrolled again)
# against the last commit's library (build/old): C2 one lane and C4, three
# alternating reps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_build_streams_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_part2.log 2>&1 || { tail -30 gpurun_out/pytest_part2.log; exit 1; }
tail -1 gpurun_out/pytest_part2.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-cpu --no-e2e --no-cold --no-flush --no-c5 --no-wide --no-read --no-zone"
for rep in 1 2 3; do
  for v in old new; do
    L=build/exp/libcassbloom.so
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/pb_${v}_$rep.json 2> gpurun_out/pb_${v}_$rep.err || { tail -5 gpurun_out/pb_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/pb_${v}_$rep.json').read().strip().splitlines()[-1]);b=d['build'];c=d['c4']
print('$v', '| C2 4-lane', round(b['value']/1e9,1), 'one-lane us', b['one_lane']['us_per_build'], b['kernels'], '| C4 us', c.get('region_us_per_step'), c.get('one_lane_us_per_step'))"
  done
done
