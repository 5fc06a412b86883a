#!/bin/bash
# Round 5: the C2 build on four lanes with the fourth lane stream made at the
# line's start (with the others) or at the build leg (BENCH_LATE_BUILD_LANE),
# alternating, three reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2 3; do
  for v in start late; do
    env=""; [ $v = late ] && env="BENCH_LATE_BUILD_LANE=1"
    env $env timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-zone --no-flush > $O/bl_$v.json 2> $O/bl_$v.err || { tail -5 $O/bl_$v.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/bl_$v.json').read().strip().splitlines()[-1]);b=d['build']
print('$v', round(b['value']/1e9,1), 'G keys/s', b['ms_per_step']*1e3, 'us/step, one lane', b['one_lane']['us_per_build'], 'C3', round(d['value']/1e12,4))"
  done
done
