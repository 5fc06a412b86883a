#!/bin/bash
# Round 5: the default line's one-lane C2 build after the cold legs, with and
# without releasing their eviction buffers (BENCH_KEEP_COLD_CACHE), two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  for v in release keep; do
    env=""; [ $v = keep ] && env="BENCH_KEEP_COLD_CACHE=1"
    env $env timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-c4 --no-c5 --no-wide > $O/c2cold_$v.json 2> $O/c2cold_$v.err || { tail -5 $O/c2cold_$v.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/c2cold_$v.json').read().strip().splitlines()[-1]);b=d['build']
print('$v', 'one lane', b['one_lane']['us_per_build'], 'cold', b['cold']['ms_per_step']*1e3, 'clean', b['cold']['clean_caches']['ms_per_step']*1e3, '4 lanes', b['ms_per_step']*1e3)"
  done
done
