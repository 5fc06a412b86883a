#!/bin/bash
# Round 5: the default line's C5 after C4 as is, after torch.cuda.empty_cache(),
# and before C4 (BENCH_EMPTY / BENCH_C5_FIRST), alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);c=d['c5'];c4=d['c4']
print('$2', 'c5', c['region_us_per_step'], c['one_lane_us_per_step'], 'c4', c4['region_us_per_step'])"
}
for rep in 1 2; do
  for v in plain empty first; do
    env=""; [ $v = empty ] && env="BENCH_EMPTY=1"; [ $v = first ] && env="BENCH_C5_FIRST=1"
    env $env timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold --no-zone --no-flush --no-wide > $O/c5ctx2_$v.json 2> $O/c5ctx2_$v.err || { tail -5 $O/c5ctx2_$v.err; exit 1; }
    show $O/c5ctx2_$v.json "$v"
  done
done
