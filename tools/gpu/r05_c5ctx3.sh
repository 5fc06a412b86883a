#!/bin/bash
# Round 5: the default line's C5 (after C4) on different lane streams:
# current + 2 torch pool streams (as is), the line's own lanes, 3 fresh
# pool streams, 3 hipStreamCreate streams (BENCH_C5_LANES), two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);c=d['c5'];c4=d['c4']
print('$2', 'c5', c['region_us_per_step'], c['one_lane_us_per_step'], 'c4', c4['region_us_per_step'], 'c3', d['ms_per_step'])"
}
for rep in 1 2; do
  for v in asis global fresh raw; do
    BENCH_C5_LANES=$v timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold --no-zone --no-flush --no-wide > $O/c5ctx3_$v.json 2> $O/c5ctx3_$v.err || { tail -5 $O/c5ctx3_$v.err; exit 1; }
    show $O/c5ctx3_$v.json "$v"
  done
done
