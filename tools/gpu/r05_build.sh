#!/bin/bash
# Round 5: the C2 build leg with device-resident timing (steps queued behind a
# spin kernel), two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-c4 --no-c5 --no-wide --no-zone --no-read --no-flush > $O/bld_$rep.json 2> $O/bld_$rep.err || { tail -20 $O/bld_$rep.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bld_$rep.json'));b=d['build']
print('C2 4-lane', b['region_us_per_step'], 'one-lane', json.dumps(b['one_lane']), 'cold', b['cold']['ms_per_step'], b['cold']['kernels_us'], 'clean', b['cold']['clean_caches']['ms_per_step'])
print('C3 cold', d['cold']['ms_per_step'], 'clean', d['cold']['clean_caches']['ms_per_step'], 'value', d['value'])"
done
