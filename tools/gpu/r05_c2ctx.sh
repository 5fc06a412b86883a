#!/bin/bash
# Round 5: which earlier leg of the default line slows its one-lane C2 build
# (15.4-15.5 us with the zone, read and flush legs off, 16.5 in the full line)?
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
i=0
for extra in "" "--no-flush" "--no-zone" "--no-read" "--no-zone --no-flush"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide $extra > $O/c2ctx_$i.json 2> $O/c2ctx_$i.err || { tail -5 $O/c2ctx_$i.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/c2ctx_$i.json').read().strip().splitlines()[-1]);b=d['build']
print('line $extra', 'one lane', b['one_lane']['us_per_build'], 'issued', b['one_lane']['host_issued_us_per_build'], '4 lanes', b['ms_per_step']*1e3)"
done
