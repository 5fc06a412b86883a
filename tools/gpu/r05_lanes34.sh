#!/bin/bash
# Round 5: the C3 headline on three and four lanes, alternating, four reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2 3 4; do
  for P in 3 4; do
    timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-zone --no-flush --probe-streams $P --steps 200 --warmup 20 > $O/l34_$P.json 2> $O/l34_$P.err || { tail -5 $O/l34_$P.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/l34_$P.json').read().strip().splitlines()[-1])
print('P=$P', round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']/1e12,4), 'T')"
  done
done
