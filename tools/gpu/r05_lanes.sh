#!/bin/bash
# Round 5: the C3 headline on three and four lanes made three ways: the
# current stream plus pool streams (as is), pool streams only, and
# hipStreamCreate streams (BENCH_LANES, a knob of bench.py at 6851b9c..c6ec882's
# successor, removed after this A/B: all within 34.9-36.5 us), two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  for P in 3 4; do
    for v in asis pool raw; do
      BENCH_LANES=$v timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-zone --no-flush --probe-streams $P --steps 200 --warmup 10 > $O/lanes_${v}_$P.json 2> $O/lanes_${v}_$P.err || { tail -5 $O/lanes_${v}_$P.err; exit 1; }
      python -c "
import json;d=json.loads(open('$O/lanes_${v}_$P.json').read().strip().splitlines()[-1])
print('$v P=$P', round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']/1e12,4), 'T')"
    done
  done
done
