#!/bin/bash
# Round 5: standalone C4 / C5 legs with a short and a long warm-up (does the
# chip's clock ramp explain why a leg run alone measures slower than the same
# leg inside the default line?).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  for w in 5 3000; do
    timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 50 --warmup $w --probe-streams 1 > $O/warm_c4_$w.json 2> $O/warm_c4_$w.err || { tail -5 $O/warm_c4_$w.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/warm_c4_$w.json').read().strip().splitlines()[-1])
c=d.get('c4',d); print('c4 warmup $w', c.get('region_us_per_step'), c.get('one_lane_us_per_step'))"
  done
  for w in 3 1000; do
    timeout -k 10 300 python bench.py --leg c5 --no-cpu --steps 20 --warmup $w > $O/warm_c5_$w.json 2> $O/warm_c5_$w.err || { tail -5 $O/warm_c5_$w.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/warm_c5_$w.json').read().strip().splitlines()[-1])['c5']
print('c5 warmup $w', d['region_us_per_step'], d['one_lane_us_per_step'])"
  done
done
