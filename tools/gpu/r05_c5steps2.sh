#!/bin/bash
# Round 5: the C5 leg alone at 20 and 200 timed steps, alternating.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1])['c5']
print('$2', d['region_us_per_step'], d['one_lane_us_per_step'], d['steps'], d['kernels_us'])"
}
for rep in 1 2; do
  for st in 20 200 60; do
    timeout -k 10 200 python bench.py --leg c5 --no-cpu --steps $st --warmup 3 > $O/c5s2_$st.json 2> $O/c5s2_$st.err || { tail -5 $O/c5s2_$st.err; exit 1; }
    show $O/c5s2_$st.json "steps $st"
  done
done
