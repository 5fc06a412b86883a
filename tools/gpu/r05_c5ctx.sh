#!/bin/bash
# Round 5: which earlier leg of the default line slows its C5 leg (201-206 us
# there against 186-194 us for the leg alone)?
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1])['c5']
print('$2', d['region_us_per_step'], d['one_lane_us_per_step'], d['steps'], d['kernels_us'])"
}
i=0
for extra in "" "--no-zone" "--no-flush" "--no-c4" "--no-wide" "--no-zone --no-flush --no-c4 --no-wide"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold $extra > $O/c5ctx_$i.json 2> $O/c5ctx_$i.err || { tail -5 $O/c5ctx_$i.err; exit 1; }
  show $O/c5ctx_$i.json "line $extra"
done
