#!/bin/bash
# Round 5: the C3 headline with the set words read by plain or non-temporal
# loads (experiment builds build/xnt0, build/xnt1: CB_SET_NT_LOADS),
# alternating, four reps. (The knob was removed after this A/B: no difference.)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2 3 4; do
  for v in 0 1; do
    EXPBENCH_LIB=build/xnt$v/libcassbloom.so timeout -k 10 200 python tools/expbench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-zone --no-flush --steps 200 --warmup 20 > $O/snt_$v.json 2> $O/snt_$v.err || { tail -5 $O/snt_$v.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/snt_$v.json').read().strip().splitlines()[-1])
print('nt=$v', round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']/1e12,4), 'T', d['roofline'].get('kernel_avg_us_one_lane'))"
  done
done
