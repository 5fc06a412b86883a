#!/bin/bash
# Round 4: the wide walk with 8 against 16 summary words screened at once
# (build/exp8, build/exp16).
set -o pipefail
mkdir -p gpurun_out
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-e2e --no-cold --no-flush --no-c4 --no-c5 --no-read --no-zone --no-cpu"
for rep in 1 2; do
  for v in 8 16; do
    EXPBENCH_LIB=build/exp$v/libcassbloom.so timeout -k 10 300 $B > gpurun_out/ws_${v}_$rep.json 2> gpurun_out/ws_${v}_$rep.err || { tail -5 gpurun_out/ws_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ws_${v}_$rep.json').read().strip().splitlines()[-1]);w=d['wide_fanout']
print('screen $v', 'wide', round(w['value']/1e6,1), 'M', w.get('kernels_us'))"
  done
done
