#!/bin/bash
# Round 4: the wide walk at six waves per SIMD (80 VGPRs, 112 B of scratch per
# lane; build/exp6) against five (96 VGPRs, 36 B; build/exp), alternating.
# Measured slower (606-617 against 782-804 M gets/s); five kept.
set -o pipefail
mkdir -p gpurun_out
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-e2e --no-cold --no-flush --no-c4 --no-c5 --no-read --no-zone --no-cpu"
for rep in 1 2 3; do
  for v in 5 6; do
    L=build/exp/libcassbloom.so
    if [ $v = 6 ]; then L=build/exp6/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/w6_${v}_$rep.json 2> gpurun_out/w6_${v}_$rep.err || { tail -5 gpurun_out/w6_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/w6_${v}_$rep.json').read().strip().splitlines()[-1]);w=d['wide_fanout']
print('waves $v', 'wide', round(w['value']/1e6,1), 'M', w.get('kernels_us'))"
  done
done
