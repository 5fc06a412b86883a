#!/bin/bash
# Round 4: the wide read path's candidate prefetch depth (bucket summary
# words loaded for 1, 2 or 4 candidates at once), alternating on one box.
set -o pipefail
mkdir -p gpurun_out
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-cpu --no-e2e --no-cold --no-flush --no-c4 --no-c5 --no-read --no-zone"
for rep in 1 2; do
  for v in pre1 pre2 pre4; do
    if [ $v = pre4 ]; then L=lsmt_amd/libcassbloom.so; else L=build/$v/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/wp_${v}_$rep.json 2> gpurun_out/wp_${v}_$rep.err || { tail -5 gpurun_out/wp_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/wp_${v}_$rep.json'));w=d['wide_fanout']
print('$v', 'wide', round(w['value']/1e6,1), 'M', w.get('kernels_us'), w.get('oracle_sample_bit_exact'))"
  done
done
