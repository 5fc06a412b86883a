#!/bin/bash
# Round 4: the wide walk screening candidates by bucket summary words loaded
# kScreen at a time (4, and 8 in build/exp8) before their zone gates — wide/read
# parity, then the wide leg against the last commit's library (build/old).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py tests/test_sstable_gpu.py tests/test_zone_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wz.log 2>&1 || { tail -30 gpurun_out/pytest_wz.log; exit 1; }
tail -1 gpurun_out/pytest_wz.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-e2e --no-cold --no-flush --no-c4 --no-c5 --no-read --no-zone"
for rep in 1 2 3; do
  for v in old new new8; do
    L=build/exp/libcassbloom.so
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    if [ $v = new8 ]; then L=build/exp8/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/wz_${v}_$rep.json 2> gpurun_out/wz_${v}_$rep.err || { tail -5 gpurun_out/wz_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/wz_${v}_$rep.json').read().strip().splitlines()[-1]);w=d['wide_fanout']
print('$v', 'wide', round(w['value']/1e6,1), 'M', w.get('oracle_sample_bit_exact'), w.get('kernels_us'))"
  done
done
