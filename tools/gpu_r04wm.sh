#!/bin/bash
# Round 4: the wide walk without staging each group's 64 DirMaps in LDS (the
# directory search reading its table's map in place) against the last commit's
# library (build/old), alternating. Measured slower (751-771 against 765-800 M
# gets/s); the change was not kept.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py tests/test_sstable_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wm.log 2>&1 || { tail -30 gpurun_out/pytest_wm.log; exit 1; }
tail -1 gpurun_out/pytest_wm.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-e2e --no-cold --no-flush --no-c4 --no-c5 --no-read --no-zone"
for rep in 1 2 3; do
  for v in old new; do
    L=build/exp/libcassbloom.so
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/wm_${v}_$rep.json 2> gpurun_out/wm_${v}_$rep.err || { tail -5 gpurun_out/wm_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/wm_${v}_$rep.json').read().strip().splitlines()[-1]);w=d['wide_fanout']
print('$v', 'wide', round(w['value']/1e6,1), 'M', w.get('oracle_sample_bit_exact'), w.get('kernels_us'))"
  done
done
