#!/bin/bash
# Round 4: key-bucket layout with slot 0 whole in the first 32 B — parity
# (read-path tests), then an A/B of the read and wide legs against the
# previous layout (build/old: the last commit's library), alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_wide_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_read2.log 2>&1 || { tail -30 gpurun_out/pytest_read2.log; exit 1; }
tail -1 gpurun_out/pytest_read2.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-cpu --no-e2e --no-cold --no-flush --no-c4 --no-c5"
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=build/old/libcassbloom.so; else L=lsmt_amd/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/bl_${v}_$rep.json 2> gpurun_out/bl_${v}_$rep.err || { tail -5 gpurun_out/bl_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/bl_${v}_$rep.json'));r=d['read_path'];w=d['wide_fanout']
print('$v', 'read', round(r['value']/1e9,3), 'G', r['kernels_us'], r['fused_equals_two_step'], '| wide', round(w['value']/1e6,1), 'M')"
  done
done
