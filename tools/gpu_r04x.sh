#!/bin/bash
# Round 4: k_format staging a line's interior dwords with plain LDS stores
# (only its first and last dwords ORed in) against the last commit's library
# (build/old), alternating. Measured flat; the change was not kept.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flush_gpu.py tests/test_sstable_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fmt.log 2>&1 || { tail -30 gpurun_out/pytest_fmt.log; exit 1; }
tail -1 gpurun_out/pytest_fmt.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 200 --no-e2e --no-cold --no-zone --no-read --no-c4 --no-c5 --no-wide"
for rep in 1 2 3; do
  for v in old new; do
    L=build/exp/libcassbloom.so
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/fmt_${v}_$rep.json 2> gpurun_out/fmt_${v}_$rep.err || { tail -5 gpurun_out/fmt_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/fmt_${v}_$rep.json').read().strip().splitlines()[-1]);f=d['flush']
print('$v', 'sorted', f['sorted_input']['ms_per_flush'], f['sorted_input']['one_lane']['ms_per_flush'], 'unsorted', f['unsorted_input']['ms_per_flush'], f['unsorted_input']['one_lane']['ms_per_flush'], 'k_format', f['sorted_input']['kernels_us'].get('k_format'), f['unsorted_input']['kernels_us'].get('k_format'), 'exact', f.get('oracle_file_bit_exact'))"
  done
done
