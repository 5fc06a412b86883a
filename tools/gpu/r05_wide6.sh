#!/bin/bash
# Round 5: the wide screen at 64, 128 and 256 fingerprint bins
# (CB_SCREEN_HBITS on the experiment build build/xw), the wide tests first.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_wide6.log 2>&1 || { tail -30 $O/pytest_wide6.log; exit 1; }
tail -1 $O/pytest_wide6.log
for rep in 1 2; do
  for h in 6 7 8; do
    CB_SCREEN_HBITS=$h EXPBENCH_LIB=build/xw/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --no-cpu --steps 20 --warmup 2 > $O/w6_h$h.json 2> $O/w6_h$h.err || { tail -20 $O/w6_h$h.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/w6_h$h.json').read().strip().splitlines()[-1])['wide_fanout']
print('hbits $h', round(d['value']/1e9,3), 'G gets/s', d['kernels_us'], d.get('oracle_sample_bit_exact'))"
  done
done
