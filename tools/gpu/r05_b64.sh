#!/bin/bash
# Round 5: small base64 values loaded as three 16-B loads (product) against
# seven dword loads (build/xb64: CB_B64_DWORD_LOADS): the SSTable and wide
# tests, then the read path and the wide fan-out, alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 500 python -u -m pytest tests/test_sstable_gpu.py tests/test_wide_gpu.py tests/test_flush_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_b64.log 2>&1 || { tail -30 $O/pytest_b64.log; exit 1; }
tail -1 $O/pytest_b64.log
for rep in 1 2; do
  for v in new old; do
    lib=lsmt_amd/libcassbloom.so; [ $v = old ] && lib=build/xb64/libcassbloom.so
    EXPBENCH_LIB=$lib timeout -k 10 300 python tools/expbench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-flush > $O/b64r_$v.json 2> $O/b64r_$v.err || { tail -20 $O/b64r_$v.err; exit 1; }
    EXPBENCH_LIB=$lib timeout -k 10 300 python tools/expbench.py --leg wide --no-cpu --steps 20 --warmup 2 > $O/b64w_$v.json 2> $O/b64w_$v.err || { tail -20 $O/b64w_$v.err; exit 1; }
    python -c "
import json
r=json.loads(open('$O/b64r_$v.json').read().strip().splitlines()[-1])['read_path']
w=json.loads(open('$O/b64w_$v.json').read().strip().splitlines()[-1])['wide_fanout']
print('$v read', round(r['value']/1e9,3), r.get('kernels_us',{}).get('k_b64_decode'), 'wide', round(w['value']/1e9,3), w['kernels_us'].get('k_b64_decode'))"
  done
done
