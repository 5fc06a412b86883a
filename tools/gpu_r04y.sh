#!/bin/bash
# Round 4: a key bucket's slot 0 holding its value (<= 16 decoded bytes), handed
# to k_b64_decode through a coalesced 16-B slot instead of a gather of the
# file's base64 — read-path parity, then read and wide legs against the last
# commit's library (build/old), alternating. Measured and not kept
# (profiles/inline_values_ab_r04.json); the code was reverted.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_wide_gpu.py tests/test_configs_gpu.py tests/test_flush_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_inl.log 2>&1 || { tail -30 gpurun_out/pytest_inl.log; exit 1; }
tail -1 gpurun_out/pytest_inl.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-e2e --no-cold --no-flush --no-c4 --no-c5"
for rep in 1 2 3; do
  for v in old new; do
    L=build/exp/libcassbloom.so
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/inl_${v}_$rep.json 2> gpurun_out/inl_${v}_$rep.err || { tail -5 gpurun_out/inl_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/inl_${v}_$rep.json').read().strip().splitlines()[-1]);r=d['read_path'];w=d['wide_fanout']
print('$v', 'read', round(r['value']/1e9,3), 'G', r['kernels_us'], r['fused_equals_two_step'], r.get('oracle_sample_bit_exact'), '| two_step', round(r['forms']['two_step']['value']/1e9,2), '| wide', round(w['value']/1e6,1), 'M', w.get('oracle_sample_bit_exact'), w.get('kernels_us'))"
  done
done
