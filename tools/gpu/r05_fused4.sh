#!/bin/bash
# Round 5: the one-launch build as shipped (one workgroup per CU): its tests,
# the build parity tests, then C2 one lane two-launch vs one-launch.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 500 python -u -m pytest tests/test_build_fused_gpu.py tests/test_gpu_parity.py tests/test_build_streams_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_fused4.log 2>&1 || { tail -30 $O/pytest_fused4.log; exit 1; }
tail -1 $O/pytest_fused4.log
for pass in 1 2 3; do
  for fz in -1 0; do
    C2_FUSED=$fz timeout -k 10 60 ./build/tools/c2_lane lsmt_amd/libcassbloom.so >> $O/c2_fused4.jsonl 2>> $O/c2_fused4.err || { tail -5 $O/c2_fused4.err; exit 1; }
  done
done
cat $O/c2_fused4.jsonl
