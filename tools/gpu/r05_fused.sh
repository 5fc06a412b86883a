#!/bin/bash
# Round 5: the one-launch single build (k_build_fused): its GPU tests and the
# build parity tests first, then one-lane C2 latency two-launch vs one-launch
# (tools/c2_lane.hip, C2_FUSED=-1 / 0), alternating, three passes; then the
# random-read fill flavours (tools/gpu/r05_fill.sh).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 500 python -u -m pytest tests/test_build_fused_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
for pass in 1 2 3; do
  for fz in -1 0; do
    C2_FUSED=$fz timeout -k 10 60 ./build/tools/c2_lane lsmt_amd/libcassbloom.so >> $O/c2_fused.jsonl 2>> $O/c2_fused.err || { tail -5 $O/c2_fused.err; exit 1; }
  done
done
cat $O/c2_fused.jsonl
bash tools/gpu/r05_fill.sh
