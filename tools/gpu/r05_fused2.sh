#!/bin/bash
# Round 5: one-lane C2 latency, two-launch vs the one-launch build at two
# and at one workgroup per CU (build/fz1*: CB_BUILD_FUSED_LDS=96 KiB), three
# alternating passes (tools/c2_lane.hip).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for pass in 1 2 3; do
  C2_FUSED=-1 timeout -k 10 60 ./build/tools/c2_lane lsmt_amd/libcassbloom.so >> $O/c2_fused2.jsonl 2>> $O/c2_fused2.err || { tail -5 $O/c2_fused2.err; exit 1; }
  for lib in lsmt_amd build/fz1 build/fz1w8; do
    C2_FUSED=0 timeout -k 10 60 ./build/tools/c2_lane $lib/libcassbloom.so >> $O/c2_fused2.jsonl 2>> $O/c2_fused2.err || { tail -5 $O/c2_fused2.err; exit 1; }
  done
done
cat $O/c2_fused2.jsonl
