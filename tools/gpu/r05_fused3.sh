#!/bin/bash
# Round 5: one-lane C2 latency: two-launch; one-launch at one workgroup per
# CU (build/fz1w8); one-launch at two per CU with half-size partition blocks
# (CB_BUILD_KPT=2: 512 partition blocks fill both slots of every CU).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for pass in 1 2 3; do
  C2_FUSED=-1 timeout -k 10 60 ./build/tools/c2_lane lsmt_amd/libcassbloom.so >> $O/c2_fused3.jsonl 2>> $O/c2_fused3.err || { tail -5 $O/c2_fused3.err; exit 1; }
  C2_FUSED=0 timeout -k 10 60 ./build/tools/c2_lane build/fz1w8/libcassbloom.so >> $O/c2_fused3.jsonl 2>> $O/c2_fused3.err || { tail -5 $O/c2_fused3.err; exit 1; }
  CB_BUILD_KPT=2 C2_FUSED=0 timeout -k 10 60 ./build/tools/c2_lane lsmt_amd/libcassbloom.so >> $O/c2_fused3.jsonl 2>> $O/c2_fused3.err || { tail -5 $O/c2_fused3.err; exit 1; }
done
cat $O/c2_fused3.jsonl
