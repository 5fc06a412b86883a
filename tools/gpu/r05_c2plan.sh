#!/bin/bash
# Round 5: one-lane C2 latency (tools/c2_lane.hip) over tile plans of the
# experiment build build/xc2: the default (32-bit entries, 256 tiles of 2^19
# bits), 16-bit entries in 2^18-bit tiles of 512 threads (CB_BUILD_SUB=1),
# 2^18-bit tiles with 32-bit entries (CB_BUILD_TB=18), 16-bit entries in
# 2^19-bit tiles (CB_BUILD_SUB=1 CB_BUILD_TB=19), two passes.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for pass in 1 2; do
  for v in "" "CB_BUILD_SUB=1" "CB_BUILD_TB=18" "CB_BUILD_SUB=1 CB_BUILD_TB=19"; do
    echo -n "[$v] " >> $O/c2plan.txt
    env $v timeout -k 10 60 ./build/tools/c2_lane build/xc2/libcassbloom.so >> $O/c2plan.txt 2>> $O/c2plan.err || { tail -5 $O/c2plan.err; exit 1; }
  done
done
cat $O/c2plan.txt
