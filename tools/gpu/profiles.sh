#!/bin/bash
# rocprofv3 trace + PMC evidence for the given shapes, one after the
# other (tools/profile_round.sh), each into gpurun_out/prof/<shape>
# (copy the summaries to profiles/ under the round's name). Run c3 after
# another shape (`c4 c5 c3 wide`), so the chip's clock has ramped up.
set -o pipefail
mkdir -p gpurun_out/prof
for shape in "$@"; do
  PROF_OUT=gpurun_out/prof/$shape bash tools/profile_round.sh $shape > gpurun_out/prof/$shape.log 2>&1 || { tail -20 gpurun_out/prof/$shape.log; exit 1; }
  echo "== $shape"; tail -12 gpurun_out/prof/$shape.log
  # the summary holds what the traces and counter dumps gave; drop them so the
  # call's gpurun_out stays under the 64 MiB it may bring back
  # (and the call's file count: keep the summary, the kernel stats and the logs)
  find gpurun_out/prof/$shape \( -name '*_kernel_trace.csv' -o -name '*_counter_collection.csv' \
    -o -name '*_agent_info.csv' -o -name '*_domain_stats.csv' \) -delete
done
