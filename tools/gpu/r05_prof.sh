#!/bin/bash
# Round 5: rocprofv3 trace + PMC evidence for the given shapes, one after the
# other (tools/profile_round.sh), each into gpurun_out/r05/prof_<shape>.
set -o pipefail
mkdir -p gpurun_out/r05
for shape in "$@"; do
  PROF_OUT=gpurun_out/r05/prof_$shape bash tools/profile_round.sh $shape > gpurun_out/r05/prof_$shape.log 2>&1 || { tail -20 gpurun_out/r05/prof_$shape.log; exit 1; }
  echo "== $shape"; tail -12 gpurun_out/r05/prof_$shape.log
  # the summary holds what the traces and counter dumps gave; drop them so the
  # call's gpurun_out stays under the 64 MiB it may bring back
  find gpurun_out/r05/prof_$shape \( -name '*_kernel_trace.csv' -o -name '*_counter_collection.csv' \) -delete
done
