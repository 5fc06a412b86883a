#!/bin/bash
# Round evidence on one GPU: the default bench line (N=1, CPU baselines
# included), then the rocprofv3 kernel-trace + PMC passes of every shape
# (tools/profile_round.sh: c3 headline, c4 builds, c5 rank slice, wide
# fan-out), each summarised into gpurun_out/prof_<shape>/summary.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_full.json
for shape in c3 c4 c5 wide; do
  PROF_OUT=gpurun_out/prof_$shape bash tools/profile_round.sh $shape > gpurun_out/prof_$shape.log 2>&1 || { tail -20 gpurun_out/prof_$shape.log; exit 1; }
  echo "== $shape"; tail -8 gpurun_out/prof_$shape.log
done
