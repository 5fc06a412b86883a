#!/bin/bash
# Round evidence on one GPU: parity suite, smoke, full bench (with the CPU
# baseline), rocprof kernel trace + PMC passes. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
tail -20 gpurun_out/profile_round.log | cut -c1-300
timeout -k 10 180 python tools/xchg_parts.py > gpurun_out/xchg_parts.json 2> gpurun_out/xchg_parts.err || { tail -20 gpurun_out/xchg_parts.err; exit 1; }
cat gpurun_out/xchg_parts.json
