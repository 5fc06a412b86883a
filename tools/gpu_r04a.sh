#!/bin/bash
# Round 4, first evidence pass: the -m gpu suite, the default bench line (C3
# headline + C2/C4/C5/wide/read/flush legs), then rocprofv3 kernel stats and
# PMC passes for the C4 workload (64 concurrent builds).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err || { tail -20 gpurun_out/bench_r04a.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04a.json || true
PROF_OUT=gpurun_out/prof_c4 bash tools/profile_round.sh --workload c4 > gpurun_out/profile_c4.log 2>&1 || { tail -20 gpurun_out/profile_c4.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_c4 --json gpurun_out/pmc_c4.json > /dev/null
tail -12 gpurun_out/profile_c4.log
timeout -k 10 400 python tools/c4_sweep.py 60 > gpurun_out/c4_sweep.jsonl 2> gpurun_out/c4_sweep.err || { tail -5 gpurun_out/c4_sweep.err; exit 1; }
cat gpurun_out/c4_sweep.jsonl | cut -c1-220
timeout -k 10 300 python tools/xcd_order.py 200 > gpurun_out/xcd_order.json 2> gpurun_out/xcd_order.err || { tail -5 gpurun_out/xcd_order.err; exit 1; }
cat gpurun_out/xcd_order.json
