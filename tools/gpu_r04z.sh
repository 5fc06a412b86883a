#!/bin/bash
# Round 4, evidence after the 64-filter build batch: the -m gpu suite, smoke(),
# the default bench line, then C4's rocprofv3 kernel stats (one lane) and PMC
# passes (profile_round.sh with --workload c4).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04s.json 2> gpurun_out/bench_r04s.err || { tail -20 gpurun_out/bench_r04s.err; exit 1; }
echo "bench wall s: $(( $(date +%s) - s ))"
python tools/bench_brief.py gpurun_out/bench_r04s.json || true
PROF_OUT=gpurun_out/prof_c4 timeout -k 10 600 bash tools/profile_round.sh --workload c4 > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_c4 --json gpurun_out/pmc_c4_r04c.json > /dev/null && cat gpurun_out/pmc_c4_r04c.json | head -40
