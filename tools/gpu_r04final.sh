#!/bin/bash
# Round 4, final pass after the wide-walk screening: the -m gpu suite, smoke(), and
# the default bench line (wall time recorded).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04t.json 2> gpurun_out/bench_r04t.err || { tail -20 gpurun_out/bench_r04t.err; exit 1; }
echo "bench wall s: $(( $(date +%s) - s ))"
python tools/bench_brief.py gpurun_out/bench_r04t.json || true
