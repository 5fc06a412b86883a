#!/bin/bash
# Whole -m gpu suite, then one bench line without the CPU, e2e and cold legs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold $* > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err || { tail -20 gpurun_out/bench_check.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_check.json
