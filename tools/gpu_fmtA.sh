#!/bin/bash
# k_format non-temporal stores A/B: flush / read-path parity tests, then the
# bench (every leg but the CPU, e2e and cold ones) with CB_FORMAT_NT=1 and 0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "create or sstable or flush or table or get_many or build or rebuild" > gpurun_out/pytest_fmt.log 2>&1 || { tail -30 gpurun_out/pytest_fmt.log; exit 1; }
tail -1 gpurun_out/pytest_fmt.log
for V in 1 0 1 0; do
CB_FORMAT_NT=$V timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold > gpurun_out/bench_fmt$V.json 2> gpurun_out/bench_fmt.err || { tail -20 gpurun_out/bench_fmt.err; exit 1; }
echo "CB_FORMAT_NT=$V"; python tools/bench_brief.py gpurun_out/bench_fmt$V.json
done
