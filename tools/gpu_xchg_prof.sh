#!/bin/bash
# Kernel durations of the exchange pieces (rocprofv3 kernel trace) on one GPU.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof -o xprof -- python3 tools/xchg_parts.py > gpurun_out/xprof.log 2>&1 || { tail -20 gpurun_out/xprof.log; exit 1; }
find gpurun_out/xprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -30
CB_SPARSE_EXCHANGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o dprof -- python3 bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist --steps 50 > gpurun_out/dprof.json 2> gpurun_out/dprof.err || { tail -20 gpurun_out/dprof.err; exit 1; }
find gpurun_out/dprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -30
