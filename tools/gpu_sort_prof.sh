#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o sprof --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-cold --no-zone --steps 8 > gpurun_out/sprof.json 2> gpurun_out/sprof.err || { tail -20 gpurun_out/sprof.err; exit 1; }
f=$(find gpurun_out/sprof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | cut -c1-160 | head -40
