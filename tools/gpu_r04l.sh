#!/bin/bash
# Round 4: the product-shape flush (1024 entries, m = 1024): LDS build for
# small filters, inline tile scan in k_format — parity, then timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/small_flush.py 200 > gpurun_out/small_flush_l.json && cat gpurun_out/small_flush_l.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sfl -o sf --output-format csv -- python tools/small_flush.py 50 > /dev/null 2> gpurun_out/prof_sfl.err || exit 1
python - <<PY
import csv,glob
f=glob.glob("gpurun_out/prof_sfl/**/sf_kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e3,2))
PY
