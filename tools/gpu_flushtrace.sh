#!/bin/bash
# Flush host timeline (CB_FLUSH_TRACE), the SSTable/flush GPU tests, then the flush leg.
set -o pipefail
mkdir -p gpurun_out
CB_FLUSH_TRACE=1 timeout -k 10 120 python tools/flush_trace.py > gpurun_out/ftrace.log 2>&1 || { tail -20 gpurun_out/ftrace.log; exit 1; }
grep -A5 "^sorted" gpurun_out/ftrace.log | tail -4
tail -4 gpurun_out/ftrace.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  -k "sstable or flush or create or may_contain or meta or rebuild" > gpurun_out/pt_fl.log 2>&1 || { tail -40 gpurun_out/pt_fl.log; exit 1; }
tail -1 gpurun_out/pt_fl.log
TS="" bash tools/gpu_sort4.sh
