#!/bin/bash
# Round 4: C2 single-build knob sweep (experiment library).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/c2_sweep.py > gpurun_out/c2_sweep.jsonl 2> gpurun_out/c2_sweep.err || { tail -5 gpurun_out/c2_sweep.err; exit 1; }
cat gpurun_out/c2_sweep.jsonl
