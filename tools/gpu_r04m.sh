#!/bin/bash
# Round 4: 16-bit sub-tile entries for single builds (C2) — golden check and
# the C2 A/B on the experiment library.
set -o pipefail
mkdir -p gpurun_out
CB_BUILD_SUB=1 timeout -k 10 120 python tools/exp_c2_check.py || exit 1
CB_BUILD_SUB=1 CB_BUILD_TB=19 timeout -k 10 120 python tools/exp_c2_check.py || exit 1
timeout -k 10 800 python tools/c2_sweep.py '[{}, {"CB_BUILD_SUB":"1"}, {"CB_BUILD_SUB":"1","CB_BUILD_TB":"19"}, {}, {"CB_BUILD_SUB":"1"}, {"CB_BUILD_SUB":"1","CB_BUILD_TB":"19"}]' > gpurun_out/c2_sub.jsonl 2> gpurun_out/c2_sub.err || { tail -5 gpurun_out/c2_sub.err; exit 1; }
cat gpurun_out/c2_sub.jsonl
