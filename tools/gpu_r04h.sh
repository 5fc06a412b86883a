#!/bin/bash
# Round 4: the C4 and C2 build-knob sweeps again, now on the experiment
# library for real (tools/expbench.py loader fix), alternating the default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/c4_sweep.py 60 '[{}, {"CB_BUILD_TILE_NT":"512","CB_BUILD_TB":"18"}, {"CB_BUILD_TB":"18"}, {"CB_BUILD_BATCH":"8"}, {"CB_BUILD_BATCH":"16"}, {"CB_BUILD_KPT":"2"}, {"CB_BUILD_STORES":"1"}, {"CB_BUILD_STORES":"2"}, {}]' > gpurun_out/c4_sweep_h.jsonl 2> gpurun_out/c4_sweep_h.err || { tail -5 gpurun_out/c4_sweep_h.err; cut -c1-200 gpurun_out/c4_sweep_h.jsonl; exit 1; }
cut -c1-200 gpurun_out/c4_sweep_h.jsonl
timeout -k 10 600 python tools/c2_sweep.py '[{}, {"CB_BUILD_KPT":"2"}, {"CB_BUILD_KPT":"1"}, {"CB_BUILD_TB":"18"}, {"CB_BUILD_TILE_NT":"512","CB_BUILD_TB":"18"}, {"CB_BUILD_STORES":"1"}, {"CB_BUILD_STORES":"2"}, {}]' > gpurun_out/c2_sweep_h.jsonl 2> gpurun_out/c2_sweep_h.err || { tail -5 gpurun_out/c2_sweep_h.err; exit 1; }
cat gpurun_out/c2_sweep_h.jsonl
