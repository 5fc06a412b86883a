#!/bin/bash
# Round 5: C2 one-lane device time behind a spin gate vs behind real builds.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/c2_gate.py > gpurun_out/r05/c2gate.txt 2> gpurun_out/r05/c2gate.err || { tail -5 gpurun_out/r05/c2gate.err; exit 1; }
cat gpurun_out/r05/c2gate.txt
