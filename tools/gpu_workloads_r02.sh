#!/bin/bash
# C4 and C5 (per-rank slice) bench lines on one GPU, each checked against the oracle.
set -o pipefail
mkdir -p gpurun_out/wl
timeout -k 10 600 python -u bench.py --workload c5 --check --no-cpu --no-e2e --no-cold --no-zone --no-flush --steps 20 --warmup 3 > gpurun_out/wl/c5.json 2> gpurun_out/wl/c5.err || { tail -20 gpurun_out/wl/c5.err; exit 1; }
grep "\[check\]" gpurun_out/wl/c5.err | tail -2
python -c "import json;d=json.load(open('gpurun_out/wl/c5.json'));print('c5', d['value'], d['ms_per_step'], d['config']['workload'], d['roofline']['frac'], d['roofline']['random_read_roofline']['frac'])"
timeout -k 10 600 python -u bench.py --workload c4 --check --no-cpu --steps 20 --warmup 3 > gpurun_out/wl/c4.json 2> gpurun_out/wl/c4.err || { tail -20 gpurun_out/wl/c4.err; exit 1; }
grep -i "check" gpurun_out/wl/c4.err | tail -2
python -c "import json;d=json.load(open('gpurun_out/wl/c4.json'));print('c4', d['value'], d['unit'], d['ms_per_step'], d['config'])"
