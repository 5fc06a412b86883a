#!/bin/bash
# Round 4, third pass: the -m gpu suite, the default bench line, the C4
# tile-pass variants, and the collective-order fence measurement.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04c.json 2> gpurun_out/bench_r04c.err || { tail -20 gpurun_out/bench_r04c.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04c.json || true
python -c "import json;d=json.load(open('gpurun_out/bench_r04c.json'));print('C2 one lane', d['build']['one_lane'], 'cold', d['build']['cold'])"
timeout -k 10 400 python tools/c4_sweep.py 60 > gpurun_out/c4_sweep_c.jsonl 2> gpurun_out/c4_sweep_c.err || { tail -5 gpurun_out/c4_sweep_c.err; exit 1; }
cut -c1-200 gpurun_out/c4_sweep_c.jsonl
bash tools/gpu_r04b.sh
bash tools/gpu_r04d.sh
