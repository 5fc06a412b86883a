#!/bin/bash
# Round-end rehearsal on one GPU: parity suite, smoke(), default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_full.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['read_path']['value'],d['read_path']['kernels_us'],d['flush']['unsorted_input']['ms_per_flush'])"
