#!/bin/bash
# Whole parity suite, smoke, then bench.py through the distributed code path
# at world size 1 (--force-dist: RCCL communicators, exchange, barriers), --check.
set -o pipefail
mkdir -p gpurun_out/fc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fc/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fc/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fc/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fc/smoke.log 2>&1 || { tail -20 gpurun_out/fc/smoke.log; exit 1; }
tail -1 gpurun_out/fc/smoke.log
timeout -k 10 600 python -u bench.py --force-dist --check --no-cpu --no-e2e --no-cold --steps 50 > gpurun_out/fc/dist1.json 2> gpurun_out/fc/dist1.err || { tail -20 gpurun_out/fc/dist1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fc/dist1.json'));print('dist1', d['value'], d.get('valid'), d.get('check'), d['exchange'] and {k: d['exchange'][k] for k in ('mode','all_fit') if k in d['exchange']}, d['read_path']['form'], d['read_path']['value'], d['read_path']['fused_equals_two_step'])"
