#!/bin/bash
# Full GPU parity suite, then the end-to-end legs (pinned host buffers:
# zero-copy set probe, staged set probe, staged per-filter probe) with the
# cold-cache legs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 200 python bench.py --no-cpu --no-zone --no-flush --steps 20 > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail gpurun_out/e2e.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e2e.json'));print(d['e2e'], d['cold'], d['build']['cold'], d['value']/1e9)"
