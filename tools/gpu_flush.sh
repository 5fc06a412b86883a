#!/bin/bash
# SsTable::create on the device: parity tests, then the flush leg of bench.py.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone > gpurun_out/flush.json 2> gpurun_out/flush.err || { tail -20 gpurun_out/flush.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/flush.json'))['flush'];[print(k, v) for k, v in d.items()]"
