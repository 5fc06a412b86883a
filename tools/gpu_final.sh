#!/bin/bash
# Round-end check on one GPU: the whole -m gpu suite, smoke(), then the
# round evidence (default bench line + rocprofv3 trace and PMC passes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu_round_evidence.sh
