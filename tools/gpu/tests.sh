#!/bin/bash
# GPU parity suite (+ optional bench) on one box. Outputs under gpurun_out/.
# Usage: bash tools/gpu/tests.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
exit $rc
