#!/bin/bash
# Exchange on one GPU: the exchange tests first (new kernels), then the whole
# parity suite, the piece timings, and bench.py's exchange (world size 1,
# dense and sparse, through the C-ABI communicator) checked against the oracle.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_exchange_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xchg.log 2>&1 || { tail -40 gpurun_out/pytest_xchg.log; exit 1; }
tail -1 gpurun_out/pytest_xchg.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for sp in 0 1; do
  CB_SPARSE_EXCHANGE=$sp timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist --check > gpurun_out/d_sp$sp.json 2> gpurun_out/d_sp$sp.err || { tail -20 gpurun_out/d_sp$sp.err; exit 1; }
  grep check gpurun_out/d_sp$sp.err
  python -c "import json;d=json.load(open('gpurun_out/d_sp$sp.json'));print('sparse=$sp',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['config']['parallelism'],d['exchange'])"
done
