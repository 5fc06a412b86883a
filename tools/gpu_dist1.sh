#!/bin/bash
# Exercise bench.py's exchange paths on one GPU: a world-size-1 RCCL group with
# the dense and the sparse (set-bit positions) all-gather, each checked against
# the oracle, standalone and under torch.distributed.run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for sp in 0 1; do
  CB_SPARSE_EXCHANGE=$sp timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist --check > gpurun_out/d_sp$sp.json 2> gpurun_out/d_sp$sp.err || { tail -20 gpurun_out/d_sp$sp.err; exit 1; }
  grep check gpurun_out/d_sp$sp.err
  python -c "import json;d=json.load(open('gpurun_out/d_sp$sp.json'));print('sparse=$sp',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['config']['parallelism'],d['exchange'])"
done
CB_SPARSE_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist > gpurun_out/d3.json 2> gpurun_out/d3.err || { tail -20 gpurun_out/d3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/d3.json'));print('torchrun sparse',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['n_gpus'],d['exchange'])"
