#!/bin/bash
# Exercise bench.py's exchange path on one GPU: a world-size-1 RCCL group,
# overlapped and sequential, standalone and under torch.distributed.run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --force-dist --check > gpurun_out/d1.json 2> gpurun_out/d1.err || { tail -20 gpurun_out/d1.err; exit 1; }
grep check gpurun_out/d1.err
python -c "import json;d=json.load(open('gpurun_out/d1.json'));print('overlap',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['config']['parallelism'])"
timeout -k 10 300 python bench.py --no-cpu --no-e2e --force-dist --overlap > gpurun_out/d2.json 2> gpurun_out/d2.err || { tail -20 gpurun_out/d2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/d2.json'));print("overlap2",d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['config']['parallelism'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu --no-e2e --force-dist > gpurun_out/d3.json 2> gpurun_out/d3.err || { tail -20 gpurun_out/d3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/d3.json'));print('torchrun',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['n_gpus'])"
