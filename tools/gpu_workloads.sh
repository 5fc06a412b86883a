#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --workload c4 --check > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
grep check gpurun_out/c4.err; cat gpurun_out/c4.json
timeout -k 10 300 python bench.py --workload c5 --no-e2e --steps 10 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5.json'));print(d['config']['workload'],d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['kernels_us'],d['alt_paths'])"
timeout -k 10 300 python bench.py > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
cat gpurun_out/c3.json
