#!/bin/bash
# Dense probe shape of C5 per GPU (10M keys x 32 filters of 2^26 bits).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --no-e2e --n-keys 10000000 --keys-per-filter 524288 --steps 10 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5.json'));print(d['path'],round(d['value']/1e9,1),'Gp/s',d['ms_per_step'],d['kernels_us'],'alt',d['alt_paths'],d['alt_kernels_us'])"
timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 10 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3.json'));print(d['path'],round(d['value']/1e9,1),'Gp/s',d['ms_per_step'],d['kernels_us'],'build',d['build']['ms_per_step'],d['build']['kernels'])"
