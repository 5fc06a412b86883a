#!/bin/bash
# GPU parity suite, then the probe bench under timing-only attribution flags
# (CB_PROBE_XFLAGS: 1 skip b-gathers, 2 skip tile streaming, 4 skip mask stores).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for x in 0 1 2 4 7; do
  CB_PROBE_XFLAGS=$x timeout -k 10 200 python bench.py --no-cpu --no-e2e > gpurun_out/sw_x$x.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw_x$x.json'));print('xflags',$x,round(d['value']/1e9,1),'Gp/s',d['ms_per_step'],d['kernels_us'],'build',d['build']['ms_per_step'],d['build']['kernels'])"
done
