#!/bin/bash
# FilterSet probe: short-circuit on/off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for sc in 1 0; do
  CB_SET_SC=$sc timeout -k 10 200 python bench.py --no-cpu --no-e2e > gpurun_out/set_sc$sc.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/set_sc$sc.json'));print('sc',$sc,round(d['value']/1e9,1),'Gp/s',d['ms_per_step'],d['kernels_us'],d['roofline']['frac'])"
done
