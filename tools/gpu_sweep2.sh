#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --no-e2e > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$label',d['path'],round(d['value']/1e9,1),d['kernels_us'],'tiled',d['alt_kernels_us'],'build',d['build']['ms_per_step'],d['build']['kernels'])"
}
run kpl1 CB_SET_KPL=1
run kpl2 CB_SET_KPL=2
run kpl4 CB_SET_KPL=4
run kpl1_nosc CB_SET_KPL=1 CB_SET_SC=0
run bkpt8 CB_BUILD_KPT=8
run bkpt16 CB_BUILD_KPT=16
run bkpt16_tb17 CB_BUILD_KPT=16 CB_BUILD_TB=17
run bkpt8_tb17 CB_BUILD_KPT=8 CB_BUILD_TB=17
