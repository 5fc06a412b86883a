#!/bin/bash
# A/B of the set probe forms on C3 (and the C5 rank shape): block-per-1024-keys
# vs the persistent k_set_probe_flow at several blocks-per-CU; gated and
# parity tests under the flow form first.
set -o pipefail
mkdir -p gpurun_out
CB_SET_FLOW=1 timeout -k 10 300 python -u -m pytest tests/test_zone_gpu.py tests/test_configs_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_flow.log 2>&1 || { tail -30 gpurun_out/pytest_flow.log; exit 1; }
tail -1 gpurun_out/pytest_flow.log
B="python bench.py --no-cpu --no-e2e --no-read --no-flush --no-cold --steps 40"
for cfg in "0 8" "1 8" "1 4" "0 8" "1 4" "1 8"; do
  set -- $cfg
  CB_SET_FLOW=$1 CB_SET_FLOW_BPC=$2 timeout -k 10 200 $B > gpurun_out/sf.json 2> gpurun_out/sf.err || { tail -20 gpurun_out/sf.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sf.json'));r=d['roofline'];print('flow=$1 bpc=$2',d['path'],round(d['value']/1e9,1),'G/s step',d['ms_per_step'],'kern',r['kernel_avg_us'],'rr',r.get('random_read_roofline',{}).get('frac'),'gated',d['zone_gate']['value']/1e9, d['zone_gate']['kernels_us'])"
done
for f in 0 1; do
  CB_SET_FLOW=$f timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 20 --n-keys 10000000 > gpurun_out/sf5.json 2> gpurun_out/sf5.err || { tail -20 gpurun_out/sf5.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sf5.json'));r=d['roofline'];print('C5shape flow=$f',round(d['value']/1e9,1),'G/s kern',r['kernel_avg_us'],'rr',r.get('random_read_roofline',{}).get('frac'))"
done
