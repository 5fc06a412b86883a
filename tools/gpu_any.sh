#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for any in 1 0; do
  CB_SET_ANY=$any timeout -k 10 200 python bench.py --no-cpu --no-e2e > gpurun_out/any$any.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/any$any.json'));r=d['roofline'];print('any',$any,d['path'],round(d['value']/1e9,1),d['kernels_us'],r['frac'],r.get('random_read_roofline',{}).get('frac'),r['algorithmic_def'][:40])"
done
CB_SET_ANY=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --n-keys 10000000 --steps 10 > gpurun_out/c5any.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/c5any.json'));print('c5',d['path'],round(d['value']/1e9,1),d['kernels_us'])"
