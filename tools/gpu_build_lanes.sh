#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-e2e --no-read --no-zone --no-flush --no-cold"
for ps in 1 2; do
  timeout -k 10 200 $B --probe-streams $ps --check > gpurun_out/bl.json 2> gpurun_out/bl.err || { tail -20 gpurun_out/bl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bl.json'));b=d['build'];print('lanes=$ps C2',round(b['value']/1e9,1),'G keys/s',b['ms_per_step'],b['kernels'])"
  timeout -k 10 300 python bench.py --workload c4 --no-cpu --check --probe-streams $ps > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
  grep check gpurun_out/c4.err
  python -c "import json;d=json.load(open('gpurun_out/c4.json'));print('lanes=$ps C4',round(d['value']/1e9,1),'G keys/s',d['ms_per_step'])"
done
