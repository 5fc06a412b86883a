#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-e2e --no-read --no-zone --no-flush --no-cold"
for cfg in "2 20" "2 100" "2 20" "2 200" "1 20" "1 100"; do
  set -- $cfg
  timeout -k 10 200 $B --probe-streams $1 --steps $2 > gpurun_out/ps.json 2> gpurun_out/ps.err || { tail -20 gpurun_out/ps.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ps.json'));r=d['roofline'];print('streams=$1 steps=$2',round(d['value']/1e9,1),'G/s step',d['ms_per_step'],'kern',r['kernel_avg_us'],r['kernel_avg_us_per_launch_events'])"
done
