#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-e2e --no-read --no-zone --no-flush --no-cold --steps 100"
for ps in 1 2 3 2; do
  timeout -k 10 200 $B --probe-streams $ps > gpurun_out/ps.json 2> gpurun_out/ps.err || { tail -20 gpurun_out/ps.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ps.json'));r=d['roofline'];print('streams=$ps',d['path'],round(d['value']/1e9,1),'G/s step',d['ms_per_step'],'kern',r['kernel_avg_us'],r['kernel_avg_us_per_launch_events'])"
done
for sp in 0 1; do
  CB_SPARSE_EXCHANGE=$sp timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist --check > gpurun_out/d_sp$sp.json 2> gpurun_out/d_sp$sp.err || { tail -20 gpurun_out/d_sp$sp.err; exit 1; }
  grep check gpurun_out/d_sp$sp.err
  python -c "import json;d=json.load(open('gpurun_out/d_sp$sp.json'));print('dist sparse=$sp',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['config']['parallelism'],d['config']['pipeline_lanes'],d['exchange'])"
done
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('full',round(d['value']/1e9,1),d['ms_per_step'],r['kernel_avg_us'],r['frac'],r['random_read_roofline']['frac'],'cold',d['cold']['value']/1e9,'rot',d['rotating_batches']['value']/1e9)"
