#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 50 > gpurun_out/b_rep$i.json 2>gpurun_out/b_rep.err || { tail gpurun_out/b_rep.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_rep$i.json'));b=d['build'];print('run $i C2',round(b['value']/1e9,2),'Gkeys/s',b['ms_per_step'],'probe',round(d['value']/1e12,3))"
done
