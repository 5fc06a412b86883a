#!/bin/bash
# C4 build store-policy A/B (CB_BUILD_STORES 0..3), twice each.
set -o pipefail
mkdir -p gpurun_out
for V in 3 0 1 2 3 0 1 2; do
CB_BUILD_STORES=$V timeout -k 10 300 python bench.py --workload c4 --steps 20 --no-cpu > gpurun_out/c4_$V.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4_$V.json'));print('C4 stores=$V',round(d['value']/1e9,2),'G keys/s',d['ms_per_step'])"
done
