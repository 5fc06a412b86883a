#!/bin/bash
# BASELINE C4 and C5 on one GPU with --check (every output against the oracle).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c4 --steps 20 --check > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4.json'));print('C4',d['value']/1e9,'G keys/s',d['ms_per_step'],d.get('check'))"
timeout -k 10 500 python bench.py --workload c5 --steps 20 --check > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5.json'));print('C5',d['value']/1e12,'T probes/s',d['ms_per_step'],d.get('check'))"
