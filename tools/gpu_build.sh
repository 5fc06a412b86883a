#!/bin/bash
# Build path on one GPU: parity tests for every build, then C2 and C4 throughput.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "build or insert_many or golden or smoke" > gpurun_out/pytest_build.log 2>&1 || { tail -30 gpurun_out/pytest_build.log; exit 1; }
tail -1 gpurun_out/pytest_build.log
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --steps 50 > gpurun_out/b_c2.json 2>gpurun_out/b_c2.err || { tail gpurun_out/b_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c2.json'))['build'];print('C2',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'],d['kernels'])"
timeout -k 10 200 python bench.py --workload c4 --steps 20 > gpurun_out/b_c4.json 2>gpurun_out/b_c4.err || { tail gpurun_out/b_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c4.json'));print('C4',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'])"
