#!/bin/bash
# Build checks on one GPU: build / host-mirror / C4 parity tests, the may_contain
# latency tool, then C2 on four lanes (three runs), the GPU-bound rate and C4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "build or insert or golden or c4 or create or rebuild or may_contain or mirror" > gpurun_out/pytest_build.log 2>&1 || { tail -30 gpurun_out/pytest_build.log; exit 1; }
tail -1 gpurun_out/pytest_build.log
for i in 1 2 3; do
timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 50 > gpurun_out/b_c2_$i.json 2>gpurun_out/b_c2.err || { tail gpurun_out/b_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c2_$i.json'));b=d['build'];print('C2 run $i',round(b['value']/1e9,2),'Gkeys/s',b['ms_per_step'],'mirror m1024',d['may_contain']['m1024'].get('mirror_ns_per_call'))"
done
timeout -k 10 300 python tools/build_gpu_bound.py > gpurun_out/build_gpu_bound.json && cat gpurun_out/build_gpu_bound.json
timeout -k 10 300 python bench.py --workload c4 --steps 20 --no-cpu > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4.json'));print('C4',round(d['value']/1e9,2),'G keys/s',d['ms_per_step'])"
