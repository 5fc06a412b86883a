#!/bin/bash
# Build checks on one GPU: build / host-mirror / C4 parity tests, then C2 on
# four and one lanes and C4 (twice each).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "build or insert or golden or c4 or create or rebuild or may_contain or mirror" > gpurun_out/pytest_build.log 2>&1 || { tail -30 gpurun_out/pytest_build.log; exit 1; }
tail -1 gpurun_out/pytest_build.log
for V in 3 3; do
for P in 4 1; do
CB_BUILD_STORES=$V timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 50 --build-streams $P > gpurun_out/b_c2_$V$P.json 2>gpurun_out/b_c2.err || { tail gpurun_out/b_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c2_$V$P.json'))['build'];print('C2 stores=$V lanes=$P',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'])"
done
CB_BUILD_STORES=$V timeout -k 10 300 python bench.py --workload c4 --steps 20 --no-cpu > gpurun_out/c4_$V.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4_$V.json'));print('C4 stores=$V',round(d['value']/1e9,2),'G keys/s',d['ms_per_step'])"
done
