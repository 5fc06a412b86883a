#!/bin/bash
# C2 build (1M keys -> 2^27 bits) and C4 over the plan knobs: tile bits and
# keys per partition thread. One bench line per setting (build legs only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "build or insert_many or golden" > gpurun_out/pytest_build.log 2>&1 || { tail -30 gpurun_out/pytest_build.log; exit 1; }
tail -1 gpurun_out/pytest_build.log
for tb in 19 20; do
  for kpt in 4 8; do
    CB_BUILD_TB=$tb CB_BUILD_KPT=$kpt timeout -k 10 120 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 50 > gpurun_out/bs_${tb}_${kpt}.json 2> gpurun_out/bs.err || { tail gpurun_out/bs.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bs_${tb}_${kpt}.json'))['build'];print('C2 tb=$tb kpt=$kpt',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'],d['kernels'])"
    CB_BUILD_TB=$tb CB_BUILD_KPT=$kpt timeout -k 10 120 python bench.py --workload c4 --no-cpu --steps 20 > gpurun_out/bc4_${tb}_${kpt}.json 2> gpurun_out/bs.err || { tail gpurun_out/bs.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bc4_${tb}_${kpt}.json'));print('C4 tb=$tb kpt=$kpt',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'])"
  done
done
