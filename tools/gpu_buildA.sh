#!/bin/bash
# Build-path A/B on one GPU: the phase-stamped ubench and the bench's C2 leg
# (four and one lanes) for each CB_BUILD_WT setting, then the build parity tests.
set -o pipefail
mkdir -p gpurun_out
K="build or insert or golden or c4 or create or rebuild"
for V in 0 1 2 3 0; do
CB_BUILD_WT=$V timeout -k 10 60 ./build/tools/ubench_build > gpurun_out/ubench_build_$V.json || exit 1
python -c "import json;d=json.load(open('gpurun_out/ubench_build_$V.json'));print('wt=$V', {k:d[k] for k in ('build_step_us','part_alone_us','tile_alone_us')}, d['tile_stamps']['phase_median_us'])"
for P in 4 3 1; do
CB_BUILD_WT=$V timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --steps 50 --build-streams $P > gpurun_out/b_c2_$V$P.json 2>gpurun_out/b_c2.err || { tail gpurun_out/b_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_c2_$V$P.json'))['build'];print('C2 wt=$V lanes=$P',round(d['value']/1e9,2),'Gkeys/s',d['ms_per_step'],d['kernels'])"
done
done
CB_BUILD_WT=3 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_build.log 2>&1 || { tail -30 gpurun_out/pytest_build.log; exit 1; }
tail -1 gpurun_out/pytest_build.log
