#!/bin/bash
# Round 4: partition pass with its key loads issued together (no per-key
# branch), unconditional LDS atomics, 32-bit position packing, seed folded into
# the hash's first plane; persistent variant for C4 — parity first, then A/B
# against the last commit's library (build/old), alternating. (the "new" arm ran the persistent kernel, "noloop" k_build_part; the kept form is "noloop")
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_build_streams_gpu.py tests/test_configs_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_part.log 2>&1 || { tail -30 gpurun_out/pytest_part.log; exit 1; }
tail -1 gpurun_out/pytest_part.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 400 --no-cpu --no-e2e --no-cold --no-flush --no-c5 --no-wide"
for rep in 1 2; do
  for v in old new noloop; do
    L=build/exp/libcassbloom.so; E=""
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    if [ $v = noloop ]; then E="CB_BUILD_LOOP=0"; fi
    env $E EXPBENCH_LIB=$L timeout -k 10 300 $B > gpurun_out/pa_${v}_$rep.json 2> gpurun_out/pa_${v}_$rep.err || { tail -5 gpurun_out/pa_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/pa_${v}_$rep.json').read().strip().splitlines()[-1]);b=d['build'];c=d['c4']
print('$v', 'C3', round(d['value']/1e12,3), '| C2 4-lane', round(b['value']/1e9,1), 'one-lane us', b['one_lane']['us_per_build'], b['kernels'], '| C4 us', c.get('region_us_per_step'), c.get('one_lane_us_per_step'), c.get('kernels_us'), 'golden', c.get('oracle_sample_bit_exact', c.get('golden')))"
  done
done
