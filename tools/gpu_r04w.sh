#!/bin/bash
# Round 4: C4 as one launch pair of 64 filters (kMaxBuildBatch 64) against two
# pairs of 32 (the last commit's library, and CB_BUILD_BATCH=32 on the new one),
# every filter's golden check, alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_build_streams_gpu.py tests/test_configs_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_b64.log 2>&1 || { tail -30 gpurun_out/pytest_b64.log; exit 1; }
tail -1 gpurun_out/pytest_b64.log
for rep in 1 2 3; do
  for v in old new new32; do
    L=build/exp/libcassbloom.so; E=""
    if [ $v = old ]; then L=build/old/libcassbloom.so; fi
    if [ $v = new32 ]; then E="CB_BUILD_BATCH=32"; fi
    env $E EXPBENCH_LIB=$L timeout -k 10 300 python tools/expbench.py --workload c4 --steps 200 --warmup 10 --no-cpu --check > gpurun_out/b64_${v}_$rep.json 2> gpurun_out/b64_${v}_$rep.err || { tail -5 gpurun_out/b64_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/b64_${v}_$rep.json').read().strip().splitlines()[-1]);c=d.get('c4',d)
print('$v', c.get('region_us_per_step'), c.get('lanes_region_us_per_step'), c.get('one_lane_us_per_step'), c.get('golden_all_filters_bit_exact'), c.get('kernels_us'))"
  done
done
