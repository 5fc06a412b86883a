#!/bin/bash
# Fused read path: its parity tests, then the read leg (two-step and fused) on 1 and 3 lanes.
set -o pipefail
mkdir -p gpurun_out/fz
timeout -k 10 300 python -u -m pytest tests/test_sstable_gpu.py tests/test_flush_gpu.py tests/test_zone_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fz/pytest.log 2>&1 || { tail -40 gpurun_out/fz/pytest.log; exit 1; }
tail -1 gpurun_out/fz/pytest.log
for l in 1 3; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-flush --steps 100 --probe-streams $l > gpurun_out/fz/b$l.json 2> gpurun_out/fz/b$l.err || { tail -20 gpurun_out/fz/b$l.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fz/b$l.json'))['read_path'];print('lanes $l', d['form'], d['fused_equals_two_step'], {k:(round(v['value']/1e9,3), v['kernels_us']) for k,v in d['forms'].items()})"
done
