#!/bin/bash
# bench.py's N-rank rehearsal on one GPU, then a default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_bench_multirank_gpu.py \
  > gpurun_out/pytest_rehearse.log 2>&1 || { tail -60 gpurun_out/pytest_rehearse.log; exit 1; }
tail -3 gpurun_out/pytest_rehearse.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(d['value'],r['frac'],r.get('frac_one_lane'),r.get('kernel_avg_us_one_lane'),r['random_read_roofline'])"
