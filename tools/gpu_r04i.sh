#!/bin/bash
# Round 4: key buckets on the read path — parity, the suite, an A/B of the
# read and wide legs with and without them (experiment library), the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_wide_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_read.log 2>&1 || { tail -40 gpurun_out/pytest_read.log; exit 1; }
tail -2 gpurun_out/pytest_read.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
B="python tools/expbench.py --steps 20 --warmup 5 --leg-steps 200 --no-cpu --no-e2e --no-cold --no-flush --no-c4 --no-c5"
for rep in 1 2; do
  for nb in 1 0; do
    CB_NO_BUCKETS=$nb timeout -k 10 300 $B > gpurun_out/bkt_${nb}_$rep.json 2> gpurun_out/bkt_${nb}_$rep.err || { tail -5 gpurun_out/bkt_${nb}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/bkt_${nb}_$rep.json'));r=d['read_path'];w=d['wide_fanout']
print('no_buckets=$nb', 'read', round(r['value']/1e9,3), 'G', r['ms_per_step'], r['kernels_us'], 'fused==two', r['fused_equals_two_step'], 'oracle', r['oracle_sample_bit_exact'], '| wide', round(w['value']/1e6,1), 'M', w.get('kernels_us'))"
  done
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04i.json 2> gpurun_out/bench_r04i.err || { tail -20 gpurun_out/bench_r04i.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04i.json || true
