#!/bin/bash
# Round 5: k_b64_decode at one and two keys per thread (CB_B64_KPT on the
# experiment build build/xkp): the SSTable tests on the experiment build with
# two, then the read path and the wide fan-out, alternating, two reps.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  for kp in 1 2; do
    CB_B64_KPT=$kp EXPBENCH_LIB=build/xkp/libcassbloom.so timeout -k 10 300 python tools/expbench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --no-flush > $O/kp_r$kp.json 2> $O/kp_r$kp.err || { tail -20 $O/kp_r$kp.err; exit 1; }
    CB_B64_KPT=$kp EXPBENCH_LIB=build/xkp/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --steps 20 --warmup 2 > $O/kp_w$kp.json 2> $O/kp_w$kp.err || { tail -20 $O/kp_w$kp.err; exit 1; }
    python -c "
import json
r=json.loads(open('$O/kp_r$kp.json').read().strip().splitlines()[-1])['read_path']
w=json.loads(open('$O/kp_w$kp.json').read().strip().splitlines()[-1])['wide_fanout']
print('kpt $kp read', round(r['value']/1e9,3), r.get('kernels_us',{}).get('k_b64_decode'), r.get('fused_equals_two_step'), r.get('oracle_sample_bit_exact'), 'wide', round(w['value']/1e9,3), w['kernels_us'].get('k_b64_decode'), w.get('oracle_sample_bit_exact'))"
  done
done
