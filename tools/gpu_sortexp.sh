#!/bin/bash
# Timing A/B of library variants (build/exp/*.so, experiment builds: their
# results are not checked) against the in-tree library on the bench's flush leg.
set -o pipefail
mkdir -p gpurun_out
cp lsmt_amd/libcassbloom.so gpurun_out/.lib_main.so
run() {
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-zone --no-read --steps 40 > gpurun_out/exp_$1.json 2> gpurun_out/exp_$1.err || { tail -30 gpurun_out/exp_$1.err; return 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/exp_$1.json'));f=d['flush']
print('$1', 'sorted', f['sorted_input']['ms_per_flush'], 'unsorted', f['unsorted_input']['ms_per_flush'], f['unsorted_input']['kernels_us'])"
}
run main || exit 1
for v in ${VARIANTS}; do
  cp build/exp/$v.so lsmt_amd/libcassbloom.so && run $v; rc=$?
  cp gpurun_out/.lib_main.so lsmt_amd/libcassbloom.so
  [ $rc -eq 0 ] || exit 1
done
rm -f gpurun_out/.lib_main.so
