#!/bin/bash
# Round 5: wide walk variants at four waves: the product, DirMaps read from
# global instead of staged per group (CB_WIDE_NO_SDM build), and the screen at
# 16 / 64 fingerprint bins (CB_SCREEN_HBITS=4 / 6; product 32), alternating.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() { python -c "import json;d=json.load(open('$1'))['wide_fanout'];print('$2', round(d['value']/1e6,1), d['kernels_us'], d.get('oracle_sample_bit_exact'))"; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --leg wide --steps 20 --warmup 2 > $O/w5_prod_$rep.json 2> $O/w5_prod_$rep.err || { tail -20 $O/w5_prod_$rep.err; exit 1; }
  show $O/w5_prod_$rep.json product
  EXPBENCH_LIB=build/expr5nosdm/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --steps 20 --warmup 2 > $O/w5_nosdm_$rep.json 2> $O/w5_nosdm_$rep.err || { tail -20 $O/w5_nosdm_$rep.err; exit 1; }
  show $O/w5_nosdm_$rep.json no-staged-dirmaps
  for h in 4 6; do
    CB_SCREEN_HBITS=$h EXPBENCH_LIB=build/expr5/libcassbloom.so timeout -k 10 300 python tools/expbench.py --leg wide --steps 20 --warmup 2 > $O/w5_h${h}_$rep.json 2> $O/w5_h${h}_$rep.err || { tail -20 $O/w5_h${h}_$rep.err; exit 1; }
    show $O/w5_h${h}_$rep.json "screen-hbits$h"
  done
done
