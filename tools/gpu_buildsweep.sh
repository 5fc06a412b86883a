#!/bin/bash
# C2 build step under build-plan overrides (CB_BUILD_KPT / CB_BUILD_TB), three lanes.
# CFGS: space-separated kpt:tb pairs.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-4:19 2:19 1:19 4:18 2:18}; do
  set -- ${cfg/:/ }
  CB_BUILD_KPT=$1 CB_BUILD_TB=$2 timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-read --no-flush --no-zone --check \
    > gpurun_out/bs_$1_$2.json 2> gpurun_out/bs_$1_$2.err || { tail -20 gpurun_out/bs_$1_$2.err; exit 1; }
  python3 -c "
import json;j=json.load(open('gpurun_out/bs_$1_$2.json'));b=j['build'];print('kpt $1 tb $2', b['ms_per_step'], b['kernels'])"
done
