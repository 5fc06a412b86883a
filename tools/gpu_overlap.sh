#!/bin/bash
# World-size-1 RCCL group on one GPU: dense / sparse exchange, serial vs
# overlapped on the comm stream, each checked against the oracle.
set -o pipefail
mkdir -p gpurun_out
for sp in 0 1; do
  for ov in "" "--overlap"; do
    tag=sp${sp}${ov:+_ov}
    CB_SPARSE_EXCHANGE=$sp timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-zone --no-flush --no-cold --force-dist --check $ov > gpurun_out/x_$tag.json 2> gpurun_out/x_$tag.err || { tail -20 gpurun_out/x_$tag.err; exit 1; }
    grep check gpurun_out/x_$tag.err
    python -c "import json;d=json.load(open('gpurun_out/x_$tag.json'));print('$tag',d['path'],round(d['value']/1e9,1),d['ms_per_step'],d['alt_paths'],d['exchange'])"
  done
done
