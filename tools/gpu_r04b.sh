#!/bin/bash
# Round 4, second pass: the collective-order event without the system-scope
# fence, measured as round 3 measured it (bench.py --force-dist at world 1,
# three lanes, dense and sparse exchange), and the -m gpu C ABI harness.
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --force-dist --steps 200 --warmup 10 --no-cpu --no-e2e --no-cold --no-zone --no-read --no-flush --no-c4 --no-c5 --no-wide"
timeout -k 10 300 $B > gpurun_out/fence_dense.json 2> gpurun_out/fence_dense.err || { tail -5 gpurun_out/fence_dense.err; exit 1; }
CB_SPARSE_EXCHANGE=1 timeout -k 10 300 $B > gpurun_out/fence_sparse.json 2> gpurun_out/fence_sparse.err || { tail -5 gpurun_out/fence_sparse.err; exit 1; }
python -c "
import json
for k in ('dense','sparse'):
    d=json.load(open(f'gpurun_out/fence_{k}.json')); print(k, d['ms_per_step']*1e3, 'us/step', d['exchange'])
"
