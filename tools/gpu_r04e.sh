#!/bin/bash
# Round 4: collective-order event with and without the system-scope fence, on
# one box (experiment build, CB_ORDER_FENCE=1 = the round-3 fenced event),
# alternating so drift shows: bench.py --force-dist at world 1, three lanes,
# dense and sparse exchange. Then the one-lane read-path and C2 profile.
set -o pipefail
mkdir -p gpurun_out/fence
B="python tools/expbench.py --force-dist --steps 400 --warmup 20 --no-cpu --no-e2e --no-cold --no-zone --no-read --no-flush --no-c4 --no-c5 --no-wide"
for rep in 1 2; do
  for f in 0 1; do
    for x in 0 1; do
      CB_ORDER_FENCE=$f CB_SPARSE_EXCHANGE=$x timeout -k 10 300 $B > gpurun_out/fence/f${f}_x${x}_$rep.json 2> gpurun_out/fence/f${f}_x${x}_$rep.err || { tail -5 gpurun_out/fence/f${f}_x${x}_$rep.err; exit 1; }
    done
  done
done
python - <<'EOF'
import json, glob
rows = {}
for p in sorted(glob.glob('gpurun_out/fence/*.json')):
    d = json.load(open(p))
    k = p.split('/')[-1][:-7]
    rows.setdefault(k, []).append(round(d['ms_per_step'] * 1e3, 2))
out = {"what": "bench.py --force-dist world 1, three lanes, 400 steps; f1 = order event with the system fence (round 3), f0 = without (round 4); x1 = sparse exchange", "us_per_step": rows}
print(json.dumps(out))
json.dump(out, open('gpurun_out/fence_ab_r04.json', 'w'))
EOF

