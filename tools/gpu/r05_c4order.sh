#!/bin/bash
# Round 5: C4's one-lane step as `--workload c4` (fresh process, C4 alone)
# against the C4 leg of a default-style line (after the C3 and C2 legs), on
# one box, alternating: the r04 verdict's 121 vs 111 us.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 200 --warmup 10 --probe-streams 1 > $O/c4o_alone_$rep.json 2> $O/c4o_alone_$rep.err || { tail -20 $O/c4o_alone_$rep.err; exit 1; }
  python -c "import json;c=json.load(open('$O/c4o_alone_$rep.json'))['c4'];print('alone one-lane',c['one_lane_us_per_step'],c['kernels_us'])"
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cold --no-c5 --no-wide --no-zone --no-read --no-flush > $O/c4o_line_$rep.json 2> $O/c4o_line_$rep.err || { tail -20 $O/c4o_line_$rep.err; exit 1; }
  python -c "import json;c=json.load(open('$O/c4o_line_$rep.json'))['c4'];print('in-line one-lane',c['one_lane_us_per_step'],'region',c['region_us_per_step'],c['kernels_us'])"
done
