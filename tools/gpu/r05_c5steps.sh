#!/bin/bash
# Round 5: the C5 leg's step time against the number of timed steps and the
# legs run before it (is the default line's C5 slower than the leg alone?).
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
show() {
python -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1])['c5']
print('$2', d['region_us_per_step'], d['one_lane_us_per_step'], d['steps'])"
}
for st in 20 600; do
  timeout -k 10 200 python bench.py --leg c5 --no-cpu --steps 20 --leg-steps $st --warmup 3 > $O/c5st_$st.json 2> $O/c5st_$st.err || { tail -5 $O/c5st_$st.err; exit 1; }
  show $O/c5st_$st.json "leg alone, leg-steps $st"
done
timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold --no-wide > $O/c5st_full.json 2> $O/c5st_full.err || { tail -5 $O/c5st_full.err; exit 1; }
show $O/c5st_full.json "default line (no cpu/e2e/cold/wide)"
timeout -k 10 200 python bench.py --leg c5 --no-cpu --steps 20 --warmup 3 > $O/c5st_b.json 2> $O/c5st_b.err || { tail -5 $O/c5st_b.err; exit 1; }
show $O/c5st_b.json "leg alone again"
