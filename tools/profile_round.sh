#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo
# root): one kernel-trace/stats pass, then PMC passes with one counter group
# each (no --pmc together with any trace domain). Output: gpurun_out/prof/.
# Usage: bash tools/profile_round.sh [extra bench.py args]
set -o pipefail
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
# the trace pass runs the bench as configured (three pipeline lanes: launches
# overlap, so per-dispatch durations are ~2x the per-step share; pmc_summary
# reports the union of each kernel's busy intervals per launch beside them);
# the PMC passes run one lane so every dispatch's counters are its own
BENCH="python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --steps 50 --warmup 5 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $BENCH > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
BENCH="$BENCH --probe-streams 1"
# the same with one lane: launches do not overlap, so each dispatch's
# duration is the kernel's own time, comparable with the bench line's
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt1 -o kt1 --output-format csv -- $BENCH > $OUT/kt1_bench.json 2> $OUT/kt1.err || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o pmc$i --output-format csv -- $BENCH > /dev/null 2> $OUT/pmc$i.err || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.err; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
