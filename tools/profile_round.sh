#!/bin/bash
# rocprofv3 evidence for one bench shape (run on the GPU box from the repo
# root): a kernel-trace/stats pass as the bench runs (lanes overlap), one with
# a single lane (each dispatch alone: its duration is the kernel's own time,
# the figure bench.py's profile check compares with its one-lane events),
# then one PMC pass per counter group, one lane, no trace domain with --pmc.
# Usage: bash tools/profile_round.sh SHAPE [extra bench.py args]
#   SHAPE: c2 (one 1M-key build per launch pair: four lanes, then one), c3
#   (the headline), c4 (64 batched builds), c5 (the C5 rank slice), wide (300
#   m=1024 tables in one wide set)
# Output: $PROF_OUT (default gpurun_out/prof_SHAPE)/summary.json
# (c3 warms up for 1000 steps per leg: its stats average every k_set_probe
# launch of the run, and on a box that has just started the first launches run
# at a low clock; round 5 measured 46.6 against 38.7 us with 5 warm-up steps
# as the call's first shape)
set -o pipefail
export TMPDIR=/tmp
SHAPE=$1
shift
OUT=${PROF_OUT:-gpurun_out/prof_$SHAPE}
mkdir -p $OUT
LANE1="--probe-streams 1"
case $SHAPE in
  c2) BENCH="python bench.py --leg c2 --no-cpu --no-cold --steps 50 --warmup 5"; META="shape=c2"; LANE1="--build-streams 1" ;;
  c3) BENCH="python bench.py --no-cpu --no-e2e --no-cold --no-c4 --no-c5 --no-wide --steps 50 --warmup 1000"; META="shape=c3" ;;
  c4) BENCH="python bench.py --workload c4 --no-cpu --steps 50 --warmup 5"; META="shape=c4 filters_per_launch=64" ;;
  c5) BENCH="python bench.py --leg c5 --no-cpu --steps 20 --warmup 3"; META="shape=c5" ;;
  wide) BENCH="python bench.py --leg wide --no-cpu --steps 10 --warmup 2"; META="shape=wide" ;;
  *) echo "unknown shape $SHAPE"; exit 2 ;;
esac
BENCH="$BENCH $*"
# the same one-lane command without the profiler first: the bench's own
# (HIP-event) step on this box, beside the traced one (tracing can lengthen
# short back-to-back launches)
timeout -k 10 300 $BENCH $LANE1 > $OUT/plain1_bench.json 2> $OUT/plain1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $BENCH > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
BENCH="$BENCH $LANE1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt1 -o kt1 --output-format csv -- $BENCH > $OUT/kt1_bench.json 2> $OUT/kt1.err || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o pmc$i --output-format csv -- $BENCH > /dev/null 2> $OUT/pmc$i.err || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.err; exit 1; }
done
python tools/pmc_summary.py $OUT --json $OUT/summary.json $META > $OUT/summary.txt && cat $OUT/summary.txt
