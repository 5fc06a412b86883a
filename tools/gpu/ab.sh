#!/bin/bash
# A/B driver for the GPU box. Every rep runs each variant once, in turn, so
# clock and thermal drift fall on all variants alike; the first failure ends
# the call. Usage:
#   LEG=<leg> [REPS=2] [STEPS=20] [WARMUP=3] [TESTS="tests/x.py ..."] [ARGS="..."] \
#     bash tools/gpu/ab.sh VARIANT [VARIANT ...]
# LEG: c5 | wide (bench.py --leg), c3 | c4 (bench.py --workload, the whole
#   default line for c3), or c2_lane (build/tools/c2_lane: one-lane C2
#   device time of the given library, tools/c2_lane.hip).
# VARIANT = label[,lib][,ENV=value ...]. lib is an experiment build of the
#   library, made in this container with
#     make -C lsmt_amd/csrc EXTRA="-DCB_EXPERIMENTS ..." BUILD=../../build/x<name>/obj \
#          OUT=../../build/x<name>/libcassbloom.so
#   and run through tools/expbench.py; without one, the product library runs
#   through bench.py. ENV settings apply to that variant only (the CB_* knobs
#   of an experiment build).
# TESTS run first (pytest -m gpu). Output: gpurun_out/ab/<label>_<rep>.json
# and .err, each summarised by tools/bench_brief.py as it lands.
# Examples (HISTORY.md lists the round-5 ones):
#   LEG=wide bash tools/gpu/ab.sh h6,build/xw,CB_SCREEN_HBITS=6 h8,build/xw,CB_SCREEN_HBITS=8
#   LEG=c2_lane bash tools/gpu/ab.sh dflt,lsmt_amd sub18,build/xc2,CB_BUILD_SUB=1
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
: "${LEG:?LEG is required}" "${REPS:=2}" "${STEPS:=20}" "${WARMUP:=3}"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    IFS=, read -r label lib envs <<< "$v"
    envs=${envs//,/ }
    out=$O/${label}_$rep
    case $LEG in
      c2_lane) cmd=(./build/tools/c2_lane "${lib:-lsmt_amd}/libcassbloom.so") ;;
      c3) cmd=(bench.py --no-cpu --steps $STEPS --warmup $WARMUP $ARGS) ;;
      c4) cmd=(bench.py --workload c4 --no-cpu --steps $STEPS --warmup $WARMUP $ARGS) ;;
      *) cmd=(bench.py --leg $LEG --no-cpu --steps $STEPS --warmup $WARMUP $ARGS) ;;
    esac
    if [ $LEG != c2_lane ]; then
      if [ -n "$lib" ]; then cmd=(python tools/expbench.py "${cmd[@]:1}"); envs="EXPBENCH_LIB=$lib/libcassbloom.so $envs"
      else cmd=(python "${cmd[@]}"); fi
    fi
    env $envs timeout -k 10 300 "${cmd[@]}" > $out.json 2> $out.err || { echo "[$label rep $rep] failed"; tail -20 $out.err; exit 1; }
    echo "== $label rep $rep"
    if [ $LEG = c2_lane ]; then cat $out.json; else python tools/bench_brief.py $out.json; fi
  done
done
