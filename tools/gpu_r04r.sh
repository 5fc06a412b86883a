#!/bin/bash
# Round 4: what bounds C4's partition pass — SQ counters for k_build_part
# (k_build_part_loop was removed after this A/B: profiles/part_loop_ab_r04.json)
# (CB_BUILD_LOOP=0) and k_build_part_loop, one lane, experiment library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/sq/avail.txt 2>&1 || true
B="python3 tools/expbench.py --workload c4 --steps 10 --warmup 3 --no-cpu --probe-streams 1"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"; do
  i=$((i+1))
  for v in 0 1; do
    CB_BUILD_LOOP=$v timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/sq/p${i}_$v -o p --output-format csv -- $B > /dev/null 2> gpurun_out/sq/p${i}_$v.err || { echo "pass $i/$v failed"; tail -5 gpurun_out/sq/p${i}_$v.err; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for v in ("0", "1"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/sq/p*_{v}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_build_part" not in k: continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), x in per.items(): acc[c].append(x)
    print("loop=" + v, {c: round(sum(x) / len(x)) for c, x in sorted(acc.items())})
PY
