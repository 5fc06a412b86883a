#!/bin/bash
# Translation (UTCL1) and latency counters per kernel for one bench command
# (round 6 diagnosis of the latency-bound read kernels). One --pmc pass per
# counter group (at most 4 TCP counters each), kernel names reduced, averages
# per dispatch printed for the kernels named on the command line.
# Usage: bash tools/gpu/tlb_pmc.sh "<bench command>" kernel [kernel ...]
# PMC_GROUPS="grp;grp": other counter groups, one pass each (O: PMC_OUT).
set -o pipefail
export TMPDIR=/tmp
O=${PMC_OUT:-gpurun_out/tlb}
mkdir -p $O
CMD=$1
shift
GRPS=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
      "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_TA_ADDR_STALL_CYCLES_sum TCP_TA_DATA_STALL_CYCLES_sum"
      "TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_LFIFO_FULL_sum")
[ -n "$PMC_GROUPS" ] && IFS=';' read -r -a GRPS <<< "$PMC_GROUPS"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $O/p$i -o p$i --output-format csv -- $CMD > /dev/null 2> $O/p$i.err || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 1; }
done
python - "$O" "$@" <<'PY'
import collections, csv, glob, sys
want = sys.argv[2:]
def short(n):
    n = n.replace("(anonymous namespace)", "anon").replace("void ", "").split("(")[0]
    return n.split("<")[0].split("::")[-1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k in want:
            per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, k, c), v in per.items():
        acc[k][c].append(v)
for k in want:
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(acc[k].items())})
PY
