#!/bin/bash
# Round 5: request sizes and rates of random 4-B reads by load flavour
# (tools/ubench_fill.hip, prebuilt into build/tools/ubench_fill).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/fill
mkdir -p $O
B=build/tools/ubench_fill
timeout -k 10 120 $B > $O/plain.json 2> $O/plain.err || exit 1
cat $O/plain.json
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d $O/p1 -o p1 --output-format csv -- $B > $O/p1.json 2> $O/p1.err || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o p2 --output-format csv -- $B > $O/p2.json 2> $O/p2.err || exit 1
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/r05/fill"
rows = collections.defaultdict(dict)
for p in ("p1", "p2"):
    for f in glob.glob(f"{O}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Kernel_Name"][:40])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
for k in sorted(rows, key=lambda x: int(x[0])):
    print(k, {n: int(v) for n, v in rows[k].items()})
PY
