#!/bin/bash
# PMC passes on the read leg (one lane): where k_get_many's time goes.
set -o pipefail
mkdir -p gpurun_out/gm
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-e2e --no-cold --no-flush --probe-streams 1 --steps 20 --warmup 2"
for form in cur; do
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/gm/$form$i -o p$i --output-format csv -- $B > /dev/null 2> gpurun_out/gm/$form$i.err || { echo "pass $form $i failed"; tail -3 gpurun_out/gm/$form$i.err; exit 1; }
done
done
python3 - <<'PY'
import csv, glob, collections
for form in ("cur",):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/gm/{form}*/*counter_collection.csv"):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)", "anon").replace("void ", "").split("(")[0].split("<")[0].split("::")[-1]
            per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, k, c), v in per.items():
            agg[k][c].append(v)
    out = {}
    for k in ("k_set_get_many", "k_get_many", "k_b64_decode", "k_set_probe"):
        if agg[k]:
            out[k] = {c: round(sum(v) / len(v)) for c, v in sorted(agg[k].items())}
            print(form, k, out[k])
    import json
    json.dump({"source": "rocprofv3 --pmc, one pass per group, bench.py read leg with --probe-streams 1; "
                         "per-dispatch counter sums averaged over dispatches", "kernels": out},
              open("gpurun_out/readpath_pmc.json", "w"), indent=1)
PY
