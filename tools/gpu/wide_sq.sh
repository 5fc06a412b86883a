set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
B="python bench.py --leg wide --no-cpu --steps 10 --warmup 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM -d $O/sqa -o sqa --output-format csv -- $B > /dev/null 2> $O/sqa.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_VMEM_TA_ADDR_FIFO_FULL -d $O/sqb -o sqb --output-format csv -- $B > /dev/null 2> $O/sqb.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS_LOAD SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR TA_BUSY_avr TA_TA_BUSY_sum -d $O/sqc -o sqc --output-format csv -- $B > /dev/null 2> $O/sqc.err || true
python - <<'PY'
import csv, glob, collections
for d in ("sqa","sqb","sqc"):
    for f in glob.glob(f"gpurun_out/r06i/{d}/*counter_collection.csv"):
        acc=collections.defaultdict(list)
        per=collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "wide_get_many" not in r["Kernel_Name"]: continue
            per[(r["Dispatch_Id"], r["Counter_Name"])]+=float(r["Counter_Value"])
        for (di,c),v in per.items(): acc[c].append(v)
        print(d, {c: round(sum(v)/len(v)) for c,v in acc.items()})
PY
