#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/ov -o ov --output-format csv -- python bench.py --no-cpu --no-e2e --force-dist --steps 10 > gpurun_out/tr/ov.json 2> gpurun_out/tr/ov.err || { tail -20 gpurun_out/tr/ov.err; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/tr/ov/*kernel_trace.csv")[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# find a window of k_set_probe launches in the timed legs
idx = [i for i, r in enumerate(rows) if "k_set_probe" in r["Kernel_Name"]]
sel = rows[idx[5] - 4: idx[5] + 12]
t0 = int(sel[0]["Start_Timestamp"])
for r in sel:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{s/1e3:9.2f} {e/1e3:9.2f} {(e-s)/1e3:7.2f} q{r["Queue_Id"]:>3} {r["Kernel_Name"][:60]}')
PY
