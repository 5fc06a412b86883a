#!/bin/bash
# Parity suite then one bench line (no CPU baseline) and a PMC-priced profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e $* > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['path'],round(d['value']/1e9,1),'Gp/s',d['ms_per_step'],d['kernels_us'],'alt',d['alt_paths'],d['alt_kernels_us'],'build',d['build']['ms_per_step'],d['build']['kernels'])"
bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
python - <<'PY'
import json, subprocess
out = subprocess.run(["python", "tools/pmc_summary.py", "gpurun_out/prof"], capture_output=True, text=True).stdout
for line in out.splitlines():
    k, j = line.split(" ", 1)
    if k.startswith("k_"):
        e = json.loads(j)
        print(k, e["avg_us"], "rd", round(e.get("read_bytes", 0) / 1e6, 1), "wr", round(e.get("write_bytes", 0) / 1e6, 1), e.get("hbm_GBps"))
PY
