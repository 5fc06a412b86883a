#!/bin/bash
# Round evidence on one GPU: the default bench line (N=1, CPU baselines
# included), then the rocprofv3 kernel-trace + PMC passes and their summary.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_full.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['read_path']['value'],d['flush']['unsorted_input']['ms_per_flush'])"
bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof --json gpurun_out/pmc_round.json > /dev/null
tail -12 gpurun_out/profile_round.log
