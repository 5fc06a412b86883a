#!/bin/bash
# Round 4 evidence on the final kernels: the -m gpu suite, the default bench
# line, rocprofv3 kernel stats + PMC for the default bench workload and for
# C4, and the build phase microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04k.json 2> gpurun_out/bench_r04k.err || { tail -20 gpurun_out/bench_r04k.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04k.json || true
PROF_OUT=gpurun_out/prof_k bash tools/profile_round.sh > gpurun_out/profile_k.log 2>&1 || { tail -20 gpurun_out/profile_k.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_k --json gpurun_out/pmc_k.json > /dev/null
grep -E "^(k_set_probe|k_set_get_many|k_build_part|k_build_tile|k_b64_decode|k_format|k_bin_sort|k_table_buckets) " gpurun_out/prof_k/summary.txt | cut -c1-400
PROF_OUT=gpurun_out/prof_c4k bash tools/profile_round.sh --workload c4 > gpurun_out/profile_c4k.log 2>&1 || { tail -20 gpurun_out/profile_c4k.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_c4k --json gpurun_out/pmc_c4k.json > /dev/null
grep -E "^(k_build_part|k_build_tile)" gpurun_out/prof_c4k/summary.txt | cut -c1-400
timeout -k 10 60 ./build/ubench_build c2 > gpurun_out/ub_c2k.json && timeout -k 10 60 ./build/ubench_build c4 > gpurun_out/ub_c4k.json && cat gpurun_out/ub_c2k.json gpurun_out/ub_c4k.json
