#!/bin/bash
# The round's validation: the whole -m gpu suite, smoke(), then the default
# bench line (gpurun_out/full/bench_full.json).
set -o pipefail
O=${OUT:-gpurun_out/full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { tail -30 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --full-line $O/bench_full_line.json > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 1; }
wc -c $O/bench_full.json
python tools/bench_brief.py $O/bench_full.json
