#!/bin/bash
# Round 5: the SSTable/flush GPU tests (bucket-event change), then one-lane
# C2 build latency (tools/c2_lane.hip) over the library built at each round-4
# commit that touched the build path, alternating, two passes; then the
# default bench line for this box.
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_sstable_gpu.py tests/test_flush_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_sst.log 2>&1 || { tail -30 $O/pytest_sst.log; exit 1; }
tail -1 $O/pytest_sst.log
LIBS="build/bisect/782570e build/bisect/85e71a5 build/bisect/56f9528 build/bisect/39859eb build/bisect/3fba026 build/bisect/f64c10e build/bisect/0ed8fcf build/bisect/1b6e81d lsmt_amd"
for pass in 1 2; do
  for d in $LIBS; do
    timeout -k 10 60 ./build/tools/c2_lane $d/libcassbloom.so >> $O/c2_lane.jsonl 2>> $O/c2_lane.err || { tail -5 $O/c2_lane.err; exit 1; }
  done
done
cat $O/c2_lane.jsonl
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python tools/bench_brief.py $O/bench_default.json
