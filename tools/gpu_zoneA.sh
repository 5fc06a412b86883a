#!/bin/bash
# Zone-read events without the system fence: zone / read-path parity tests,
# then the bench's zone-gated and read legs (three runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "zone or get_many or gated or sstable" > gpurun_out/pytest_zone.log 2>&1 || { tail -30 gpurun_out/pytest_zone.log; exit 1; }
tail -1 gpurun_out/pytest_zone.log
for i in 1 2 3; do
timeout -k 10 400 python bench.py --no-cpu --no-e2e --no-cold --no-flush --steps 50 > gpurun_out/bench_z$i.json 2> gpurun_out/bench_z.err || { tail -20 gpurun_out/bench_z.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench_z$i.json'))
print('run $i probe',round(d['value']/1e12,3),'zone',round(d['zone_gate']['value']/1e12,3),d['zone_gate']['ms_per_step'],'read',round(d['read_path']['value']/1e9,2))"
done
