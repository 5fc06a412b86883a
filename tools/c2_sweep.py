"""C2 (one build of 1M keys -> m = 2^27) under build-knob settings of the
experiment library (tools/expbench.py): one process per setting, printing
the bench's C2 build field (four lanes, one lane, kernel times). Usage:
python tools/c2_sweep.py ['[{"CB_BUILD_KPT": "2"}, ...]'] > out.jsonl"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS = [{}, {"CB_BUILD_KPT": "2"}, {"CB_BUILD_KPT": "1"}, {"CB_BUILD_TB": "18"},
            {"CB_BUILD_TB": "18", "CB_BUILD_KPT": "2"}, {"CB_BUILD_TILE_NT": "512", "CB_BUILD_TB": "18"}]
if len(sys.argv) > 1:
    SETTINGS = json.loads(sys.argv[1])
for env in SETTINGS:
    e = dict(os.environ, **env)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "expbench.py"), "--steps", "20", "--warmup", "5",
                        "--leg-steps", "200", "--no-cpu", "--no-e2e", "--no-cold", "--no-zone", "--no-read",
                        "--no-flush", "--no-c4", "--no-c5", "--no-wide"],
                       capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)
    if p.returncode:
        print(json.dumps({"env": env, "error": p.stderr[-800:]}), flush=True)
        break
    b = json.loads(p.stdout.strip().splitlines()[-1])["build"]
    print(json.dumps({"env": env, "us_per_step_4_lanes": b["region_us_per_step"], "one_lane_us": b["one_lane"]["us_per_build"],
                      "kernels_us": b["kernels"]}), flush=True)
