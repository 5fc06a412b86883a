"""C4 (64 concurrent builds of 2^18 keys, m = 2^25) under build-knob settings
of the experiment library (tools/expbench.py): one process per setting,
printing the bench's C4 step (HIP events) and kernel times. Usage: python
tools/c4_sweep.py [steps] > out.jsonl"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
steps = sys.argv[1] if len(sys.argv) > 1 else "100"
SETTINGS = [{}, {"CB_BUILD_TB": "18"}, {"CB_BUILD_TILE_NT": "512", "CB_BUILD_TB": "18"},
            {"CB_BUILD_TILE_NT": "512", "CB_BUILD_TB": "17"}, {"CB_BUILD_TILE_NT": "512"}, {"CB_BUILD_BATCH": "8"}]
if len(sys.argv) > 2:  # a JSON list of settings instead
    SETTINGS = json.loads(sys.argv[2])
for lanes in ("1", "3"):
    for env in SETTINGS:
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "expbench.py"), "--workload", "c4",
                            "--steps", steps, "--warmup", "5", "--no-cpu", "--probe-streams", lanes]
                           + (["--check"] if os.environ.get("C4_SWEEP_CHECK") == "1" else []),
                           capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)
        if p.returncode:
            print(json.dumps({"env": env, "lanes": lanes, "error": p.stderr[-800:]}), flush=True)
            break
        d = json.loads(p.stdout.strip().splitlines()[-1])
        leg = d["c4"]
        print(json.dumps({"env": env, "lanes": lanes, "golden": d.get("golden_all_filters_bit_exact", leg.get("golden_all_filters_bit_exact")),
                          "region_us_per_step": leg["region_us_per_step"],
                          "one_lane_us_per_step": leg["one_lane_us_per_step"], "ms_per_step": leg["ms_per_step"],
                          "kernels_us": leg["kernels_us"]}), flush=True)
