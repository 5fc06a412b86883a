"""One-screen summary of a bench.py JSON line (the legs a round compares)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])  # the line (a leg run prints only its leg)
r = d.get("roofline")
if r:
    print(f"probe C3 {d['value'] / 1e12:.3f} T/s {d['ms_per_step'] * 1e3:.1f} us/step  frac {r['frac']} "
          f"one-lane {r.get('frac_one_lane')} ({r.get('kernel_avg_us_one_lane')} us)  "
          f"rr {r['random_read_roofline']['frac']}")
b = d.get("build")
if b:
    br = b.get("roofline") or {}
    print(f"build C2 {b['value'] / 1e9:.1f} G keys/s {b['ms_per_step'] * 1e3:.2f} us/step lanes {b.get('pipeline_lanes')} "
          f"one-lane {b.get('one_lane', {}).get('us_per_build')} us cold {(b.get('cold') or {}).get('ms_per_step')} ms "
          f"frac {br.get('frac')} one-lane {br.get('frac_one_lane')} traffic {br.get('traffic')} "
          f"{b.get('kernels_us', b.get('kernels'))}")
rp = d.get("read_path")
if rp:
    print(f"read path {rp['value'] / 1e9:.2f} G gets/s")
f = d.get("flush")
if f:
    for k in ("sorted_input", "unsorted_input", "unsorted_shared_prefix_input"):
        if k in f:
            print(f"flush {k}: {f[k]['ms_per_flush']} ms  {f[k].get('kernels_us', '')}")
for k in ("c4", "c5"):
    leg = d.get(k)
    if leg:
        rf = leg.get("roofline", {})
        print(f"{k}: {leg['value'] / (1e9 if k == 'c4' else 1e12):.3f} {'G keys' if k == 'c4' else 'T probes'}/s "
              f"region {leg['region_us_per_step']} us/step one-lane {leg['one_lane_us_per_step']} us frac {rf.get('frac')} "
              f"golden {leg.get('golden_all_filters_bit_exact', leg.get('golden_slice_bit_exact'))} "
              f"oracle {leg.get('oracle_sample_bit_exact', leg.get('oracle_row_bit_exact'))} {leg.get('kernels_us', '')}")
w = d.get("wide_fanout")
if w:
    print(f"wide fan-out: {w['value'] / 1e6:.2f} M gets/s over {w['tables']} tables, oracle {w.get('oracle_sample_bit_exact')} "
          f"{w['kernels_us']}")
