"""Summarise tools/profile_round.sh output: per-kernel average duration
(kernel trace) and HBM-side bytes per launch from the PMC passes.

Read bytes are priced per request size (32/64/128 B request counters) because
gfx950's FETCH_SIZE counts a 128-B request as 64 B (MI355X_MICROARCH.md §HBM);
FETCH_SIZE is reported beside it. WRITE_SIZE is exact for 16-B/lane stores.
Usage: python tools/pmc_summary.py gpurun_out/prof [--json out.json] [key=value ...]
(key=value pairs are copied into the JSON, e.g. shape=c4 filters_per_launch=64)
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)", "anon").replace("void ", "")
    name = name.split("(")[0]
    return name.split("<")[0].split("::")[-1]


def main():
    root = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    meta = {}
    for a in sys.argv[2:]:
        if "=" in a:
            k, v = a.split("=", 1)
            meta[k] = int(v) if v.isdigit() else v
    dur = {}
    stats = glob.glob(os.path.join(root, "kt", "*kernel_stats.csv"))
    if stats:
        for r in csv.DictReader(open(stats[0])):
            k = short(r["Name"])
            c, t = int(r["Calls"]), float(r["TotalDurationNs"])
            if k in dur:  # template instances of one kernel: merged
                c, t = c + dur[k]["calls"], t + dur[k]["avg_us"] * 1e3 * dur[k]["calls"]
            dur[k] = {"calls": c, "avg_us": t / c / 1e3}
    # the one-lane trace (kt1: launches do not overlap, so a dispatch's
    # duration is the kernel's own time): the figure bench.py's profile check
    # compares with its event-timed one-lane step
    dur1 = {}
    stats1 = glob.glob(os.path.join(root, "kt1", "*kernel_stats.csv"))
    if stats1:
        for r in csv.DictReader(open(stats1[0])):
            k = short(r["Name"])
            c, t = int(r["Calls"]), float(r["TotalDurationNs"])
            if k in dur1:  # template instances of one kernel: merged
                c, t = c + dur1[k]["calls"], t + dur1[k]["avg_us"] * 1e3 * dur1[k]["calls"]
            dur1[k] = {"calls": c, "avg_us": t / c / 1e3}
    # busy time per launch: the union of each kernel's [start, end) intervals
    # over its dispatches, / dispatches (= the average duration when launches
    # do not overlap; the per-step share when pipeline lanes overlap them)
    busy = {}
    traces = glob.glob(os.path.join(root, "kt", "*kernel_trace.csv"))
    if traces:
        iv = collections.defaultdict(list)
        for r in csv.DictReader(open(traces[0])):
            iv[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        for k, lst in iv.items():
            lst.sort()
            tot, cur_s, cur_e = 0, None, None
            for s0, e0 in lst:
                if cur_e is None or s0 > cur_e:
                    if cur_e is not None:
                        tot += cur_e - cur_s
                    cur_s, cur_e = s0, e0
                else:
                    cur_e = max(cur_e, e0)
            if cur_e is not None:
                tot += cur_e - cur_s
            busy[k] = tot / len(lst) / 1e3
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(int(r["Dispatch_Id"]), short(r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, k, c), v in per.items():
            ctr[k][c].append(v)
    res = {}
    for k in sorted(set(dur) | set(dur1) | set(ctr)):
        c = {n: sum(v) / len(v) for n, v in ctr[k].items()}
        e = {"avg_us": round(dur.get(k, {}).get("avg_us", 0.0), 3), "calls": dur.get(k, {}).get("calls", 0)}
        if k in busy:
            e["busy_us_per_launch"] = round(busy[k], 3)
        if k in dur1:
            e["avg_us_one_lane"] = round(dur1[k]["avg_us"], 3)
            e["calls_one_lane"] = dur1[k]["calls"]
        e.update({n: round(v, 1) for n, v in c.items()})
        if all(n in c for n in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
            rd = 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + 128 * c["TCC_EA0_RDREQ_128B_sum"]
            e["read_bytes"] = int(rd)
        if "WRITE_SIZE" in c:
            e["write_bytes"] = int(c["WRITE_SIZE"] * 1024)
        if "read_bytes" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["read_bytes"] + e["write_bytes"]
            t = e.get("busy_us_per_launch") or e["avg_us"]
            if t:
                e["hbm_GBps"] = round(e["hbm_bytes_per_launch"] / (t * 1e3), 1)
        res[k] = e
    # the bench's own one-lane step (HIP events) in the traced run (kt1) and
    # in the plain run before it, for the shape the summary is for
    lines = {}
    for tag, fn in (("traced", "kt1_bench.json"), ("plain", "plain1_bench.json")):
        try:
            d = json.loads(open(os.path.join(root, fn)).read().strip().splitlines()[-1])
        except Exception:
            continue
        shape = meta.get("shape")
        us = None
        if shape == "c4" and d.get("c4"):
            us = d["c4"].get("one_lane_us_per_step")
        elif shape == "c5" and d.get("c5"):
            us = d["c5"].get("one_lane_us_per_step")
        elif shape == "wide" and d.get("wide_fanout"):
            us = d["wide_fanout"].get("kernels_us", {}).get("k_wide_get_many")
        elif shape == "c2" and d.get("build"):
            us = d["build"].get("one_lane", {}).get("us_per_build")
        elif shape == "c3" and d.get("roofline"):
            us = d["roofline"].get("kernel_avg_us_one_lane")
        if us:
            lines[tag] = us
    if lines:
        meta["events_one_lane_us"] = lines
    for k, e in res.items():
        print(k, json.dumps(e))
    if out_json:
        with open(out_json, "w") as fh:
            json.dump(dict({"source": "tools/profile_round.sh + tools/pmc_summary.py", "kernels": res}, **meta), fh,
                      indent=1)


if __name__ == "__main__":
    main()
