"""CPU checks of bench.py's contract with the driver (no GPU): the defaults
that make `python bench.py` an N=1 run of minutes, the C3 workload shape
BASELINE.json names, and the helpers that fill the JSON line's `roofline`
(committed random-read ceiling and PMC traffic) and `cpu_baseline`
(usable host CPUs)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _parse(argv):
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_defaults_are_the_c3_single_gpu_run():
    a = _parse([])
    assert a.gpus == 1 and a.workload == "c3"
    assert (a.n_keys, a.filters, a.m_bits, a.keys_per_filter) == (1 << 20, 32, 1 << 26, 1 << 19)
    assert (a.build_keys, a.build_m_bits) == (1 << 20, 1 << 27)  # C2
    assert a.steps > 0 and a.warmup >= 0
    assert a.probe_streams in (1, 2, 3, 4) and a.build_streams in (1, 2, 3, 4)


def test_driver_flags_parse():
    a = _parse(["--gpus", "8", "--steps", "20", "--warmup", "3"])
    assert (a.gpus, a.steps, a.warmup) == (8, 20, 3)
    with pytest.raises(SystemExit):
        _parse(["--probe-streams", "5"])
    with pytest.raises(SystemExit):
        _parse(["--build-streams", "5"])  # GPU_MAX_HW_QUEUES is 4 on the box


def test_metric_names_the_baseline_metric():
    import json
    with open(os.path.join(ROOT, "BASELINE.json")) as fh:
        base = json.load(fh)
    text = json.dumps(base).lower()
    assert "probe" in bench.METRIC.lower() and "build" in bench.METRIC.lower()
    assert "probe" in text or "bloom" in text
    assert bench.HBM_PEAK_GBS == 8000.0


def test_roofline_inputs_come_from_committed_profiles():
    rr = bench._random_read_roofline()
    assert rr is not None and 1e10 < rr < 2e11  # reads/s of the measured random-read ceiling
    t = bench._pmc_traffic("k_set_probe")
    assert t is not None and 1e8 < t < 1e9  # HBM bytes per C3 launch (PMC)
    assert bench._pmc_traffic("no_such_kernel") is None


def test_host_cpus_is_consistent():
    c = bench.host_cpus()
    assert 1 <= c["usable"] <= c["nproc"]
    assert c["usable"] <= c["affinity"]
    if c["cgroup_quota"]:
        assert c["usable"] <= c["cgroup_quota"]
    assert "nproc" in c["note"]


def test_gpu_scripts_parse_and_name_existing_legs():
    # tools/gpu/*.sh are what a round runs on the box (full validation,
    # profiles, A/Bs): syntax-checked here, and the A/B driver's legs and the
    # profile shapes must be ones bench.py / profile_round.sh accept
    import glob
    import subprocess
    scripts = sorted(glob.glob(os.path.join(ROOT, "tools", "gpu", "*.sh")))
    assert {os.path.basename(s) for s in scripts} >= {"ab.sh", "full.sh", "profiles.sh"}
    for s in scripts + [os.path.join(ROOT, "tools", "profile_round.sh")]:
        subprocess.run(["bash", "-n", s], check=True)
    a = _parse(["--leg", "c5"])
    assert a.leg == "c5" and _parse(["--leg", "wide"]).leg == "wide"
    assert _parse(["--workload", "c4"]).workload == "c4"
    text = open(os.path.join(ROOT, "tools", "profile_round.sh")).read()
    for shape in ("c3)", "c4)", "c5)", "wide)"):
        assert shape in text


def test_compact_line_fits_the_driver_tail():
    """The stdout line stays under 8 KB with every leg present, ends with the
    legs the driver's ~9 KB tail must show (build, e2e, cold, may_contain),
    and keeps the contract keys and each leg's numbers (the 14.7
    KB round-5 line lost build, e2e and cold to the tail). Input: round 5's
    full default line (profiles/bench_r05k.json) with a round-6-sized build
    roofline added."""
    import json
    with open(os.path.join(ROOT, "profiles", "bench_r05k.json")) as fh:
        line = json.load(fh)
    line["build"]["roofline"] = {"bound": "hbm", "achieved": 2171.3, "peak": 8000.0, "unit": "GB/s",
                                 "frac": 0.4903, "frac_one_lane": 0.2714, "kernel": "k_build_part+k_build_tile",
                                 "kernel_avg_us": 8.55, "kernel_avg_source": "x" * 200,
                                 "algorithmic_bytes": 33554432, "algorithmic_def": "y" * 120,
                                 "traffic": 41234567, "traffic_over_algorithmic": 1.229,
                                 "traffic_source": "profiles/pmc_c2_r06.json",
                                 "profile_check": {"source": "z" * 80, "kernels": ["k_build_part", "k_build_tile"],
                                                   "step_us": 15.4, "frac": 0.2721,
                                                   "ratio_to_line_frac_one_lane": 1.0026}}
    c = bench.compact_line(line)
    text = json.dumps(c, separators=(",", ":"))
    assert len(text) <= bench.LINE_BUDGET, len(text)
    keys = list(c)
    assert keys[-4:] == ["build", "e2e", "cold", "may_contain"]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in c, k
    assert c["roofline"]["frac"] == line["roofline"]["frac"] and c["roofline"]["traffic"]
    assert c["cpu_baseline"]["sample"] and c["cpu_baseline"]["kind"] == "port"
    b = c["build"]
    assert b["value"] and b["one_lane"]["us_per_build"] and b["roofline"]["frac"] and b["roofline"]["traffic"]
    assert "error" not in json.dumps(c["may_contain"])
    assert c["c5"]["golden_slice_bit_exact"] is True and c["c4"]["roofline"]["traffic"]
    # numbers survive: every leg's value is the full line's, rounded
    for leg in ("c4", "c5", "wide_fanout", "read_path"):
        assert abs(c[leg]["value"] - line[leg]["value"]) < 1


def test_c2_leg_and_profile_shape_exist():
    assert _parse(["--leg", "c2"]).leg == "c2"
    text = open(os.path.join(ROOT, "tools", "profile_round.sh")).read()
    assert "c2)" in text and "--leg c2" in text and "--build-streams 1" in text


def test_compact_line_of_this_round_fits_at_eight_ranks():
    """This round's full default line (profiles/bench_r06o_full.json), with
    what a line at N = 8 adds (the exchange's mode and counters, one
    rccl_world entry per rank), still compacts under the budget, the tail
    legs last; the N = 1-only legs (read path, wide fan-out) only shrink it."""
    import json
    with open(os.path.join(ROOT, "profiles", "bench_r06o_full.json")) as fh:
        line = json.load(fh)
    line["n_gpus"] = 8
    line["exchange"] = {"sparse_steps": 20, "mode": "sparse", "cap": 1234567, "all_fit": True}
    line["rccl_world"] = [8] * 8
    c = bench.compact_line(line)
    text = json.dumps(c, separators=(",", ":"))
    assert len(text) <= bench.LINE_BUDGET, len(text)
    assert list(c)[-4:] == ["build", "e2e", "cold", "may_contain"]
    assert c["rccl_world"] == [8] * 8 and c["exchange"]["mode"] == "sparse"
    assert c["wide_fanout"]["one_lane"]["value"] and c["wide_fanout"]["lanes_equal"] is True
