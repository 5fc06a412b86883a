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
