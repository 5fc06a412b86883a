"""Synthetic key generator (lsmt_amd/workload.py) vs the oracle's C generator
and the golden fixture."""
import hashlib

import numpy as np

from lsmt_amd import workload
from oracle import oracle


def test_keys_match_golden_and_oracle(golden):
    k = workload.key_range(1, 2000)
    assert [bytes(r).decode() for r in k[:8]] == golden["keys_seed1_first8"]
    assert hashlib.sha256(k.tobytes()).hexdigest() == golden["keys_seed1_2000_sha256"]
    assert np.array_equal(k, oracle.gen_keys(1, 2000))
    assert np.array_equal(workload.key_range(77, 50, first=123), oracle.gen_keys(77, 50, first=123))


def test_keys_distinct_and_hex():
    k = workload.key_range(3, 200_000)
    assert len(np.unique(k.view("S16"))) == 200_000
    assert set(np.unique(k)).issubset(set(b"0123456789abcdef"))


def test_probe_lookups_layout():
    look = workload.probe_lookups(1000, 4, 100, seed_base=100, absent_seed=999)
    # even i -> present key(100 + j%4, (j//4) % 100), j = i/2
    for i in (0, 2, 10, 998):
        j = i // 2
        assert bytes(look[i]) == bytes(workload.keys(100 + j % 4, [(j // 4) % 100])[0])
    assert bytes(look[7]) == bytes(workload.keys(999, [7])[0])


def test_var_keys_shape():
    rng = np.random.default_rng(0)
    data, offs = workload.var_keys(rng, 100)
    assert offs[0] == 0 and offs[-1] == len(data) and np.all(np.diff(offs.astype(np.int64)) >= 0)
