import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through the C ABI")
    config.addinivalue_line("markers", "slow: large-config test (seconds to tens of seconds)")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def gpu():
    """The product module on a real GPU. Fails (not skips) without one: the
    gpu-marked tests are only selected where a GPU is expected."""
    import lsmt_amd
    n = lsmt_amd.device_count()
    assert n > 0, "gpu-marked test selected but no HIP device is visible"
    return lsmt_amd
