import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def orc():
    from oracle import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def galois_fixture():
    import json

    import numpy as np

    with open(os.path.join(ROOT, "tests", "golden", "galois_tables.json")) as f:
        g = json.load(f)
    return {k: np.frombuffer(bytes.fromhex(g[k]), np.uint8) for k in ("GINV", "GEXP", "GMULT")}
