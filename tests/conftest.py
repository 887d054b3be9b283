import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU-side parity cases")


def pytest_collection_modifyitems(config, items):
    # GPU tests need a visible device; on the CPU container they are deselected by -m "not gpu".
    pass


@pytest.fixture(scope="session")
def nba_data():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "nba.json")) as f:
        return json.load(f)


@pytest.fixture(params=["chain", "host"])
def sp_mode(request, monkeypatch):
    """Both one-pair FIND SHORTEST PATH paths (NBG_SP_MODE, read per query): the
    device-driven level loop (default) and the host-driven level loop."""
    monkeypatch.setenv("NBG_SP_MODE", request.param)
    return request.param
