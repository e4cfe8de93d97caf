import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kube-dtn_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and runs the HIP path")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "samples.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    from kdtn import Engine
    eng = Engine(device=0, tick_in_usec=15.625, vxlan_base=5000)
    yield eng
    eng.close()
