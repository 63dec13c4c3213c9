import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); runs on the GPU box")


def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)


def load_case(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    with open(os.path.join(GOLDEN, name + ".gz"), "rb") as f:
        gz = f.read()
    return meta, gz


CASES = manifest()["cases"]
CORRUPT = manifest()["corrupt"]


@pytest.fixture(scope="session")
def device():
    import parallelparsing_amd as pp
    return pp.Device.default(0)
