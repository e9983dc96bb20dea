import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zstd-decompressor_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C ABI")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def resources():
    d = os.path.join(ROOT, "tests", "golden", "resources")
    return {n: open(os.path.join(d, n), "rb").read() for n in sorted(os.listdir(d))}
