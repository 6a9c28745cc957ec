import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "trik-media-sensors-dsp_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "oracle_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def table(oracle_mod):
    """The oracle's 2^24-entry (rgb << 32 | hsv) table, index Y | U<<8 | V<<16."""
    return oracle_mod.yuv_table(closed=False)
