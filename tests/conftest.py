import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs (set GM_SLOW=1)")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("GM_SLOW"):
        return
    skip = pytest.mark.skip(reason="slow oracle case; set GM_SLOW=1")
    for it in items:
        if "slow" in it.keywords:
            it.add_marker(skip)
