import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def golden():
    return load_golden
