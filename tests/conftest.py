"""Shared test setup: the `gpu` marker, repo paths, golden-fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def golden(name):
    path = os.path.join(GOLDEN, name)
    if name.endswith(".json"):
        with open(path) as f:
            return json.load(f)
    return np.load(path, allow_pickle=False)


@pytest.fixture(scope="session")
def maps():
    m = golden("maps.npz")
    return {k: m[k] for k in m.files}
