"""Shared fixtures. `-m gpu` tests need an MI355X; everything else runs on CPU."""
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
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblrt_hip.so)")
    config.addinivalue_line("markers", "slow: exhaustive sweeps (opt in with LRT_EXHAUSTIVE=1)")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def images():
    with np.load(os.path.join(GOLDEN, "images.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu():
    """Initialise the library on cuda:0 once per session (fails loudly without it)."""
    import learnraytracing_amd as lrt
    lrt.InitializeTest()
    yield lrt
    lrt.ShutdownTest()
