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


def _scene_bytes(scene):
    sph, mat = scene
    return b"".join(bytes(x) for x in sph) + b"".join(bytes(x) for x in mat)


@pytest.fixture(autouse=True)
def _scene_guard(request):
    """GPU tests start on the reference's default scene (parallel.cpp:15-51). A test that
    changes the scene restores it (try/finally, or a function-scoped scene fixture); one that
    does not would hand its scene to whatever test runs next -- the r3_ae red run, where a
    9-sphere oracle comparison rendered a module fixture's 1000-sphere scene -- so the leak is
    reported here, loudly, at the next test's start."""
    if "gpu" in request.keywords and "gpu" in request.fixturenames:
        import learnraytracing_amd as lrt
        if lrt.lib().lrt_device_count() > 0 and _scene_bytes(lrt.get_scene()) != _scene_bytes(lrt.default_scene()):
            lrt.set_scene(*lrt.default_scene())
            pytest.fail("the library held a non-default scene at this test's start: an earlier test leaked it "
                        "(it was reset to the default scene)")
    yield
