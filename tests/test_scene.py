"""The build-defined 1000-sphere scene (BASELINE configs 4-5) is deterministic and has
the documented shape."""
import numpy as np

from learnraytracing_amd import _lib as L
from learnraytracing_amd.scene import _XorShift32, random_scene, scene_arrays, scene_from_arrays

import oracle


def test_generator_rng_is_the_reference_rng(kat):
    r = _XorShift32(1)
    assert [r.next() for _ in range(16)] == kat["xorshift32_from_1"]
    r = _XorShift32(1)
    assert np.array_equal(np.array([r.f01() for _ in range(16)], np.float32),
                          np.array(kat["random01_from_1"], np.float32))


def test_random_scene_deterministic_and_shaped():
    a = scene_arrays(*random_scene(1000, 1))
    b = scene_arrays(*random_scene(1000, 1))
    c = scene_arrays(*random_scene(1000, 2))
    assert a == b and a != c
    s = np.array(a[0], np.float32).reshape(-1, 4)
    m = np.array(a[1], np.float32).reshape(-1, 9)
    assert s.shape == (1000, 4) and m.shape == (1000, 9)
    assert np.array_equal(s[0], [0, -100.5, -1, 100])
    emissive = np.nonzero((m[:, 4:7] > 0).any(axis=1))[0]
    assert emissive.tolist() == [1]
    types = np.bincount(m[:, 0].astype(int), minlength=3)
    assert types[0] > 600 and types[1] > 120 and types[2] > 50
    small = s[2:]
    assert (small[:, 3] >= 0.05).all() and (small[:, 3] <= 0.12).all()
    assert np.allclose(small[:, 1], small[:, 3] - 0.5, atol=1e-6)   # resting on the ground


def test_scene_roundtrip():
    sph, mat = random_scene(50, 3)
    s, m = scene_arrays(sph, mat)
    s2, m2 = scene_arrays(*scene_from_arrays(s, m))
    assert np.array_equal(np.float32(s), np.float32(s2)) and np.array_equal(np.float32(m), np.float32(m2))


def test_oracle_renders_random_scene():
    s, m = (np.array(v, np.float32) for v in scene_arrays(*random_scene(200, 5)))
    buf, rays = oracle.orc_render(48, 27, 1, 8, spheres=s, mats=m)
    assert rays >= 48 * 27 and np.isfinite(buf).all()
    assert L.MAX_SPHERES >= 1000
