"""The device Scatter in the reference's shape (lrt_trace.h `Scatter`, parallel.cpp:78-196)
against the reference's own Scatter (oracle/_ref, ref_scatter), case by case.

Cases are real hits: random rays through the scene, their closest hit found by the
reference's HitWorld (parallel.cpp:54-73), then Scatter from a random RNG state. Every
output must be bit-identical: the bool (Metal's absorption, :147), the attenuation, the
scattered Ray (its ctor's second normalisation, maths.h:133-137), lightE (the light loop,
:93-133, the self test :98), the counted shadow rays and the RNG state after.

Scenes: the reference's 9 spheres, fuzzed 9-sphere scenes (1-3 lights, TIR, rough metal,
emissive spheres hit directly), and random_scene(1000, 1) (shadow rays through the BVH;
libref1000.so). The CPU test runs the host build of the device code; the GPU test runs
one thread per case on the device (lrt_scatter_eval, on_device = 1).
"""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import oracle  # noqa: E402  (test infrastructure)

from learnraytracing_amd import _lib as L  # noqa: E402
from learnraytracing_amd.scene import random_scene, scene_arrays, scene_from_arrays  # noqa: E402

_P = ctypes.c_void_p


def _ptr(a):
    return a.ctypes.data_as(_P)


def make_cases(lib, s, n_cases, seed):
    """(ids, rays, recs, seeds): hits found by the reference's HitWorld on its current scene."""
    g = np.random.default_rng(seed)
    cnt = len(s) // 4
    ids, rays, recs = [], [], []
    out = np.zeros(7, np.float32)
    tries = 0
    while len(ids) < n_cases and tries < 50 * n_cases:
        tries += 1
        if tries % 4 == 0:   # from inside / near a sphere: inside hits, dielectric exits
            k = int(g.integers(0, cnt))
            o = s[4 * k:4 * k + 3] + g.normal(0, 0.3 * abs(s[4 * k + 3]) + 1e-3, 3)
        else:
            o = g.uniform([-4, -0.4, -6], [4, 3, 4])
        d = g.normal(size=3)
        o = o.astype(np.float32)
        d = d.astype(np.float32)
        i = lib.ref_hit_world(_ptr(o), _ptr(d), ctypes.c_float(0.001), ctypes.c_float(1e7), _ptr(out))
        if i < 0:
            continue
        ids.append(i)
        rays.append(np.concatenate([o, d]))
        recs.append(out.copy())
    seeds = (g.integers(0, 2**32, len(ids), dtype=np.uint64).astype(np.uint32) | 1).astype(np.uint32)
    return (np.array(ids, np.int32), np.array(rays, np.float32).reshape(-1),
            np.array(recs, np.float32).reshape(-1), seeds)


def ref_scatter(lib, ids, rays, recs, seeds):
    n = len(ids)
    out = np.zeros((n, 12), np.float32)
    ret = np.zeros(n, np.int32)
    cnt = np.zeros(n, np.int32)
    st = np.zeros(n, np.uint32)
    o12 = np.zeros(12, np.float32)
    c = ctypes.c_int(0)
    u = ctypes.c_uint32(0)
    for i in range(n):
        ret[i] = lib.ref_scatter(int(ids[i]), _ptr(rays[6 * i:6 * i + 6]), _ptr(recs[7 * i:7 * i + 7]),
                                 ctypes.c_uint32(int(seeds[i])), _ptr(o12), ctypes.byref(c), ctypes.byref(u))
        out[i] = o12
        cnt[i] = c.value
        st[i] = u.value
    return out, ret, cnt, st


def lrt_scatter(s, m, ids, rays, recs, seeds, on_device):
    sph, mat = scene_from_arrays(s, m)
    n = len(ids)
    sa = (L.Sphere * len(sph))(*sph)
    ma = (L.Material * len(mat))(*mat)
    out = np.zeros((n, 12), np.float32)
    ret = np.zeros(n, np.int32)
    cnt = np.zeros(n, np.int32)
    st = np.zeros(n, np.uint32)
    L.check(L.lib().lrt_scatter_eval(sa, ma, len(sph), _ptr(ids), _ptr(rays), _ptr(recs), _ptr(seeds), n,
                                     _ptr(out), _ptr(ret), _ptr(cnt), _ptr(st), on_device))
    return out, ret, cnt, st


def scenes():
    """(name, n, spheres, mats): n selects the reference build (9: libref.so, 1000: libref1000.so)."""
    from make_golden import fuzz_scene
    yield ("default", 9, None, None)
    for k in (3, 7, 11, 20):
        s, m = fuzz_scene(k)
        yield (f"fuzz{k}", 9, s, m)
    yield ("scene1000", 1000, None, None)


def check_scene(name, n, s, m, on_device, n_cases=600):
    if not oracle.have_ref(n):
        pytest.skip(f"oracle/_ref build for n={n} missing")
    lib = oracle.ref(n)
    if s is not None:
        lib.ref_set_scene(_ptr(s), _ptr(m))
    try:
        if s is None:
            s, m = oracle.ref_scene(n)
        if n == 1000:   # the reference build's static scene is random_scene(1000, 1)
            s2, m2 = (np.array(v, np.float32) for v in scene_arrays(*random_scene(1000, 1)))
            assert np.array_equal(s, s2) and np.array_equal(m, m2)
        ids, rays, recs, seeds = make_cases(lib, s, n_cases, seed=len(name) * 7919 + n)
        want = ref_scatter(lib, ids, rays, recs, seeds)
    finally:
        if n == 9:
            lib.ref_reset_scene()
    got = lrt_scatter(s, m, ids, rays, recs, seeds, on_device)
    types = m.reshape(-1, 9)[ids, 0].astype(int)
    emissive = (m.reshape(-1, 9)[ids, 4:7] > 0).any(axis=1)
    # the cases cover what they are meant to
    assert len(ids) >= n_cases // 2
    assert (want[2] > 0).any()                    # shadow rays were counted
    assert (want[0][:, 9:] != 0).any()            # ... and some reached a light (lightE)
    if name in ("default", "scene1000"):
        assert set(types.tolist()) == {0, 1, 2}   # Lambert, Metal, Dielectric
        assert (want[1] == 0).any()               # Metal absorbed somewhere (:147)
    for k, what in enumerate(("out", "ret", "rays", "state")):
        a, b = want[k], got[k]
        bad = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).reshape(len(ids), -1).any(axis=1))[0]
        assert bad.size == 0, (f"{name}: {what} differs in {bad.size} of {len(ids)} cases, first case "
                               f"{bad[0]} (material {ids[bad[0]]}, type {types[bad[0]]}, emissive "
                               f"{emissive[bad[0]]}): ref {a[bad[0]]} vs lrt {b[bad[0]]}")


@pytest.mark.parametrize("scene", list(scenes()), ids=lambda t: t[0])
def test_scatter_host_matches_reference(scene):
    check_scene(*scene, on_device=0)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2], ids=["per_lane", "packet"])
@pytest.mark.parametrize("scene", list(scenes()), ids=lambda t: t[0])
def test_scatter_device_matches_reference(gpu, scene, mode):
    """mode 2 sends every wave's shadow rays (64 unrelated cases) through the packet
    traversal: exact whatever the rays' coherence."""
    check_scene(*scene, on_device=mode)
