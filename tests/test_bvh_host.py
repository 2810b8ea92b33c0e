"""The BVH closest hit against the reference's linear scan, on the host (no GPU): the
library builds the BVH exactly as for the device and runs the device traversal code
(lrt_bvh_stats), comparing (id, t) with the HitWorld scan bit for bit for every ray."""
import ctypes

import numpy as np
import pytest

from learnraytracing_amd import _lib as L
from learnraytracing_amd.scene import random_scene


def stats(spheres, rays):
    sa = (L.Sphere * len(spheres))(*spheres)
    rays = np.ascontiguousarray(rays, np.float32)
    out = (ctypes.c_double * 7)()
    L.check(L.lib().lrt_bvh_stats(sa, len(spheres), rays.ctypes.data_as(ctypes.c_void_p), len(rays), out))
    # the LDS stack guard: no traversal (closest hit, shadow, two-query) writes an entry beyond
    # the levels the device stack is sized to for this scene
    assert 0 <= out[5] <= out[6] <= 24, list(out)
    return list(out)


def random_rays(g, m, lo, hi):
    o = g.uniform(lo, hi, (m, 3))
    d = g.normal(size=(m, 3))
    return np.concatenate([o, d], axis=1).astype(np.float32)


def adversarial_scene(g, n):
    """Overlapping spheres of widely varying radii (incl. a few huge ones and some
    coincident centres) scattered in a box -- not the generator's tidy layout."""
    sph = []
    for i in range(n):
        c = g.uniform(-20, 20, 3)
        r = float(g.choice([g.uniform(0.01, 0.5), g.uniform(0.5, 5.0), g.uniform(50, 200)], p=[0.8, 0.18, 0.02]))
        if i % 37 == 0 and sph:
            c = np.array([sph[-1].center.x, sph[-1].center.y, sph[-1].center.z])   # coincident centres
        sph.append(L.Sphere(L.f3(*c), r))
    return sph


@pytest.mark.parametrize("n", [17, 200, 1000, 4096])
def test_random_scene_random_rays(n):
    g = np.random.default_rng(n)
    sph, _ = random_scene(n, 1)
    rays = random_rays(g, 4000, [-6, -0.6, -7], [6, 3, 4])
    res = stats(sph, rays)
    assert res[4] == 0.0
    assert res[1] < n / 4 or n < 100      # the BVH actually culls


@pytest.mark.parametrize("seed", range(6))
def test_adversarial_scenes(seed):
    g = np.random.default_rng(100 + seed)
    sph = adversarial_scene(g, int(g.integers(20, 600)))
    rays = random_rays(g, 3000, -25, 25)
    assert stats(sph, rays)[4] == 0.0


def test_axis_aligned_and_surface_rays():
    g = np.random.default_rng(7)
    sph, _ = random_scene(500, 3)
    rays = []
    for axis in range(3):
        for sgn in (1.0, -1.0):
            for _ in range(300):
                o = g.uniform([-6, -0.6, -7], [6, 2, 3])
                d = np.zeros(3)
                d[axis] = sgn
                rays.append(np.concatenate([o, d]))
    # rays leaving sphere surfaces (as bounce and shadow rays do), incl. towards the inside
    for _ in range(2000):
        s = sph[int(g.integers(0, len(sph)))]
        c = np.array([s.center.x, s.center.y, s.center.z])
        nrm = g.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        rays.append(np.concatenate([c + s.radius * nrm, g.normal(size=3)]))
    assert stats(sph, np.array(rays, np.float32))[4] == 0.0


@pytest.mark.parametrize("n,leaf", [(4096, 1), (4096, 16), (1000, 2)])
def test_stack_depth_bound_deepest_trees(monkeypatch, n, leaf):
    """The deepest trees the builder makes (leaf size 1: 4096 leaves; a colinear chain of
    spheres whose median splits recurse to the depth cap): every traversal's stack stays
    within the LDS allocation (parallel.cpp:54-73's HitWorld answer unchanged)."""
    monkeypatch.setenv("LRT_BVH_LEAF", str(leaf))
    g = np.random.default_rng(n + leaf)
    sph, _ = random_scene(n, 1)
    res = stats(sph, random_rays(g, 3000, [-6, -0.6, -7], [6, 3, 4]))
    assert res[4] == 0.0 and res[5] >= 1
    chain = [L.Sphere(L.f3(0.01 * i, 0.0, 0.0), 0.004) for i in range(n)]   # colinear, tiny
    o = np.zeros((3000, 3))
    o[:, 0] = g.uniform(-1, 0.01 * n + 1, 3000)
    o[:, 1] = g.uniform(-0.01, 0.01, 3000)
    o[:, 2] = -1.0
    d = np.tile([0.0, 0.0, 1.0], (3000, 1)) + g.normal(0, 0.002, (3000, 3))
    rays = np.concatenate([o, d], axis=1).astype(np.float32)
    rays2 = np.concatenate([np.array([[-1.0, 0.0, 0.0]] * 100), np.tile([1.0, 0.0, 0.0], (100, 1))], axis=1)
    res = stats(chain, np.concatenate([rays, rays2.astype(np.float32)]))
    assert res[4] == 0.0


@pytest.mark.parametrize("bad", [1, 40])
def test_non_finite_spheres(bad):
    """Spheres with NaN / inf centres or radii stay out of the tree and are tested by every
    ray (the build never orders them), so the result still equals the linear scan."""
    g = np.random.default_rng(bad)
    sph, _ = random_scene(300, 2)
    vals = [float("nan"), float("inf"), -float("inf")]
    for k, i in enumerate(g.choice(np.arange(1, 300), bad, replace=False)):
        s = sph[int(i)]
        if k % 2:
            s.radius = vals[k % 3]
        else:
            s.center = L.f3(vals[k % 3], s.center.y, s.center.z)
    rays = random_rays(g, 3000, [-6, -0.6, -7], [6, 3, 4])
    assert stats(sph, rays)[4] == 0.0
