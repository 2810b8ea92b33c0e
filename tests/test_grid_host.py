"""The uniform grid's closest hit (lrt_grid.h) against the reference's linear scan, on the
host (no GPU): the library builds the grid exactly as for the device and runs the device's
walk compiled for the host (lrt_grid_stats). For every ray the closest (id, t), the bounded
shadow answer (towards the scan's winner and towards another sphere) and the two-query loop
must equal HitWorld's scan (parallel.cpp:54-73, maths.cpp:51-94) bit for bit.
The rays that stress a DDA are here on purpose: axis-aligned rays, rays in a cell plane and
through cell corners, grazing rays along a flat field, rays starting on sphere surfaces and
exactly on cell boundaries, and far origins that must take the fallback scan."""
import ctypes

import numpy as np
import pytest

from learnraytracing_amd import _lib as L
from learnraytracing_amd.scene import random_scene
from test_bvh_host import adversarial_scene, random_rays


def gstats(spheres, rays):
    sa = (L.Sphere * len(spheres))(*spheres)
    rays = np.ascontiguousarray(rays, np.float32)
    out = (ctypes.c_double * 10)()
    L.check(L.lib().lrt_grid_stats(sa, len(spheres), rays.ctypes.data_as(ctypes.c_void_p), len(rays), out))
    return list(out)


@pytest.mark.parametrize("n", [17, 200, 1000, 4096])
def test_random_scene_random_rays(n):
    g = np.random.default_rng(n + 1)
    sph, _ = random_scene(n, 1)
    res = gstats(sph, random_rays(g, 4000, [-6, -0.6, -7], [6, 3, 4]))
    assert res[3] == 0.0, res
    assert res[1] < n / 4 or n < 100   # the walk tests few spheres


@pytest.mark.parametrize("n", [1, 2, 3, 5, 9, 16])
def test_small_scenes(n):
    """Scenes at or below kBvhMinSpheres get the grid too (opt-in: LRT_F_GRID /
    LRT_ACCEL=grid): the reference's own 9 spheres (configs 1-3) and tiny random scenes."""
    from learnraytracing_amd.scene import default_scene
    g = np.random.default_rng(40 + n)
    sph = default_scene()[0] if n == 9 else random_scene(max(n, 2), 1)[0][:n]
    assert len(sph) == n
    res = gstats(sph, random_rays(g, 3000, [-4, -0.6, -3], [4, 3, 3]))
    assert res[3] == 0.0, res
    if n == 9:   # the ground alone is tested first; the 8 others are walked
        assert res[8] == 1.0 and res[1] < 5, res


def test_config4_scene_gets_the_grid():
    """random_scene(1000, 1) (configs 4-5): the policy picks the grid; the ground and the
    light are tested first by every ray and the cells form one or two layers."""
    sph, _ = random_scene(1000, 1)
    res = gstats(sph, random_rays(np.random.default_rng(3), 500, [-6, -0.6, -7], [6, 3, 4]))
    assert res[9] == 1.0 and res[8] == 2.0 and res[6] <= 2, res


@pytest.mark.parametrize("seed", range(6))
def test_adversarial_scenes(seed):
    g = np.random.default_rng(200 + seed)
    sph = adversarial_scene(g, int(g.integers(20, 600)))
    assert gstats(sph, random_rays(g, 3000, -25, 25))[3] == 0.0


def _cells(sph):
    """The grid's planes as the host builds them are not exported; rays through the planes of
    a guessed lattice over the spheres' box still hit real cell planes often: the lattice is
    the build's own (same extent, per-axis counts from lrt_grid_stats)."""
    res = gstats(sph, np.array([[0, 5, 0, 0, -1, 0]], np.float32))
    c = np.array([[s.center.x, s.center.y, s.center.z] for s in sph[2:]])
    r = np.array([s.radius for s in sph[2:]])
    lo, hi = (c - r[:, None]).min(0), (c + r[:, None]).max(0)
    return lo, hi, np.array(res[5:8], int)


def test_axis_aligned_plane_and_corner_rays():
    g = np.random.default_rng(11)
    sph, _ = random_scene(1000, 1)
    lo, hi, n = _cells(sph)
    h = (hi - lo) / n
    rays = []
    for axis in range(3):
        for sgn in (1.0, -1.0):
            for _ in range(200):
                o = g.uniform(lo - 0.5, hi + 0.5)
                d = np.zeros(3)
                d[axis] = sgn
                rays.append(np.concatenate([o, d]))
    for _ in range(1500):   # origins on (approximate) cell planes and corners, any direction
        k = g.integers(0, n + 1)
        o = lo + k * h + g.choice([0.0, 1e-7, -1e-7], size=3)
        d = g.normal(size=3)
        if g.uniform() < 0.5:   # through another lattice corner
            k2 = g.integers(0, n + 1)
            d = lo + k2 * h - o + 1e-6
        rays.append(np.concatenate([o, d]))
    assert gstats(sph, np.array(rays, np.float32))[3] == 0.0


def test_grazing_and_surface_rays():
    """Bounce and shadow rays leave the ground and sphere surfaces at every angle, down to
    grazing the flat field, where the walk crosses the most cells."""
    g = np.random.default_rng(12)
    sph, _ = random_scene(1000, 1)
    rays = []
    for _ in range(2500):
        x, z = g.uniform(-5.5, 5.5), g.uniform(-6.5, 2.5)
        a = g.uniform(0, 2 * np.pi)
        el = g.choice([g.uniform(0, 0.02), g.uniform(0, 0.3), g.uniform(0, 1.5)])
        rays.append([x, -0.5, z, np.cos(a) * np.cos(el), np.sin(el), np.sin(a) * np.cos(el)])
    for _ in range(2500):
        s = sph[int(g.integers(0, len(sph)))]
        c = np.array([s.center.x, s.center.y, s.center.z])
        nrm = g.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        rays.append(np.concatenate([c + s.radius * nrm, g.normal(size=3)]))
    assert gstats(sph, np.array(rays, np.float32))[3] == 0.0


def test_far_origins_take_the_fallback_scan():
    """Origins far beyond the scene (the walk's rounding bound exceeds the padding) scan every
    sphere; nearer ones walk, and the few whose answer could lie beyond the padding's reach
    (origins away from the spheres, GridFarClear) finish with the scan. All exact."""
    g = np.random.default_rng(13)
    sph, _ = random_scene(300, 2)
    far = []
    for _ in range(300):
        d = g.normal(size=3)
        d /= np.linalg.norm(d)
        far.append(np.concatenate([-d * 1e4 + g.uniform(-1, 1, 3), d]))
    res = gstats(sph, np.array(far, np.float32))
    assert res[3] == 0.0 and res[4] > 0.5, res
    near = gstats(sph, random_rays(g, 500, -8, 8))
    assert near[3] == 0.0 and near[4] < 0.01, near


def test_non_finite_and_degenerate_scenes():
    """Spheres with inf / NaN fields go to the spheres tested first; zero-radius spheres and
    coincident spheres stay in cells. A scene of only big spheres has no walk at all."""
    g = np.random.default_rng(14)
    sph, _ = random_scene(200, 4)
    sph[5] = L.Sphere(L.f3(float("inf"), 0, 0), 0.1)
    sph[6] = L.Sphere(L.f3(0, float("nan"), 0), 0.1)
    sph[7] = L.Sphere(L.f3(1, 0, 1), 0.0)
    sph[8] = L.Sphere(L.f3(sph[9].center.x, sph[9].center.y, sph[9].center.z), sph[9].radius)
    assert gstats(sph, random_rays(g, 2000, [-6, -0.6, -7], [6, 3, 4]))[3] == 0.0
    big = [L.Sphere(L.f3(*g.uniform(-5, 5, 3)), float(r)) for r in (100, 200, 300, 0.1)]
    assert gstats(big, random_rays(g, 500, -10, 10))[3] == 0.0
