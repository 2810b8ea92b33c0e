"""The accelerated closest hits (BVH, uniform grid) against the reference's own HitWorld on the
rays that stress them most: near-tangent rays from far origins (round-4 verdict, What's weak 1).

HitSphere (maths.cpp:51-94) forms ifHit = dot(rs,rs) - rsProj^2 - r^2 by cancellation, so for a
ray that grazes a sphere from far away its computed "hit" point can lie well off the sphere --
~ulp(|c - o|^2) / r, or ~sqrt(ulp(|c - o|^2)) for tiny spheres. A structure that culls by the
sphere's box must pad the box by that much (hit_excursion, lrt_grid_build.h).
Here every ray aims at a chosen sphere at the tangent angle asin(r / dist) +- 5 % from 10-400
units away, and (id, t) must equal the reference's scan bit for bit:
  * the reference: its own HitSphere looped over the array (oracle/ref_harness.cpp
    ref_hit_spheres, HitWorld's loop, parallel.cpp:54-73) and, for random_scene(1000, 1), its
    own HitWorld over that static scene (libref1000.so);
  * ours: lrt_accel_eval (the device traversal code compiled for the host here; the device
    itself in the -m gpu cases).
The bound itself is checked by brute force too (numpy float32 = the reference's arithmetic).
"""
import ctypes

import numpy as np
import pytest

import oracle
from learnraytracing_amd import _lib as L
from learnraytracing_amd.scene import random_scene

_P = ctypes.c_void_p


def _ptr(a):
    return a.ctypes.data_as(_P)


def sphere_array(sph):
    return np.array([[s.center.x, s.center.y, s.center.z, s.radius] for s in sph], np.float32)


def box50_scene(seed=5, n=300):
    """300 spheres of radius 0.001-0.2 in a 50-unit box (the verdict's grid probe)."""
    g = np.random.default_rng(seed)
    c = g.uniform(-25, 25, (n, 3))
    r = np.exp(g.uniform(np.log(0.001), np.log(0.2), n))
    return [L.Sphere(L.f3(*map(float, c[i])), float(r[i])) for i in range(n)]


def tangent_rays(arr, n, seed, dmin=10.0, dmax=400.0, targets=None):
    """n rays, each at the tangent angle (+-5 %) of a target sphere from dist in [dmin, dmax]."""
    g = np.random.default_rng(seed)
    tid = g.choice(targets if targets is not None else np.arange(len(arr)), n)
    c = arr[tid, :3].astype(np.float64)
    r = np.abs(arr[tid, 3]).astype(np.float64)
    dist = np.exp(g.uniform(np.log(dmin), np.log(dmax), n))
    u = g.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = c + u * dist[:, None]
    w = g.normal(size=(n, 3))
    w -= (w * u).sum(1, keepdims=True) * u
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    th = np.arcsin(np.minimum(1.0, r / dist)) * g.uniform(0.95, 1.05, n)
    d = -u * np.cos(th)[:, None] + w * np.sin(th)[:, None]
    return np.concatenate([o, d], axis=1).astype(np.float32)


def accel(sph, rays, acc, mode=0):
    sa = (L.Sphere * len(sph))(*sph)
    r = np.ascontiguousarray(rays, np.float32)
    ids = np.zeros(len(r), np.int32)
    ts = np.zeros(len(r), np.float32)
    L.check(L.lib().lrt_accel_eval(sa, len(sph), _ptr(r), len(r), acc, mode, _ptr(ids), _ptr(ts)))
    return ids, ts


def assert_same(got, want, what):
    gi, gt = got
    wi, wt = want
    hit = wi >= 0
    bad = (gi != wi) | (hit & (gt.view(np.uint32) != wt.view(np.uint32)))
    assert not bad.any(), f"{what}: {int(bad.sum())} of {len(bad)} rays differ from the reference " \
                          f"(first: ray {int(np.argmax(bad))}, id {int(gi[bad][0])} vs {int(wi[bad][0])})"


def _need_ref(n=9):
    if not oracle.have_ref(n):
        pytest.skip(f"the reference build (oracle/_ref, n={n}) is not present")


SCENES = {
    "random1000": lambda: random_scene(1000, 1)[0],
    "box50": box50_scene,
}


@pytest.mark.parametrize("acc", [1, 2], ids=["bvh", "grid"])
@pytest.mark.parametrize("scene", sorted(SCENES))
def test_tangent_far_rays_vs_reference_scan(scene, acc):
    _need_ref()
    sph = SCENES[scene]()
    arr = sphere_array(sph)
    targets = np.arange(2, len(arr)) if scene == "random1000" else None   # the field, not the ground
    rays = np.concatenate([tangent_rays(arr, 6000, 1, 10, 60, targets), tangent_rays(arr, 6000, 2, 60, 400, targets)])
    want = oracle.ref_hit_spheres(rays, arr)
    assert (want[0] >= 0).mean() > 0.2   # the rays do graze their targets
    assert_same(accel(sph, rays, acc), want, f"{scene} / {'bvh' if acc == 1 else 'grid'}")


def test_tangent_far_rays_vs_reference_hitworld_1000():
    """The same against the reference's own HitWorld with random_scene(1000, 1) as its static
    scene (libref1000.so), both structures."""
    _need_ref(1000)
    sph = random_scene(1000, 1)[0]
    arr = sphere_array(sph)
    rays = tangent_rays(arr, 3000, 3, 10, 400, np.arange(2, len(arr)))
    lib = oracle.ref(1000)
    out = np.zeros(7, np.float32)
    wi = np.zeros(len(rays), np.int32)
    wt = np.zeros(len(rays), np.float32)
    for i, r in enumerate(rays):
        o, d = r[:3].copy(), r[3:].copy()
        wi[i] = lib.ref_hit_world(_ptr(o), _ptr(d), ctypes.c_float(0.001), ctypes.c_float(1e7), _ptr(out))
        wt[i] = out[6] if wi[i] >= 0 else 0.0
    for acc in (1, 2):
        assert_same(accel(sph, rays, acc), (wi, wt), f"hitworld1000 / {acc}")


def config4_rays(n, seed):
    """Config 4's ray mix on random_scene(1000, 1): pinhole camera rays of the 3840x2160 view
    (parallel.cpp:299-307), bounce rays from their first hits (Lambert: normal + a random unit
    vector) -- the field and the ground out to the horizon, ~35 units -- and shadow rays from
    those hits towards the light."""
    sph = random_scene(1000, 1)[0]
    arr = sphere_array(sph)
    g = np.random.default_rng(seed)
    eye = np.array([0, 2, 3], np.float64)
    w = eye / np.linalg.norm(eye)
    u = np.cross([0, 1, 0], w)
    u /= np.linalg.norm(u)
    v = np.cross(w, u)
    hh = np.tan(np.radians(30))
    px, py = g.uniform(size=n), g.uniform(size=n)
    d = -w[None] + ((2 * px - 1) * 3840 / 2160 * hh)[:, None] * u[None] + ((2 * py - 1) * hh)[:, None] * v[None]
    cam = np.concatenate([np.repeat(eye[None], n, 0), d], 1).astype(np.float32)
    ids, ts = oracle.ref_hit_spheres(cam, arr)
    hit = ids >= 0
    dn = cam[hit, 3:] / np.linalg.norm(cam[hit, 3:], axis=1, keepdims=True)
    P = cam[hit, :3] + dn * ts[hit, None]
    N = P - arr[ids[hit], :3]
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    rv = g.normal(size=(len(P), 3))
    rv /= np.linalg.norm(rv, axis=1, keepdims=True)
    bounce = np.concatenate([P, N + rv], 1)
    shadow = np.concatenate([P, arr[1, :3] + g.normal(scale=0.1, size=(len(P), 3)) - P], 1)
    return sph, np.concatenate([cam, bounce, shadow]).astype(np.float32)


def test_grid_config4_rays_walk_exactly():
    """Config 4's own rays (origins up to ~35 units out) are exact and none of them needs the
    scan: the pad covers candidates up to tsafe (1.6 scene radii) from any origin, the near
    test (farthest corner of the centre box) holds for the camera and the field, and the cone
    test (GridFarT) clears the ground points beyond whose rays leave the field."""
    _need_ref()
    sph, rays = config4_rays(6000, 9)
    sa = (L.Sphere * len(sph))(*sph)
    out = (ctypes.c_double * 10)()
    L.check(L.lib().lrt_grid_stats(sa, len(sph), _ptr(rays), len(rays), out))
    assert out[3] == 0.0, list(out)
    assert out[4] < 2e-4, list(out)   # fraction of rays that scanned
    assert_same(accel(sph, rays, 2), oracle.ref_hit_spheres(rays, sphere_array(sph)), "config4 rays / grid")
    assert_same(accel(sph, rays, 1), oracle.ref_hit_spheres(rays, sphere_array(sph)), "config4 rays / bvh")


def hit_excursion(D, r):   # lrt_grid_build.h
    E = np.ldexp(D * D, -19)
    return E / (np.sqrt(r * r + E) + r) + np.ldexp(24.0 * D, -24)


@pytest.mark.parametrize("seed", range(3))
def test_hit_excursion_bounds_the_reference_arithmetic(seed):
    """Brute force of the bound the padding rests on: HitSphere's arithmetic in float32 (numpy
    rounds every operation; no FMA) on near-tangent rays, spheres of r 1e-3..1 at 1..500 units;
    the computed hit point lies within r + hit_excursion(|c - o| + r, r) of the center."""
    g = np.random.default_rng(100 + seed)
    f = np.float32
    worst = 0.0
    for _ in range(40):
        n = 50000
        r = f(np.exp(g.uniform(np.log(1e-3), 0.0)))
        c = g.uniform(-30, 30, 3).astype(f)
        dist = np.exp(g.uniform(0.0, np.log(500.0)))
        u = g.normal(size=(n, 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        o = (c[None].astype(np.float64) + u * dist).astype(f)
        w = g.normal(size=(n, 3))
        w -= (w * u).sum(1, keepdims=True) * u
        w /= np.linalg.norm(w, axis=1, keepdims=True)
        off = float(r) * g.uniform(0.9, 1.1, n) * (1 + g.normal(size=n) * np.sqrt(50 * 2.0 ** -24) * dist / float(r))
        v = (c[None] + w * off[:, None] - o).astype(f)
        s = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]   # normalize(): v * (1 / |v|)
        d = v * (f(1) / np.sqrt(s))[:, None]
        rs = (c[None] - o).astype(f)
        P = (rs[:, 0] * d[:, 0] + rs[:, 1] * d[:, 1]) + rs[:, 2] * d[:, 2]
        S = (rs[:, 0] * rs[:, 0] + rs[:, 1] * rs[:, 1]) + rs[:, 2] * rs[:, 2]
        H = (S - P * P) - r * r
        hit = H < 0
        h = np.sqrt(-np.where(hit, H, f(0)))
        t1, t2 = P - h, P + h
        cand = np.where(t1 > f(0.001), t1, np.where(t2 > f(0.001), t2, f(np.inf)))
        ok = hit & np.isfinite(cand)
        if not ok.any():
            continue
        X = o[ok].astype(np.float64) + cand[ok, None].astype(np.float64) * d[ok].astype(np.float64)
        dev = np.linalg.norm(X - c.astype(np.float64), axis=1) - float(r)
        D = np.linalg.norm((c[None].astype(np.float64) - o[ok]), axis=1) + float(r)
        worst = max(worst, float((dev / hit_excursion(D, float(r))).max()))
    assert 0.05 < worst < 1.0, worst


@pytest.mark.gpu
@pytest.mark.parametrize("acc,mode", [(1, 1), (1, 2), (2, 1)], ids=["bvh-lane", "bvh-packet", "grid"])
@pytest.mark.parametrize("scene", sorted(SCENES))
def test_tangent_far_rays_device_vs_reference(gpu, scene, acc, mode):
    _need_ref()
    sph = SCENES[scene]()
    arr = sphere_array(sph)
    targets = np.arange(2, len(arr)) if scene == "random1000" else None
    rays = np.concatenate([tangent_rays(arr, 4096, 5, 10, 60, targets), tangent_rays(arr, 4096, 6, 60, 400, targets)])
    assert_same(accel(sph, rays, acc, mode), oracle.ref_hit_spheres(rays, arr), f"{scene} device {acc}/{mode}")
