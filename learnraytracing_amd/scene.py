"""Scenes for the path tracer.

`default_scene()` is the reference's 9-sphere scene (src/cpu/parallel.cpp:15-51),
read back from the library so there is one source of truth.

`random_scene(n, seed)` is the build-defined N-sphere scene of BASELINE configs 4-5
(the reference has no such scene). It is generated with the
reference's own XorShift32 / RandomFloat01 (maths.cpp:7-20) in pure Python so the
same (n, seed) gives the same spheres everywhere:
  sphere 0      the reference's ground sphere (0, -100.5, -1), r 100, Lambert 0.8
  sphere 1      the reference's emissive sphere (-1.5, 1.5, 0), r 0.3, emissive (30, 25, 15)
  spheres 2..   small spheres resting on the ground (y = r - 0.5) on a jittered grid
                covering x in [-5, 5], z in [-6, 2] (the camera's view of the ground),
                radius 0.05-0.12; 70 % Lambert, 20 % Metal (roughness 0-0.5),
                10 % Dielectric (ri 1.5). No other emissive sphere, so each Lambert
                bounce traces exactly one shadow ray, as in the default scene.
"""
from __future__ import annotations

import ctypes
import math

from . import _lib as L


def default_scene():
    """Return (spheres, materials) as lists of ctypes structs (9 entries)."""
    sph = (L.Sphere * 9)()
    mat = (L.Material * 9)()
    n = ctypes.c_int(0)
    L.check(L.lib().lrt_default_scene(sph, mat, 9, ctypes.byref(n)))
    return list(sph)[: n.value], list(mat)[: n.value]


class _XorShift32:
    """maths.cpp:7-20 with an explicit state."""

    def __init__(self, seed: int):
        self.s = (seed & 0xFFFFFFFF) | 1

    def next(self) -> int:
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 15) & 0xFFFFFFFF
        self.s = x
        return x

    def f01(self) -> float:
        # exact float32 value of (x & 0xFFFFFF) / 16777216.0f
        return (self.next() & 0xFFFFFF) / 16777216.0


def random_scene(n: int = 1000, seed: int = 1):
    if n < 2:
        raise ValueError("random_scene needs n >= 2 (ground + light)")
    rng = _XorShift32(seed)
    sph = [L.Sphere(L.f3(0, -100.5, -1), 100.0), L.Sphere(L.f3(-1.5, 1.5, 0.0), 0.3)]
    mat = [L.Material(L.LAMBERT, L.f3(0.8, 0.8, 0.8), L.f3(0, 0, 0), 0.0, 0.0),
           L.Material(L.LAMBERT, L.f3(0.8, 0.6, 0.2), L.f3(30, 25, 15), 0.0, 0.0)]
    m = n - 2
    cols = max(1, int(math.ceil(math.sqrt(m * 10.0 / 8.0))))
    rows = max(1, int(math.ceil(m / cols)))
    dx, dz = 10.0 / cols, 8.0 / rows
    for k in range(m):
        i, j = k % cols, k // cols
        r = 0.05 + 0.07 * rng.f01()
        x = -5.0 + (i + 0.5) * dx + (rng.f01() - 0.5) * max(0.0, dx - 2 * r)
        z = -6.0 + (j + 0.5) * dz + (rng.f01() - 0.5) * max(0.0, dz - 2 * r)
        sph.append(L.Sphere(L.f3(x, r - 0.5, z), r))
        c = rng.f01()
        if c < 0.7:
            mat.append(L.Material(L.LAMBERT, L.f3(rng.f01(), rng.f01(), rng.f01()), L.f3(0, 0, 0), 0.0, 0.0))
        elif c < 0.9:
            mat.append(L.Material(L.METAL, L.f3(0.5 + 0.5 * rng.f01(), 0.5 + 0.5 * rng.f01(),
                                               0.5 + 0.5 * rng.f01()), L.f3(0, 0, 0), 0.5 * rng.f01(), 0.0))
        else:
            mat.append(L.Material(L.DIELECTRIC, L.f3(1, 1, 1), L.f3(0, 0, 0), 0.0, 1.5))
    return sph, mat


def scene_arrays(spheres, materials):
    """(spheres, materials) -> flat float lists in the oracle's layout:
    4 floats per sphere (center, radius), 9 per material (type, albedo, emissive,
    roughness, ri)."""
    s, m = [], []
    for sp in spheres:
        s += [sp.center.x, sp.center.y, sp.center.z, sp.radius]
    for mt in materials:
        m += [float(mt.type), mt.albedo.x, mt.albedo.y, mt.albedo.z,
              mt.emissive.x, mt.emissive.y, mt.emissive.z, mt.roughness, mt.ri]
    return s, m


def scene_from_arrays(s, m):
    n = len(s) // 4
    sph = [L.Sphere(L.f3(s[4 * i], s[4 * i + 1], s[4 * i + 2]), s[4 * i + 3]) for i in range(n)]
    mat = [L.Material(int(m[9 * i]), L.f3(m[9 * i + 1], m[9 * i + 2], m[9 * i + 3]),
                      L.f3(m[9 * i + 4], m[9 * i + 5], m[9 * i + 6]), m[9 * i + 7], m[9 * i + 8])
           for i in range(n)]
    return sph, mat
