#!/usr/bin/env python3
"""BVH traversal statistics on the host (no GPU): camera rays of a W x H image through
random_scene(n) -> nodes visited / spheres tested per ray, and a bitwise check against
the linear scan. Usage: python tools/bvh_stats.py [n] [W H]"""
import ctypes
import sys

import numpy as np

sys.path[:0] = [".", "oracle"]
import oracle  # noqa: E402
import learnraytracing_amd as lrt  # noqa: E402
from learnraytracing_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (3840, 2160)
sph, _ = lrt.random_scene(n, 1)
cam = oracle.orc_camera(W, H)
g = np.random.default_rng(0)
m = 20000
rays = np.zeros((m, 6), np.float32)
O = oracle.ref() if oracle.have_ref() else None
for i in range(m):
    u, v = g.uniform(), g.uniform()
    out = np.zeros(6, np.float32)
    if O:
        O.ref_get_ray(oracle._ptr(cam), (i * 2654435761 + 1) & 0xFFFFFFFF | 1, float(u), float(v), oracle._ptr(out))
    else:   # pinhole approximation
        out[:3] = cam[:3]
        out[3:] = cam[12:15] + u * cam[15:18] + v * cam[18:21] - cam[:3]
    rays[i] = out
res = (ctypes.c_double * 7)()
sa = (L.Sphere * n)(*sph)
L.check(L.lib().lrt_bvh_stats(sa, n, rays.ctypes.data_as(ctypes.c_void_p), m, res))
print(f"n={n}: nodes/ray {res[0]:.1f} spheres/ray {res[1]:.1f} max nodes {res[2]:.0f} "
      f"max spheres {res[3]:.0f} mismatch {res[4]:.4f} stack {res[5]:.0f} of {res[6]:.0f} levels")
