#!/usr/bin/env python3
"""Host-only cost model of the two acceleration structures (no GPU): config 4's ray mix
through random_scene(n) -- camera rays, bounce rays from their first hits (normal + a random
unit vector, Lambert's direction), shadow rays from those hits towards the light -- traced
by the BVH (lrt_bvh_stats: node visits, sphere tests) and the grid (lrt_grid_stats: cells,
sphere tests), each checked bit for bit against the linear scan.
Usage: python tools/accel_stats.py [n] [rays]"""
import ctypes
import sys

import numpy as np

sys.path[:0] = [".", "oracle"]
import learnraytracing_amd as lrt  # noqa: E402
from learnraytracing_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
W, H = 3840, 2160
sph, _ = lrt.random_scene(n, 1)
sa = (L.Sphere * n)(*sph)
C = np.array([[s.center.x, s.center.y, s.center.z] for s in sph], np.float32)
g = np.random.default_rng(0)
# camera (parallel.cpp:299-307, pinhole)
eye = np.array([0, 2, 3], np.float32)
w = eye / np.linalg.norm(eye)
u = np.cross([0, 1, 0], w)
u /= np.linalg.norm(u)
v = np.cross(w, u)
hh = np.tan(np.radians(30))
hw = W / H * hh
px, py = g.uniform(size=m), g.uniform(size=m)
dirs = (-w[None] + ((2 * px - 1) * hw)[:, None] * u[None] + ((2 * py - 1) * hh)[:, None] * v[None]).astype(np.float32)
dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
cam = np.concatenate([np.repeat(eye[None], m, 0), dirs], 1).astype(np.float32)
ids = np.zeros(m, np.int32)
ts = np.zeros(m, np.float32)
L.check(L.lib().lrt_accel_eval(sa, n, cam.ctypes.data_as(ctypes.c_void_p), m, 1, 0,
                               ids.ctypes.data_as(ctypes.c_void_p), ts.ctypes.data_as(ctypes.c_void_p)))
hit = ids >= 0
P = cam[hit, :3] + cam[hit, 3:] * ts[hit, None]
N = P - C[ids[hit]]
N /= np.linalg.norm(N, axis=1, keepdims=True)
z = g.uniform(-1, 1, len(P))
a = g.uniform(0, 2 * np.pi, len(P))
r = np.sqrt(1 - z * z)
rv = np.stack([r * np.cos(a), r * np.sin(a), z], 1)
bounce = np.concatenate([P, N + rv], 1).astype(np.float32)
light = C[1] + g.normal(scale=0.1, size=(len(P), 3))
shadow = np.concatenate([P, light - P], 1).astype(np.float32)


def run(name, rays):
    rays = np.ascontiguousarray(rays, np.float32)
    b = (ctypes.c_double * 7)()
    L.check(L.lib().lrt_bvh_stats(sa, n, rays.ctypes.data_as(ctypes.c_void_p), len(rays), b))
    q = (ctypes.c_double * 10)()
    L.check(L.lib().lrt_grid_stats(sa, n, rays.ctypes.data_as(ctypes.c_void_p), len(rays), q))
    print(f"{name:7s} BVH: nodes {b[0]:5.2f} spheres {b[1]:5.2f} (mismatch {b[4]:.4f}) | grid: cells {q[0]:5.2f} "
          f"spheres {q[1]:5.2f} max {q[2]:4.0f} (mismatch {q[3]:.4f}, fallback {q[4]:.4f}) "
          f"grid {q[5]:.0f}x{q[6]:.0f}x{q[7]:.0f} big {q[8]:.0f} pick {q[9]:.0f}")


run("camera", cam)
run("bounce", bounce)
run("shadow", shadow)
