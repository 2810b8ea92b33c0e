#!/usr/bin/env python3
"""Diagnostic (GPU): localise a library variant's miscompare on the 1000-sphere goldens.

    LRT_LIB=build_exp/liblrt_<V>.so python tools/miscompare_probe.py [--kernel v0|pool]

1. renders the config-4 golden window (scene1000_c4_s64: the reference's own render at 64
   spp) and lists the pixels that differ;
2. re-renders each differing pixel ALONE (a 1x1 window: same seeds, same arithmetic, but
   no other pixel in its wave) -- a pixel that is right alone and wrong in its tile points
   at cross-lane state (LDS stack slots, the packet traversal's wave-uniform stack);
3. runs the BVH closest hit on the device (per lane and packet, lrt_accel_eval BVH modes 1/2)
   against the host build of the same traversal (mode 0) on 2^18 random and coherent rays.
Prints one JSON line.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import learnraytracing_amd as lrt  # noqa: E402
from learnraytracing_amd import _lib as L  # noqa: E402
from learnraytracing_amd.scene import random_scene  # noqa: E402


def render(kflags, **kw):
    job = lrt.Job(flags=kflags, **kw)
    d = job.desc()
    buf = np.zeros((d.row_count, d.x_count, 4), np.float32)
    rays = lrt.render_host(job, buf)
    return buf, rays


def main():
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "v0"
    kflags = {"v0": 2, "pool": 512}[kernel]
    with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
        fx = json.load(f)["fixtures"]["scene1000_c4_s64"]
    with np.load(os.path.join(ROOT, "tests", "golden", "images.npz"), allow_pickle=False) as z:
        want = z["scene1000_c4_s64"]
    lrt.InitializeTest()
    sph, mat = random_scene(1000, 1)
    lrt.set_scene(sph, mat)
    kw = dict(width=fx["w"], height=fx["h"], frames=fx["frames"], max_depth=fx["max_depth"])
    buf, rays = render(kflags, x0=fx["x0"], x_count=fx["xc"], y0=fx["y0"], row_count=fx["yc"], **kw)
    info = L.last_launch()
    bad = np.argwhere((buf[..., :3].view(np.uint32) != want[..., :3].view(np.uint32)).any(axis=-1))
    alone_ok = 0
    alone = []
    for ly, lx in bad[:64]:
        b1, _ = render(kflags, x0=fx["x0"] + int(lx), x_count=1, y0=fx["y0"] + int(ly), row_count=1, **kw)
        ok = np.array_equal(b1[0, 0, :3].view(np.uint32), want[ly, lx, :3].view(np.uint32))
        alone_ok += int(ok)
        alone.append([int(fx["x0"] + lx), int(fx["y0"] + ly), bool(ok)])
    # device traversal vs its host build
    sa = (L.Sphere * len(sph))(*sph)
    g = np.random.default_rng(5)
    n = 1 << 18
    o = g.uniform([-6, -0.45, -7], [6, 3, 4], (n, 3))
    d = g.normal(size=(n, 3))
    rr = np.ascontiguousarray(np.concatenate([o, d], axis=1).astype(np.float32).reshape(-1))
    res = {}
    for mode in (0, 1, 2):
        ids = np.zeros(n, np.int32)
        ts = np.zeros(n, np.float32)
        L.check(L.lib().lrt_accel_eval(sa, len(sph), rr.ctypes.data_as(ctypes.c_void_p), n, 1, mode,
                                       ids.ctypes.data_as(ctypes.c_void_p), ts.ctypes.data_as(ctypes.c_void_p)))
        res[mode] = (ids, ts)
    dev_mis = {m: int(((res[m][0] != res[0][0]) | (res[m][1].view(np.uint32) != res[0][1].view(np.uint32))).sum())
               for m in (1, 2)}
    print(json.dumps({"lib": os.environ.get("LRT_LIB", "in-tree"), "kernel": kernel, "instance": info,
                      "rays": rays, "want_rays": fx["rays"], "bad_pixels": int(len(bad)),
                      "alone_checked": len(alone), "alone_ok": alone_ok, "alone": alone[:16],
                      "bvh_eval_mismatch_vs_host": dev_mis}), flush=True)
    lrt.ShutdownTest()


if __name__ == "__main__":
    main()
