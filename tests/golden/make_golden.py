"""Generate the golden fixtures in tests/golden/ from the reference ITSELF.

Run in the build container (needs /root/reference):
    make -C oracle ref ref1000 && python tests/golden/make_golden.py

Every fixture comes from the reference's own maths.cpp / parallel.cpp compiled in place
(oracle/ref_harness.cpp). The reference's scene is a fixed static array whose size is
kSphereCount (parallel.cpp:15-27), so the 1000-sphere crops come from a second build of
the same sources in which only the two scene initialisers of a scratch copy of
parallel.cpp (in /tmp, never committed) hold random_scene(1000, 1)
(oracle/gen_ref_scene.py, `make -C oracle ref1000`).
Images are stored as float32 RGB (the reference never touches alpha).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

P = oracle._ptr


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def fuzz_scene(seed):
    """A random 9-sphere scene for Mode F: every material type, roughness 0..1, ri in
    [1.1, 2.4] (TIR), 1-3 emissive spheres, spheres that may overlap/contain the
    camera. Deterministic in `seed` (numpy PCG64)."""
    g = np.random.default_rng(seed)
    s = np.zeros(36, np.float32)
    m = np.zeros(81, np.float32)
    s[0:4] = [0, -100.5, -1, 100]
    m[0:9] = [0, .8, .8, .8, 0, 0, 0, 0, 0]
    n_emit = int(g.integers(1, 4))
    emit = set(g.choice(np.arange(1, 9), n_emit, replace=False).tolist())
    for i in range(1, 9):
        s[4 * i:4 * i + 3] = g.uniform([-2.5, -0.5, -2.5], [2.5, 2.0, 1.5])
        s[4 * i + 3] = g.uniform(0.15, 0.8)
        t = int(g.integers(0, 3))
        alb = g.uniform(0.1, 1.0, 3)
        row = [t, *alb, 0, 0, 0, 0, 0]
        if t == 1:
            row[7] = float(g.choice([0.0, g.uniform(0, 1)]))
        if t == 2:
            row[8] = g.uniform(1.1, 2.4)
        if i in emit:
            row[0] = 0
            row[4:7] = g.uniform(0.5, 30.0, 3)
        m[9 * i:9 * i + 9] = row
    return s, m


def fuzz_camera(seed, w, h):
    g = np.random.default_rng(10_000 + seed)
    frm = g.uniform([-3, 0.2, 1], [3, 3, 4]).astype(np.float32)
    at = g.uniform([-1, -0.3, -1.5], [1, 0.8, 0.5]).astype(np.float32)
    up = np.array([0, 1, 0], np.float32)
    cam = np.zeros(22, np.float32)
    vfov, ap, focus = float(g.uniform(30, 90)), float(g.uniform(0, 0.3)), float(g.uniform(1, 5))
    oracle.ref().ref_make_camera(P(frm), P(at), P(up), np.float32(vfov).item(), np.float32(w / h).item(),
                                 np.float32(ap).item(), np.float32(focus).item(), P(cam))
    return cam, dict(look_from=frm.tolist(), look_at=at.tolist(), vfov=vfov, aperture=ap, focus=focus)


def main():
    assert oracle.have_ref(), "build oracle/_ref/libref.so first (make -C oracle ref)"
    r = oracle.ref()
    import ctypes
    r.ref_make_camera.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_float] * 4 + [ctypes.c_void_p]
    manifest = {"generator": "tests/golden/make_golden.py", "source": "reference src/cpu compiled in place "
                "(clang++ -O2 -ffp-contract=off), oracle/ref_harness.cpp", "fixtures": {}}
    arrays = {}

    # ---- KATs ---------------------------------------------------------------------------
    kat = {}
    xs = (ctypes.c_uint32 * 16)()
    r.ref_xorshift(1, 16, xs)
    kat["xorshift32_from_1"] = list(xs)
    fs = np.zeros(16, np.float32)
    r.ref_random01(1, 16, P(fs))
    kat["random01_from_1"] = fs.tolist()
    for kind, name in enumerate(["unit_disk", "unit_vector", "unit_sphere"]):
        o = np.zeros(64 * 3, np.float32)
        end = r.ref_sampler(kind, 12345, 64, P(o))
        kat[name] = {"seed": 12345, "n": 64, "out": o.tolist(), "end_state": int(end)}
    # HitSphere: the reference's own commented check (main.cpp:215-226) + random cases
    g = np.random.default_rng(7)
    cases = [([0, 0, 0], [0, 0, -1], [0, 0, 0, 0.5], 0.001, 1e7)]
    for _ in range(200):
        cases.append((g.uniform(-2, 2, 3).tolist(), g.uniform(-1, 1, 3).tolist(),
                      g.uniform(-2, 2, 3).tolist() + [float(g.uniform(0.1, 1.5))], 0.001, 1e7))
    hs = []
    for o, d, sph, tmin, tmax in cases:
        out = np.zeros(7, np.float32)
        o32, d32, s32 = (np.array(v, np.float32) for v in (o, d, sph))
        hit = r.ref_hit_sphere(P(o32), P(d32), P(s32), ctypes.c_float(tmin), ctypes.c_float(tmax), P(out))
        hs.append({"o": o32.tolist(), "d": d32.tolist(), "sphere": s32.tolist(), "tmin": tmin, "tmax": tmax,
                   "hit": int(hit), "out": out.tolist() if hit else None})
    kat["hit_sphere"] = hs
    cams = {}
    for (w, h) in [(1280, 720), (320, 180), (1920, 1080), (3840, 2160), (7680, 4320), (160, 90)]:
        c = np.zeros(22, np.float32)
        r.ref_default_camera(w, h, P(c))
        cams[f"{w}x{h}"] = c.tolist()
    kat["default_camera"] = cams
    kat["schlick"] = [[c, ri, float(r.ref_schlick(c, ri))] for c, ri in
                      [(0.5, 1.5), (0.0, 1.5), (1.0, 1.5), (0.25, 2.4), (0.9, 1.1), (0.7, 1 / 1.5)]]
    # GetRay under explicit states, 1280x720 camera
    cam = np.array(cams["1280x720"], np.float32)
    gr = []
    for k in range(64):
        seed = (k * 2654435761 + 1) & 0xFFFFFFFF | 1
        u, v = float(np.float32(g.uniform())), float(np.float32(g.uniform()))
        out = np.zeros(6, np.float32)
        end = r.ref_get_ray(P(cam), seed, u, v, P(out))
        gr.append({"seed": seed, "u": u, "v": v, "out": out.tolist(), "end_state": int(end)})
    kat["get_ray"] = gr
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f)
    manifest["fixtures"]["kat.json"] = {"what": "XorShift32/RandomFloat01/samplers/HitSphere/camera/schlick/GetRay"}

    # ---- Mode R: config 1 (the reference as written, single thread) ---------------------
    w, h = 320, 180
    buf = np.zeros((h, w, 4), np.float32)
    rays = r.ref_render_mode_r(w, h, 0, 1, 1, P(buf))
    arrays["mode_r_320x180"] = buf[..., :3].copy()
    manifest["fixtures"]["mode_r_320x180"] = {"mode": "R", "w": w, "h": h, "frames": 1, "max_depth": 20,
                                              "rays": int(rays), "md5_rgba": md5(buf),
                                              "sum_rgba": float(buf.astype(np.float64).sum())}

    # ---- Mode P ---------------------------------------------------------------------------
    def mode_p(name, w, h, frames, depth, x0=0, xc=None, y0=0, yc=None, frame0=0):
        buf, rays = oracle.ref_render_p(w, h, frames, depth, frame0, x0, xc, y0, yc, procs=8)
        arrays[name] = buf[..., :3].copy()
        manifest["fixtures"][name] = {"mode": "P", "w": w, "h": h, "x0": x0, "xc": buf.shape[1], "y0": y0,
                                      "yc": buf.shape[0], "frame0": frame0, "frames": frames,
                                      "max_depth": depth, "rays": int(rays), "md5_rgba": md5(buf)}

    mode_p("p_160x90_s4_d8", 160, 90, 4, 8)
    mode_p("p_320x180_s4_d8", 320, 180, 4, 8)
    mode_p("p_96x54_s1_d50", 96, 54, 1, 50)
    mode_p("p_128x72_s2_d20", 128, 72, 2, 20)          # DrawTest depth (kMaxDepth 20)
    mode_p("p_128x72_f5_s3_d8", 128, 72, 3, 8, frame0=5)  # progressive resume from frame 5
    mode_p("c2_crop", 1280, 720, 4, 8, x0=600, xc=64, y0=300, yc=32)     # config 2 window
    mode_p("c3_crop", 1920, 1080, 16, 50, x0=900, xc=48, y0=500, yc=24)  # config 3 window
    mode_p("c5_crop", 7680, 4320, 2, 8, x0=3800, xc=32, y0=2100, yc=16)  # config 5 geometry

    # ---- Mode F: fuzzed 9-sphere scenes and cameras --------------------------------------
    fuzz = []
    for k in range(20):
        s, m = fuzz_scene(k)
        w, h = 64, 36
        cam, camdesc = fuzz_camera(k, w, h)
        depth = [8, 20, 50][k % 3]
        buf, rays = oracle.ref_render_p(w, h, 2, depth, 0, scene=(s, m), cam22=cam, procs=4)
        arrays[f"f{k:02d}"] = buf[..., :3].copy()
        fuzz.append({"name": f"f{k:02d}", "spheres": s.tolist(), "mats": m.tolist(), "camera": cam.tolist(),
                     "camera_params": camdesc, "w": w, "h": h, "frames": 2, "max_depth": depth,
                     "rays": int(rays), "md5_rgba": md5(buf)})
    manifest["fuzz"] = fuzz

    # ---- 1000-sphere crops: the reference itself with random_scene(1000, 1) as its static
    # scene (oracle/_ref/libref1000.so, `make -C oracle ref1000`; see module docstring).
    # Small frame counts plus the real spp of configs 4 (64) and 5 (256) on small windows.
    from learnraytracing_amd.scene import random_scene, scene_arrays
    assert oracle.have_ref(1000), "build oracle/_ref/libref1000.so first (make -C oracle ref1000)"
    s, m = (np.array(v, np.float32) for v in scene_arrays(*random_scene(1000, 1)))
    rs, rm = oracle.ref_scene(1000)
    assert np.array_equal(rs.view(np.uint32), s.view(np.uint32)) and np.array_equal(rm.view(np.uint32), m.view(np.uint32))
    for name, (w, h, x0, xc, y0, yc, frames, depth) in {
            "scene1000_c4_crop": (3840, 2160, 1900, 32, 1000, 16, 2, 8),
            "scene1000_c5_crop": (7680, 4320, 3600, 32, 1900, 16, 1, 8),
            "scene1000_c4_s64": (3840, 2160, 1700, 24, 1180, 12, 64, 8),
            "scene1000_c5_s256": (7680, 4320, 3500, 12, 2300, 8, 256, 8)}.items():
        buf, rays = oracle.ref_render_p(w, h, frames, depth, 0, x0, xc, y0, yc, procs=8, n=1000)
        arrays[name] = buf[..., :3].copy()
        manifest["fixtures"][name] = {"mode": "P", "scene": "random_scene(1000, seed=1)", "w": w, "h": h,
                                      "x0": x0, "xc": xc, "y0": y0, "yc": yc, "frame0": 0, "frames": frames,
                                      "max_depth": depth, "rays": int(rays), "md5_rgba": md5(buf),
                                      "source": "reference src/cpu compiled in place with its static scene "
                                                "replaced by random_scene(1000, 1) (oracle/_ref/libref1000.so)"}

    # ---- libm: digests of glibc's sinf/cosf over the path's whole input domain ----------
    k = np.arange(1 << 24, dtype=np.uint32)
    phi = (np.float32(2.0) * np.float32(3.1415926)) * (k.astype(np.float32) * np.float32(1.0 / 16777216.0))
    phi = phi.astype(np.float32)
    pw = np.linspace(0, 1, 1 << 20, dtype=np.float32)
    sr = np.linspace(0, 64, 1 << 20, dtype=np.float32)
    manifest["libm"] = {
        "glibc": "2.35 (x86-64 FMA ifunc variants)",
        "domain": "phi = (2*kPI) * (k * 2^-24), k in [0, 2^24)",
        "sinf_sha256": hashlib.sha256(oracle.orc_libm(0, phi).tobytes()).hexdigest(),
        "cosf_sha256": hashlib.sha256(oracle.orc_libm(1, phi).tobytes()).hexdigest(),
        "powf5_linspace01_2p20_sha256": hashlib.sha256(oracle.orc_libm(2, pw).tobytes()).hexdigest(),
        "powf_srgb_linspace064_2p20_sha256": hashlib.sha256(oracle.orc_libm(3, sr).tobytes()).hexdigest(),
    }

    np.savez_compressed(os.path.join(HERE, "images.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(arrays), "images;", sum(a.nbytes for a in arrays.values()) / 1e6, "MB raw")


if __name__ == "__main__":
    main()
