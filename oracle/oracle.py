"""TEST INFRASTRUCTURE ONLY — Python front end of the CPU checkers.

    orc  : liblrt_oracle.so — the plain-C restatement (lrt_oracle.c), any scene size,
           thread-safe, built anywhere with gcc (`make -C oracle`).
    ref  : _ref/libref.so   — the reference's OWN maths.cpp/parallel.cpp compiled in
           place (ref_harness.cpp); present only where /root/reference was available
           at build time (travels to the GPU box as a built file). Optional.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORC_PATH = os.path.join(HERE, "liblrt_oracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref.so")
# the reference compiled with random_scene(1000, 1) as its static scene (make ref1000)
REF1000_PATH = os.path.join(HERE, "_ref", "libref1000.so")

_P = ctypes.c_void_p
_ll = ctypes.c_longlong


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_P)


def build_orc() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "liblrt_oracle.so"], check=True)


_orc = None


def orc():
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_PATH):
            build_orc()
        lib = ctypes.CDLL(ORC_PATH)
        lib.orc_render_p.restype = _ll
        lib.orc_render_p.argtypes = [_P, _P, ctypes.c_int, _P] + [ctypes.c_int] * 9 + [_P, ctypes.c_int]
        lib.orc_render_p_ex.restype = _ll
        lib.orc_render_p_ex.argtypes = ([_P, _P, ctypes.c_int, _P] + [ctypes.c_int] * 10 +
                                        [_P, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int])
        lib.orc_render_r.restype = _ll
        lib.orc_render_r.argtypes = [_P, _P] + [ctypes.c_int] * 6 + [ctypes.POINTER(ctypes.c_uint32), _P]
        lib.orc_libm_eval.restype = None
        lib.orc_libm_eval.argtypes = [ctypes.c_int, _P, _P, _ll]
        lib.orc_xorshift32.restype = ctypes.c_uint32
        lib.orc_random01.restype = ctypes.c_float
        lib.orc_default_camera.argtypes = [ctypes.c_int, ctypes.c_int, _P]
        lib.orc_make_camera.argtypes = [_P, _P, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, _P]
        lib.orc_hit_sphere.argtypes = [_P, _P, _P, ctypes.c_float, ctypes.c_float, _P]
        _orc = lib
    return _orc


def have_ref(n: int = 9) -> bool:
    return os.path.exists(REF_PATH if n == 9 else REF1000_PATH)


_refs = {}


def ref(n: int = 9):
    """The reference's own sources compiled in place: n = 9 its default scene (libref.so),
    n = 1000 its static scene replaced by random_scene(1000, 1) (libref1000.so)."""
    if n not in _refs:
        lib = ctypes.CDLL(REF_PATH if n == 9 else REF1000_PATH)
        for f in ("ref_render_mode_r", "ref_render_mode_p", "ref_render_mode_p_procs"):
            getattr(lib, f).restype = _ll
        lib.ref_render_mode_r.argtypes = [ctypes.c_int] * 5 + [_P]
        lib.ref_render_mode_p.argtypes = [ctypes.c_int] * 9 + [_P, _P]
        lib.ref_render_mode_p_procs.argtypes = [ctypes.c_int] * 9 + [_P, _P, ctypes.c_int]
        lib.ref_sampler.restype = ctypes.c_uint32
        lib.ref_get_ray.restype = ctypes.c_uint32
        lib.ref_get_ray.argtypes = [_P, ctypes.c_uint32, ctypes.c_float, ctypes.c_float, _P]
        lib.ref_schlick.restype = ctypes.c_float
        lib.ref_schlick.argtypes = [ctypes.c_float, ctypes.c_float]
        lib.ref_hit_sphere.argtypes = [_P, _P, _P, ctypes.c_float, ctypes.c_float, _P]
        lib.ref_hit_world.argtypes = [_P, _P, ctypes.c_float, ctypes.c_float, _P]
        lib.ref_trace.argtypes = [_P, _P, ctypes.c_int, ctypes.c_uint32, _P]
        lib.ref_scatter.argtypes = [ctypes.c_int, _P, _P, ctypes.c_uint32, _P, _P, _P]
        lib.ref_draw_test.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]
        lib.ref_initialize_threads.argtypes = [ctypes.c_int]
        if hasattr(lib, "ref_hit_spheres_batch"):
            lib.ref_hit_spheres_batch.argtypes = [_P, ctypes.c_int, _P, ctypes.c_int, _P, _P]
            lib.ref_hit_spheres_batch.restype = None
        _refs[n] = lib
    return _refs[n]


def ref_hit_spheres(rays, spheres):
    """HitWorld's loop over an arbitrary sphere array with the reference's own HitSphere
    (ref_harness.cpp ref_hit_spheres; parallel.cpp:54-73, maths.cpp:51-94). rays: (n, 6)
    o.xyz, d.xyz (through the Ray ctor); spheres: (m, 4) center.xyz, radius.
    Returns (ids int32, ts float32; t = 0 where nothing is hit)."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    spheres = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    ids = np.zeros(len(rays), np.int32)
    ts = np.zeros(len(rays), np.float32)
    ref(9).ref_hit_spheres_batch(_ptr(rays), len(rays), _ptr(spheres), len(spheres), _ptr(ids), _ptr(ts))
    return ids, ts


def ref_drawtest_rate(width, height, budget_s, threads):
    """The reference's own DrawTest as main.cpp:165 calls it -- enkiTS over `threads` workers,
    kMaxDepth 20, the shared racy RNG (parallel.cpp:297-323, maths.cpp:5) -- on successive
    frames of one buffer for about budget_s. Returns (Mray/s, frames, rays, seconds).
    The reference's default scene (libref.so) only; output is non-deterministic by design."""
    r = ref(9)
    buf = np.zeros(width * height * 4, np.float32)
    r.ref_initialize_threads(threads)
    try:
        rays = frames = 0
        t0 = time.perf_counter()
        while True:
            rays += r.ref_draw_test(0.0, frames, width, height, _ptr(buf))
            frames += 1
            dt = time.perf_counter() - t0
            if dt >= budget_s:
                break
    finally:
        r.ref_shutdown()
    return rays / dt / 1e6, frames, rays, dt


def ref_scene(n: int = 9):
    """The static scene a reference build holds, in the oracle layout (spheres, mats)."""
    r = ref(n)
    cnt = r.ref_scene_count()
    s = np.zeros(4 * cnt, np.float32)
    m = np.zeros(9 * cnt, np.float32)
    r.ref_get_scene(_ptr(s), _ptr(m))
    return s, m


# ---- convenience wrappers ---------------------------------------------------------------
def default_scene_arrays():
    """The reference scene in the oracle layout, from the reference itself if built,
    else from the restatement's constants (parallel.cpp:15-51)."""
    s = np.array([0, -100.5, -1, 100, 2, 1, -1, .5, 0, 0, -1, .5, -2, 0, -1, .5, 2, 0, 1, .5,
                  0, 0, 1, .5, -2, 0, 1, .5, .5, 1, .5, .5, -1.5, 1.5, 0, .3], np.float32)
    m = np.array([0, .8, .8, .8, 0, 0, 0, 0, 0,
                  0, .8, .4, .4, 0, 0, 0, 0, 0,
                  0, .4, .8, .4, 0, 0, 0, 0, 0,
                  1, .4, .4, .8, 0, 0, 0, 0, 0,
                  1, .4, .8, .4, 0, 0, 0, 0, 0,
                  1, .4, .8, .4, 0, 0, 0, .2, 0,
                  1, .4, .8, .4, 0, 0, 0, .6, 0,
                  2, .4, .4, .4, 0, 0, 0, 0, 1.5,
                  0, .8, .6, .2, 30, 25, 15, 0, 0], np.float32)
    return s, m


def default_threads() -> int:
    """Worker threads for the restatement: the host share a GPU box gives one GPU (its
    OMP_NUM_THREADS, 16 there), not every CPU of the machine; all CPUs here."""
    n = int(os.environ.get("OMP_NUM_THREADS") or 0)
    return max(1, min(n, os.cpu_count() or 1)) if n > 0 else min(16, os.cpu_count() or 1)


def orc_render(width, height, frames=1, depth=8, frame0=0, x0=0, xc=None, y0=0, yc=None,
               spheres=None, mats=None, cam22=None, buf=None, threads=0):
    """Mode P through the C restatement. Returns (buf[yc, xc, 4], rays)."""
    xc = width - x0 if xc is None else xc
    yc = height - y0 if yc is None else yc
    if spheres is None:
        spheres, mats = default_scene_arrays()
    spheres = np.ascontiguousarray(spheres, np.float32)
    mats = np.ascontiguousarray(mats, np.float32)
    if buf is None:
        buf = np.zeros((yc, xc, 4), np.float32)
    cam = None if cam22 is None else np.ascontiguousarray(cam22, np.float32)
    threads = threads or default_threads()
    rays = orc().orc_render_p(_ptr(spheres), _ptr(mats), len(spheres) // 4, _ptr(cam), width, height,
                              x0, xc, y0, yc, frame0, frames, depth, _ptr(buf), threads)
    return buf, rays


FEATURE_NAMES = ("normal", "world_pos", "albedo", "color_std", "normal_std", "world_pos_std")


def orc_render_ex(width, height, frames=1, depth=8, frame0=0, x0=0, xc=None, y0=0, yc=None,
                  spheres=None, mats=None, cam22=None, buf=None, flags=0, features=None, max_frame=4,
                  threads=0):
    """orc_render plus the GL path's opt-in modes: flags & 64 = no double lighting;
    features = {name: float32 buffer[yc, xc, 4]} updated in place. Returns (buf, rays)."""
    xc = width - x0 if xc is None else xc
    yc = height - y0 if yc is None else yc
    if spheres is None:
        spheres, mats = default_scene_arrays()
    spheres = np.ascontiguousarray(spheres, np.float32)
    mats = np.ascontiguousarray(mats, np.float32)
    if buf is None:
        buf = np.zeros((yc, xc, 4), np.float32)
    cam = None if cam22 is None else np.ascontiguousarray(cam22, np.float32)
    fp = None
    if features is not None:
        fp = (ctypes.c_void_p * 6)()
        for i, name in enumerate(FEATURE_NAMES):
            b = features.get(name)
            if b is not None:
                assert b.dtype == np.float32 and b.flags.c_contiguous and b.size == yc * xc * 4
                fp[i] = b.ctypes.data
    rays = orc().orc_render_p_ex(_ptr(spheres), _ptr(mats), len(spheres) // 4, _ptr(cam), width, height,
                                 x0, xc, y0, yc, frame0, frames, depth, flags, _ptr(buf), fp, max_frame,
                                 threads or default_threads())
    return buf, rays


def orc_render_r(width, height, frames=1, depth=20, frame0=0, state=1, spheres=None, mats=None):
    """Mode R (reference stream) through the C restatement. Returns (buf, rays, end_state)."""
    if spheres is None:
        spheres, mats = default_scene_arrays()
    buf = np.zeros((height, width, 4), np.float32)
    st = ctypes.c_uint32(state)
    rays = orc().orc_render_r(_ptr(spheres), _ptr(mats), len(spheres) // 4, width, height, frame0, frames,
                              depth, ctypes.byref(st), _ptr(buf))
    return buf, rays, st.value


def orc_libm(kind: int, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    orc().orc_libm_eval(kind, _ptr(x), _ptr(out), x.size)
    return out


def orc_camera(width, height):
    c = np.zeros(22, np.float32)
    orc().orc_default_camera(width, height, _ptr(c))
    return c


def ref_render_p(width, height, frames=1, depth=8, frame0=0, x0=0, xc=None, y0=0, yc=None,
                 scene=None, cam22=None, procs=1, n=9):
    """Mode P / F through the reference itself. scene=(spheres, mats) overrides the
    reference's statics for the call; n picks the build (9: libref.so, 1000: libref1000.so).
    Returns (buf, rays)."""
    r = ref(n)
    xc = width - x0 if xc is None else xc
    yc = height - y0 if yc is None else yc
    buf = np.zeros((yc, xc, 4), np.float32)
    if scene is not None:
        r.ref_set_scene(_ptr(np.ascontiguousarray(scene[0], np.float32)),
                        _ptr(np.ascontiguousarray(scene[1], np.float32)))
    try:
        cam = None if cam22 is None else np.ascontiguousarray(cam22, np.float32)
        rays = r.ref_render_mode_p_procs(width, height, x0, xc, y0, yc, frame0, frames, depth,
                                         _ptr(cam), _ptr(buf), procs)
    finally:
        if scene is not None:
            r.ref_reset_scene()
    return buf, rays
