"""The C-ABI library: it loads without a GPU, exports every symbol include/lrt.h
declares, its structs have the reference layouts, and its host-only entry points
(camera, default scene, shard geometry, argument validation) behave."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from learnraytracing_amd import _lib as L
from learnraytracing_amd import dist as D
from learnraytracing_amd.renderer import Job, default_camera, make_camera


def header_functions(path=None):
    src = open(path or L.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\**\s*(lrt_\w+)\s*\(", src, flags=re.M)))


def exported_functions():
    """The dynamic symbols the library defines under the lrt_ prefix."""
    import shutil
    import subprocess
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    out = subprocess.run([nm, "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("lrt_")})


def test_library_exports_every_declared_symbol():
    api, diag = header_functions(), header_functions(L.DIAG_HEADER_PATH)
    assert len(api) >= 16 and len(diag) >= 5
    lib = L.lib()
    for n in api + diag:
        assert hasattr(lib, n), n
    assert set(api) == set(L.SIGNATURES), "ctypes signatures out of sync with include/lrt.h"
    assert set(diag) == set(L.DIAG_SIGNATURES), "ctypes signatures out of sync with include/lrt_diag.h"


def test_removed_entry_points_and_flags_are_gone():
    """Round 6 trimmed the surface: no no-op lrt_host_unregister, no removed-kernel flags."""
    src = open(L.HEADER_PATH).read()
    for name in ("LRT_F_V1", "LRT_F_V2S", "LRT_F_V2 ", "LRT_F_V3", "lrt_host_unregister"):
        assert name not in src, name
    assert "lrt_host_unregister" not in exported_functions()


def test_exported_symbol_set_is_the_two_headers():
    """The renderer API (include/lrt.h) holds no diagnostics; the library exports exactly the
    renderer API plus the diagnostics of include/lrt_diag.h, nothing else under lrt_."""
    api, diag = header_functions(), header_functions(L.DIAG_HEADER_PATH)
    assert not set(api) & set(diag)
    for n in api:
        assert not re.search(r"_stats$|_eval(_|$)", n), f"diagnostic {n} in the renderer API"
    assert exported_functions() == sorted(api + diag)


def test_library_is_gfx950_code():
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert L.lib().lrt_version().decode().endswith("gfx950")


def test_library_carries_roctx_ranges():
    """SURVEY §5 tracing: the C-ABI's work entry points push roctx ranges (rocprofv3
    --marker-trace), so the library imports the roctx API and names its ranges."""
    import shutil
    import subprocess
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    und = subprocess.run([nm, "-D", "--undefined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    assert "roctxRangePushA" in und and "roctxRangePop" in und
    blob = open(L.LIB_PATH, "rb").read()
    for name in (b"lrt_draw_test", b"lrt_render_device", b"lrt_render_host", b"lrt_set_scene"):
        assert name + b"\0" in blob


def test_struct_layouts_match_reference():
    assert ctypes.sizeof(L.Float3) == 12          # maths.h float3
    assert ctypes.sizeof(L.Sphere) == 16          # maths.h Sphere
    assert ctypes.sizeof(L.Material) == 36        # parallel.cpp Material
    assert [getattr(L.Material, f).offset for f in ("type", "albedo", "emissive", "roughness", "ri")] == \
        [0, 4, 16, 28, 32]
    assert ctypes.sizeof(L.Camera) == 88          # maths.h Camera


def test_camera_matches_reference(kat):
    for key, want in kat["default_camera"].items():
        w, h = (int(v) for v in key.split("x"))
        assert np.array_equal(np.array(default_camera(w, h).to22(), np.float32), np.array(want, np.float32)), key
    c = make_camera((0, 2, 3), (0, 0, 0), (0, 1, 0), 60, 1280 / 720, 0.1, 3)
    assert np.array_equal(np.array(c.to22(), np.float32), np.array(kat["default_camera"]["1280x720"], np.float32))


def test_default_scene_matches_reference():
    spheres = (L.Sphere * 9)()
    mats = (L.Material * 9)()
    n = ctypes.c_int()
    assert L.lib().lrt_default_scene(spheres, mats, 9, ctypes.byref(n)) == 0 and n.value == 9
    s, m = oracle.default_scene_arrays()
    got_s = np.array([[sp.center.x, sp.center.y, sp.center.z, sp.radius] for sp in spheres], np.float32).ravel()
    got_m = np.array([[mt.type, *mt.albedo.tolist(), *mt.emissive.tolist(), mt.roughness, mt.ri] for mt in mats],
                     np.float32).ravel()
    assert np.array_equal(got_s, s) and np.array_equal(got_m, m)
    if oracle.have_ref():
        rs, rm = np.zeros(36, np.float32), np.zeros(81, np.float32)
        oracle.ref().ref_get_scene(oracle._ptr(rs), oracle._ptr(rm))
        assert np.array_equal(rs, s) and np.array_equal(rm, m)
    assert L.lib().lrt_default_scene(spheres, mats, 8, ctypes.byref(n)) == L.LRT_E_INVALID


@pytest.mark.parametrize("h,rb,g", [(720, 8, 1), (720, 8, 2), (720, 8, 8), (181, 8, 3), (7, 8, 4), (4320, 16, 8),
                                    (1, 1, 1), (0, 4, 2)])
def test_shard_geometry(h, rb, g):
    total = 0
    seen = []
    for p in range(g):
        n = L.lib().lrt_shard_rows(h, rb, g, p)
        assert n == D.shard_rows(h, rb, g, p)
        rows = D.shard_global_rows(h, rb, g, p)
        assert len(rows) == n and (rows < max(h, 1)).all()
        seen.extend(rows.tolist())
        total += n
    assert total == h and sorted(seen) == list(range(h))
    assert D.max_shard_rows(h, rb, g) == max(L.lib().lrt_shard_rows(h, rb, g, p) for p in range(g))
    assert L.lib().lrt_shard_rows(h, rb, g, g) == L.LRT_E_INVALID


def test_validation_before_device_use():
    """Invalid descriptors are rejected with LRT_E_INVALID; valid ones without
    lrt_initialize() with LRT_E_STATE -- no GPU needed for either."""
    lib = L.lib()
    buf = np.zeros(64 * 36 * 4, np.float32)
    rays = ctypes.c_longlong()

    def call(**kw):
        d = Job(width=64, height=36, **kw).desc()
        return lib.lrt_render_host(ctypes.byref(d), buf.ctypes.data_as(ctypes.c_void_p), ctypes.byref(rays))

    assert call(max_depth=65) == L.LRT_E_INVALID
    assert call(max_depth=-1) == L.LRT_E_INVALID
    assert call(x0=10, x_count=60) == L.LRT_E_INVALID
    assert call(frames=-1) == L.LRT_E_INVALID
    assert call(y0=30, row_count=7) == L.LRT_E_INVALID
    assert call(row_block=8, row_period=2, row_phase=2, row_count=1) == L.LRT_E_INVALID
    assert call(row_block=8, row_period=4, row_phase=3, row_count=9) == L.LRT_E_INVALID   # maps past row 35
    assert "image" in lib.lrt_last_error().decode() or "row" in lib.lrt_last_error().decode()
    if os.environ.get("HIP_VISIBLE_DEVICES") == "" or not _gpu_present():
        assert call() == L.LRT_E_STATE
    assert lib.lrt_draw_test(0.0, 0, 0, 36, buf.ctypes.data_as(ctypes.c_void_p), None) == L.LRT_E_INVALID


def _gpu_present():
    import torch
    return torch.cuda.device_count() > 0
