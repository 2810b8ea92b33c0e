"""GPU parity for the exact kernel instances behind BASELINE configs 4 and 5.

Configs 4 (3840x2160, 64 spp) and 5 (7680x4320, 256 spp, 8 GPUs) render the 1000-sphere
scene through the BVH with a pixel's frames spread over 16 lanes (trace_kernel<8, *, true,
16>) and many lerp rounds per task. Each test renders a window of that geometry at the
config's REAL spp and checks it bit for bit against the reference's own sources built
with random_scene(1000, 1) as their static scene (tests/golden: scene1000_c4_s64,
scene1000_c5_s256), against the C restatement on larger windows, and against the GPU's
own linear scan (LRT_F_NO_BVH, the reference's HitWorld loop, parallel.cpp:54-73).
lrt_last_launch() names the instance each render launched, so the tests assert they ran
the one the benchmark runs. References: parallel.cpp:54-73 (HitWorld), :262,280-286
(lerp chain over frames).
"""
import numpy as np
import pytest

import oracle
from learnraytracing_amd import _lib as L

pytestmark = pytest.mark.gpu

NO_BVH = 32
V0, POOL = 2, 512   # LRT_F_SIMPLE (trace_kernel), LRT_F_POOL (pool_kernel)
BVH, GRID = 1024, 2048   # LRT_F_BVH, LRT_F_GRID: the closest-hit structure (the grid is the default here)
KERNELS = pytest.mark.parametrize("kflags", [V0, POOL, V0 | BVH, POOL | BVH],
                                  ids=["v0-grid", "pool-grid", "v0-bvh", "pool-bvh"])


def _bitwise(got, want, what):
    g = got[..., :3]
    if not np.array_equal(g.view(np.uint32), np.ascontiguousarray(want[..., :3]).view(np.uint32)):
        d = np.abs(g.astype(np.float64) - want[..., :3].astype(np.float64))
        raise AssertionError(f"{what}: {int((g != want[..., :3]).any(axis=-1).sum())} pixels differ, "
                             f"max |diff| {d.max():.3g}")


@pytest.fixture(scope="module")
def _scene1000_arrays():
    from learnraytracing_amd.scene import random_scene, scene_arrays
    sph, mat = random_scene(1000, 1)
    return (sph, mat), tuple(np.array(v, np.float32) for v in scene_arrays(sph, mat))


@pytest.fixture
def scene1000(gpu, _scene1000_arrays):
    """random_scene(1000, 1) on the devices for one test, then the default scene again (the
    scene guard in conftest.py checks that every GPU test starts on the default scene)."""
    (sph, mat), arrays = _scene1000_arrays
    gpu.set_scene(sph, mat)
    try:
        yield arrays
    finally:
        gpu.set_scene(*gpu.default_scene())


def _render(gpu, flags=0, **kw):
    job = gpu.Job(flags=flags, **kw)
    d = job.desc()
    buf = np.zeros((d.row_count, d.x_count, 4), np.float32)
    rays = gpu.render_host(job, buf)
    return buf, rays, L.last_launch()


def _assert_instance(info, kflags, frames, samp="0"):
    """The instance the benchmark runs for this geometry: trace_kernel with 16 frame lanes
    per pixel (v0), or pool_kernel with its tile size for `frames`; through the uniform grid
    (the library's pick for random_scene(1000)) or, with LRT_F_BVH, the BVH."""
    assert info["acc"] == ("bvh" if kflags & BVH else "grid") and info["maxd"] == "8", info
    if kflags & POOL:
        assert info["kernel"] == "pool_kernel" and info["pix"] == str(64 if frames <= 64 else 16), info
    else:
        assert info["kernel"] == "trace_kernel" and info["split"] == "16" and info["samp"] == samp, info


@KERNELS
@pytest.mark.parametrize("name", ["scene1000_c4_s64", "scene1000_c5_s256"])
def test_config_instance_vs_reference_golden(gpu, scene1000, manifest, images, name, kflags):
    """64 / 256 spp windows of configs 4 / 5 equal the reference's own render."""
    fx = manifest["fixtures"][name]
    assert fx["source"].startswith("reference")
    buf, rays, info = _render(gpu, flags=kflags, width=fx["w"], height=fx["h"], frames=fx["frames"],
                              max_depth=fx["max_depth"], x0=fx["x0"], x_count=fx["xc"], y0=fx["y0"], row_count=fx["yc"])
    _assert_instance(info, kflags, fx["frames"])
    _bitwise(buf, images[name], name)
    assert rays == fx["rays"]


@KERNELS
def test_config4_window_vs_oracle_and_linear_scan(gpu, scene1000, kflags):
    """A 64x24 window of config 4 at 64 spp: BVH == C restatement == GPU linear scan."""
    s, m = scene1000
    kw = dict(width=3840, height=2160, frames=64, max_depth=8, x0=1880, x_count=64, y0=1000, row_count=24)
    a, ra, info = _render(gpu, flags=kflags, **kw)
    _assert_instance(info, kflags, 64)
    want, wr = oracle.orc_render(3840, 2160, 64, 8, 0, 1880, 64, 1000, 24, spheres=s, mats=m, threads=16)
    _bitwise(a, want, "config4 window vs oracle")
    assert ra == wr
    b, rb, info_b = _render(gpu, flags=NO_BVH | kflags, **kw)
    assert info_b["acc"] == "scan" and info_b["kernel"] == info["kernel"]
    assert rb == ra and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@KERNELS
def test_config4_many_tiles_bvh_equals_linear_scan(gpu, scene1000, kflags):
    """Enough 64-spp tiles that the persistent grid refills from its queues several times
    (every block runs many tasks): BVH == linear scan, rays included."""
    # pool tiles are 8x8 pixels at 64 spp: a larger window for more tiles than blocks
    xc, yc = (768, 96) if not kflags & POOL else (1536, 192)
    kw = dict(width=3840, height=2160, frames=64, max_depth=8, x0=1536, x_count=xc, y0=900, row_count=yc)
    a, ra, info = _render(gpu, flags=kflags, **kw)
    _assert_instance(info, kflags, 64)
    assert int(info["tasks"]) > int(info["grid"])
    b, rb, _ = _render(gpu, flags=NO_BVH | kflags, **kw)
    assert rb == ra and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@KERNELS
def test_config5_shard_of_8_vs_oracle(gpu, scene1000, kflags):
    """Rank 3's row-block-cyclic shard of an 8-GPU config-5 frame (row blocks of 8, 256 spp
    per pixel -- the strong-scaling shape, BVH without sample mode): two row bands of a
    24-column window against the restatement."""
    s, m = scene1000
    W, H, rb, G, ph, y0 = 7680, 4320, 8, 8, 3, 2048
    a, ra, info = _render(gpu, flags=kflags, width=W, height=H, frames=256, max_depth=8, x0=3800, x_count=24, y0=y0,
                          row_count=16, row_block=rb, row_period=G, row_phase=ph)
    _assert_instance(info, kflags, 256)
    rays = 0
    for band in range(2):   # local rows 8*band.. map to y0 + band*rb*G + ph*rb ..
        gy = y0 + band * rb * G + ph * rb
        want, wr = oracle.orc_render(W, H, 256, 8, 0, 3800, 24, gy, rb, spheres=s, mats=m, threads=16)
        _bitwise(a[band * rb:(band + 1) * rb], want, f"config5 shard band {band}")
        rays += wr
    assert ra == rays


@pytest.mark.parametrize("scene", ["config2_window", "scene1000"])
def test_pool_tile_order_keeps_every_pixel(gpu, request, scene):
    """The pool kernel's heaviest-first tile order (tile_order in lrt_hip.hip): the first
    launch of a render signature records per-tile costs in the order of a cost probe
    (probe_kernel; or one borrowed from the same geometry), the later ones hand tiles out by
    descending measured cost. Every launch must give the same bits and ray count."""
    kw = (dict(width=1280, height=720, frames=4, max_depth=8, x0=256, x_count=256, y0=128, row_count=128)
          if scene == "config2_window" else
          dict(width=3840, height=2160, frames=64, max_depth=8, x0=1800, x_count=64, y0=900, row_count=64))
    if scene == "scene1000":
        request.getfixturevalue("scene1000")
    runs = [_render(gpu, flags=POOL, **kw) for _ in range(4)]
    orders = [info.get("order") for _, _, info in runs]
    assert orders[0] in ("3", "4") and orders[-1] == "2", orders   # recorded, then reordered
    for k, (buf, rays, _) in enumerate(runs[1:], 1):
        _bitwise(buf, runs[0][0], f"{scene} launch {k} vs the recording launch")
        assert rays == runs[0][1]



@pytest.mark.parametrize("acc", [0, BVH], ids=["grid", "bvh"])
def test_probe_ordered_first_launch_vs_oracle(gpu, scene1000, acc):
    """A render signature whose geometry has no measured order yet runs its first (recording)
    launch in the order of the tile-cost probe (probe_kernel + probe_order_kernel, order=4;
    the grid's and the BVH's probe here, the 9-sphere one in test_gpu_multidev). The probe only
    permutes the tiles: pixels and ray count equal the restatement's. No other test uses the
    window's shape, so no order can be borrowed."""
    s, m = scene1000
    x0 = 1712 if acc else 1616   # a window per structure: each one's first launch probes
    kw = dict(width=3840, height=2160, frames=64, max_depth=8, x0=x0, x_count=88, y0=1000, row_count=40)
    want, wr = oracle.orc_render(3840, 2160, 64, 8, 0, x0, 88, 1000, 40, spheres=s, mats=m, threads=16)
    buf, rays, info = _render(gpu, flags=POOL | acc, **kw)
    assert info["kernel"] == "pool_kernel" and info["acc"] == ("bvh" if acc else "grid") and info["order"] == "4", info
    _bitwise(buf, want, "probe-ordered first launch")
    assert rays == wr
    buf2, rays2, info2 = _render(gpu, flags=POOL | acc, **kw)   # then the measured order, recording again
    assert info2["order"] == "5", info2
    _bitwise(buf2, want, "measured order")
    assert rays2 == wr


FAR_CAMERAS = {
    # the round-4 verdict's probe: far and narrow, every camera ray from ~80 units away
    "far_narrow": ((0, 40, 70), (0, -0.4, -2), 8.0),
    # low over the ground from ~35 units: rays graze the field (the grid's cone test and scan)
    "grazing": ((30, 0.2, 18), (0, -0.4, -2), 20.0),
}


@pytest.mark.parametrize("cam_name", sorted(FAR_CAMERAS))
@KERNELS
def test_far_camera_window_vs_oracle(gpu, scene1000, kflags, cam_name):
    """Config 4's scene from cameras far outside it: the grid's and the BVH's
    padding covers the reference's own hit points only for origins near the spheres; rays from
    farther away inflate the BVH's boxes by their own bound, or finish the grid's walk with the
    scan when the walk cannot be certain. Every pixel must still equal the restatement's."""
    s, m = scene1000
    frm, at, vfov = FAR_CAMERAS[cam_name]
    w, h = 640, 360
    dist = float(np.linalg.norm(np.subtract(frm, at)))
    cam = gpu.make_camera(frm, at, (0, 1, 0), vfov, w / h, 0.1, dist)
    kw = dict(width=w, height=h, frames=16, max_depth=8, x0=288, x_count=64, y0=150, row_count=40, camera=cam)
    a, ra, info = _render(gpu, flags=kflags, **kw)
    assert info["acc"] == ("bvh" if kflags & BVH else "grid"), info
    want, wr = oracle.orc_render(w, h, 16, 8, 0, 288, 64, 150, 40, spheres=s, mats=m, cam22=cam.to22(), threads=16)
    _bitwise(a, want, f"{cam_name} camera window")
    assert ra == wr


@pytest.mark.parametrize("cam_name", sorted(FAR_CAMERAS))
def test_far_camera_window_wavefront_vs_oracle(gpu, scene1000, cam_name):
    """The same far cameras through the v4 wavefront kernels (LRT_F_WAVEFRONT), whose extend
    kernel traces the BVH: its per-ray excursion margins hold there too."""
    s, m = scene1000
    frm, at, vfov = FAR_CAMERAS[cam_name]
    w, h = 640, 360
    dist = float(np.linalg.norm(np.subtract(frm, at)))
    cam = gpu.make_camera(frm, at, (0, 1, 0), vfov, w / h, 0.1, dist)
    kw = dict(width=w, height=h, frames=4, max_depth=8, x0=288, x_count=64, y0=150, row_count=40, camera=cam)
    a, ra, info = _render(gpu, flags=256, **kw)
    assert info["kernel"] == "wf_extend" and info["bvh"] == "1", info
    want, wr = oracle.orc_render(w, h, 4, 8, 0, 288, 64, 150, 40, spheres=s, mats=m, cam22=cam.to22(), threads=16)
    _bitwise(a, want, f"{cam_name} camera window (wavefront)")
    assert ra == wr
