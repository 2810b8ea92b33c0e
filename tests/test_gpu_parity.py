"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors
and the CPU oracle on the same seeded inputs. The bar is BIT-EXACT: every pixel,
every channel, and the counted rays, equal (the stated tolerance of north_star is
1e-4 per channel; we assert 0 and report the max |diff| on failure).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _assert_bitwise(got_rgba, want_rgb, what):
    got = got_rgba[..., :3]
    if not np.array_equal(got.view(np.uint32), np.ascontiguousarray(want_rgb).view(np.uint32)):
        d = np.abs(got.astype(np.float64) - want_rgb.astype(np.float64))
        bad = int((got != want_rgb).any(axis=-1).sum())
        raise AssertionError(f"{what}: {bad} pixels differ, max |diff| {d.max():.3g}, "
                             f"pixels > 1e-4: {int((d > 1e-4).any(axis=-1).sum())}")


def _render(lrt, w, h, frames, depth, frame0=0, x0=0, xc=None, y0=0, yc=None, camera=None, flags=0,
            buf=None):
    job = lrt.Job(width=w, height=h, frame0=frame0, frames=frames, max_depth=depth, x0=x0, x_count=xc,
                  y0=y0, row_count=yc, camera=camera, flags=flags)
    d = job.desc()
    if buf is None:
        buf = np.zeros((d.row_count, d.x_count, 4), np.float32)
    rays = lrt.render_host(job, buf)
    return buf, rays


@pytest.mark.parametrize("name", ["p_160x90_s4_d8", "p_320x180_s4_d8", "p_96x54_s1_d50", "p_128x72_s2_d20",
                                  "p_128x72_f5_s3_d8", "c2_crop", "c3_crop", "c5_crop"])
def test_golden_mode_p(gpu, manifest, images, name):
    fx = manifest["fixtures"][name]
    buf, rays = _render(gpu, fx["w"], fx["h"], fx["frames"], fx["max_depth"], fx["frame0"],
                        fx["x0"], fx["xc"], fx["y0"], fx["yc"])
    _assert_bitwise(buf, images[name], name)
    assert rays == fx["rays"]


@pytest.mark.parametrize("flags", [0, 1, 2, 3, 256, 257, 512, 513])
@pytest.mark.parametrize("name", ["p_160x90_s4_d8", "p_96x54_s1_d50"])
def test_golden_kernel_variants(gpu, manifest, images, flags, name):
    """Every kernel (the policy's pick, v0 LRT_F_SIMPLE, v4 LRT_F_WAVEFRONT, v5 LRT_F_POOL),
    with LDS-staged or global scene reads, gives the same bits."""
    fx = manifest["fixtures"][name]
    buf, rays = _render(gpu, fx["w"], fx["h"], fx["frames"], fx["max_depth"], flags=flags)
    _assert_bitwise(buf, images[name], f"{name} flags={flags}")
    assert rays == fx["rays"]


def test_golden_fuzz(gpu, manifest, images):
    from learnraytracing_amd import _lib as L
    from learnraytracing_amd.scene import scene_from_arrays
    try:
        for fz in manifest["fuzz"]:
            gpu.set_scene(*scene_from_arrays(fz["spheres"], fz["mats"]))
            cam = L.Camera()
            vals = fz["camera"]
            names = ("origin", "a", "u", "r", "lowerLeftCorner", "horizontalVec", "verticalVec")
            for i, n in enumerate(names):
                setattr(cam, n, L.f3(*vals[3 * i:3 * i + 3]))
            cam.lensRadius = vals[21]
            buf, rays = _render(gpu, fz["w"], fz["h"], fz["frames"], fz["max_depth"], camera=cam)
            _assert_bitwise(buf, images[fz["name"]], fz["name"])
            assert rays == fz["rays"], fz["name"]
    finally:
        gpu.set_scene(*gpu.default_scene())


@pytest.mark.parametrize("name", ["scene1000_c4_crop", "scene1000_c5_crop"])
def test_golden_scene1000(gpu, manifest, images, name):
    fx = manifest["fixtures"][name]
    try:
        gpu.set_scene(*gpu.random_scene(1000, 1))
        buf, rays = _render(gpu, fx["w"], fx["h"], fx["frames"], fx["max_depth"], 0, fx["x0"], fx["xc"],
                            fx["y0"], fx["yc"])
    finally:
        gpu.set_scene(*gpu.default_scene())
    _assert_bitwise(buf, images[name], name)
    assert rays == fx["rays"]


def test_config2_full_frame_vs_oracle(gpu):
    """BASELINE config 2 at full size: 1280x720, 4 spp, 8 bounces, bit-exact vs the
    C oracle (11.67 M rays) and ray count equal."""
    buf, rays = _render(gpu, 1280, 720, 4, 8)
    want, wrays = oracle.orc_render(1280, 720, 4, 8)
    _assert_bitwise(buf, want[..., :3], "config2 full frame")
    assert rays == wrays


def test_config3_rows_vs_oracle(gpu):
    """Config 3 geometry (1920x1080, 16 spp, 50 bounces) on a band of 40 full rows."""
    buf, rays = _render(gpu, 1920, 1080, 16, 50, y0=520, yc=40)
    want, wrays = oracle.orc_render(1920, 1080, 16, 50, y0=520, yc=40)
    _assert_bitwise(buf, want[..., :3], "config3 rows")
    assert rays == wrays


def test_draw_test_dropin(gpu):
    """DrawTest semantics (kMaxDepth 20, default camera, one frame per call) against
    the oracle, frames 0..2 progressively into the same buffer."""
    w, h = 200, 120
    bb = np.zeros(w * h * 4, np.float32)
    want = np.zeros((h, w, 4), np.float32)
    for f in range(3):
        rays = gpu.DrawTest(0.0, f, w, h, bb)
        _, wr = oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
        assert rays == wr
    _assert_bitwise(bb.reshape(h, w, 4), want[..., :3], "DrawTest x3")


def test_draw_test_pinned_backbuffer(gpu):
    """A page-locked backbuffer is rendered in place over PCIe (zero copy): same bits and
    rays as the oracle, frames 0..2, and the caller's alpha is left as it was."""
    w, h = 200, 117
    bb = gpu.pinned_backbuffer(w * h * 4)
    bb[3::4] = 0.25
    want = np.zeros((h, w, 4), np.float32)
    for f in range(3):
        rays = gpu.DrawTest(0.0, f, w, h, bb)
        _, wr = oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
        assert rays == wr
    _assert_bitwise(bb.reshape(h, w, 4), want[..., :3], "DrawTest pinned x3")
    assert np.all(bb[3::4] == 0.25)


def test_host_alloc_backbuffer(gpu):
    """lrt_host_alloc (main.cpp:40's `new float[]` made page-locked): DrawTest into it equals
    DrawTest into pageable memory, bit for bit, rays included."""
    import ctypes
    w, h = 96, 54
    n = w * h * 4
    p = ctypes.c_void_p()
    assert gpu.lib().lrt_host_alloc(n * 4, ctypes.byref(p)) == 0 and p.value
    try:
        a = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(n,))
        a[:] = 0.0
        b = np.zeros(n, np.float32)
        for f in range(2):
            assert gpu.DrawTest(0.0, f, w, h, a) == gpu.DrawTest(0.0, f, w, h, b)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    finally:
        assert gpu.lib().lrt_host_free(p) == 0


@pytest.mark.parametrize("kflags,frames", [(0, 6), (0, 40), (256, 6)], ids=["v0", "v0-samples", "wavefront"])
def test_render_host_pinned_window(gpu, kflags, frames):
    """lrt_render_host on a pinned buffer: a window of 37 rows x 90 columns equals the
    pageable call bit for bit (and so the one-launch render), alpha included; v0 (also with
    many frames, sample mode's merge) and the wavefront kernels (which stage instead)."""
    job = gpu.Job(width=160, height=90, frames=frames, max_depth=8, x0=30, x_count=90, y0=40, row_count=37,
                  flags=kflags)
    a = np.random.default_rng(3).uniform(0, 1, 37 * 90 * 4).astype(np.float32)
    b = gpu.pinned_backbuffer(37 * 90 * 4)
    b[:] = a
    ra = gpu.render_host(job, a)
    rb = gpu.render_host(job, b)
    assert ra == rb > 0
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_fused_frames_equal_single_frame_calls(gpu):
    """S samples in one call == S one-sample calls (the progressive lerp chain)."""
    a, ra = _render(gpu, 256, 144, 6, 8)
    b = np.zeros_like(a)
    rb = 0
    for f in range(6):
        _, r = _render(gpu, 256, 144, 1, 8, frame0=f, buf=b)
        rb += r
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and ra == rb


def test_alpha_untouched(gpu):
    buf = np.full((36, 64, 4), 7.25, np.float32)
    _render(gpu, 64, 36, 2, 8, buf=buf)
    assert (buf[..., 3] == 7.25).all()


def test_row_block_cyclic_shards_assemble_bitwise(gpu):
    """G shards rendered with row_period=G, gathered and un-interleaved by the
    unshard kernel, equal the single-call frame bit for bit (per-pixel seeds)."""
    import torch
    w, h, G, rb = 320, 181, 3, 8
    full, rays_full = _render(gpu, w, h, 2, 8)
    max_rows = gpu.shard_rows(h, rb, G, 0)
    gathered = torch.zeros((G, max_rows, w, 4), dtype=torch.float32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    for g in range(G):
        job = gpu.Job(width=w, height=h, frames=2, max_depth=8, row_block=rb, row_period=G, row_phase=g)
        gpu.render_tensor(job, gathered[g], rays)
    out = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
    from learnraytracing_amd.renderer import unshard_tensor
    unshard_tensor(gathered, out, w, h, rb, G)
    torch.cuda.synchronize()
    _assert_bitwise(out.cpu().numpy(), full[..., :3], "sharded assemble")
    assert int(rays.item()) == rays_full


def test_present_bgra8_matches_linear_to_srgb(gpu):
    """Present step (main.cpp:109-141) vs the same formula on the host with glibc powf."""
    import torch
    from learnraytracing_amd.renderer import present_tensor
    g = np.random.default_rng(3)
    w, h = 97, 33
    rgba = g.uniform(-0.5, 60.0, (h, w, 4)).astype(np.float32)
    rgba[0, :8, 0] = [0.0, -0.0, 1e-30, 1.0, 0.5, 49.0, 1e6, -3.0]
    t = torch.from_numpy(rgba).cuda()
    out = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    present_tensor(t, out, w, h)
    got = out.cpu().numpy().view(np.uint32).reshape(h, w)

    def srgb(x):
        x = np.where(x < 0, np.float32(0), x).astype(np.float32)
        p = oracle.orc_libm(3, x)
        y = (np.float32(1.055) * p - np.float32(0.055)).astype(np.float32)
        y = np.where(y < 0, np.float32(0), y).astype(np.float32)
        u = (y * np.float32(255.9)).astype(np.float32)
        return np.minimum(u.astype(np.uint64), 255).astype(np.uint32)

    want = srgb(rgba[..., 2]) | (srgb(rgba[..., 1]) << 8) | (srgb(rgba[..., 0]) << 16)
    assert np.array_equal(got, want)


def test_libm_device_exhaustive_path_domain(gpu, manifest):
    """Device sinf/cosf over every input the path can produce (2^24 values) hash to
    glibc's outputs; powf digests likewise."""
    import hashlib
    import torch
    from learnraytracing_amd import _lib as L
    k = torch.arange(1 << 24, dtype=torch.int64)
    phi = (np.float32(2.0) * np.float32(3.1415926)) * (k.numpy().astype(np.float32) * np.float32(2.0 ** -24))
    phi = torch.from_numpy(phi.astype(np.float32)).cuda()
    out = torch.empty_like(phi)

    def dev(kind, x):
        o = torch.empty_like(x)
        L.check(L.lib().lrt_libm_eval_device(kind, x.data_ptr(), o.data_ptr(), x.numel()))
        return o.cpu().numpy()

    lm = manifest["libm"]
    assert hashlib.sha256(dev(0, phi).tobytes()).hexdigest() == lm["sinf_sha256"]
    assert hashlib.sha256(dev(1, phi).tobytes()).hexdigest() == lm["cosf_sha256"]
    # the path's branch-free sincosf (lrt_libm.h): both results over the same domain
    assert hashlib.sha256(dev(6, phi).tobytes()).hexdigest() == lm["sinf_sha256"]
    assert hashlib.sha256(dev(7, phi).tobytes()).hexdigest() == lm["cosf_sha256"]
    pw = torch.from_numpy(np.linspace(0, 1, 1 << 20, dtype=np.float32)).cuda()
    assert hashlib.sha256(dev(2, pw).tobytes()).hexdigest() == lm["powf5_linspace01_2p20_sha256"]
    sr = torch.from_numpy(np.linspace(0, 64, 1 << 20, dtype=np.float32)).cuda()
    assert hashlib.sha256(dev(3, sr).tobytes()).hexdigest() == lm["powf_srgb_linspace064_2p20_sha256"]
    del out


def test_powf5_device_fast_path_domain(gpu):
    """The device's powf5 (fast path + glibc fallback) on every float of [2^-14, 1] equals the
    host build, which tests/test_libm.py checks against glibc on the same floats."""
    import torch
    from learnraytracing_amd import _lib as L
    from test_libm import product
    lo, hi, step = 0x38800000, 0x3F800000, 1 << 24
    for a in range(lo, hi + 1, step):
        x = np.arange(a, min(a + step, hi + 1), dtype=np.uint32).view(np.float32)
        d_in = torch.from_numpy(x).cuda()
        d_out = torch.empty_like(d_in)
        L.check(L.lib().lrt_libm_eval_device(2, d_in.data_ptr(), d_out.data_ptr(), d_in.numel()))
        got = d_out.cpu().numpy()
        want = product(2, x)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), hex(a)


def test_fast_sqrt_rcp_correctly_rounded(gpu):
    """The device's short sqrt / reciprocal sequences (lrt_trace.h sqrt_rn, rcp_rn) equal
    IEEE sqrtf and 1/x bit for bit: every mantissa at exponents around the fast paths'
    limits and in the path's range, plus 2^24 random bit patterns (signs, zeros,
    denormals, inf, NaN). tools/fpexact.hip checks all 2^32 inputs."""
    import torch
    from learnraytracing_amd import _lib as L
    m = np.arange(1 << 23, dtype=np.uint32)
    exps = [0, 1, 20, 23, 24, 30, 31, 32, 33, 100, 126, 127, 128, 150, 220, 250, 251, 252, 253, 254, 255]
    pats = [m | np.uint32(e << 23) for e in exps]
    pats.append(np.random.default_rng(5).integers(0, 1 << 32, 1 << 24, dtype=np.uint64).astype(np.uint32))
    bits = np.concatenate(pats)
    bits = np.concatenate([bits, bits | np.uint32(0x80000000)])
    x = bits.view(np.float32)
    with np.errstate(all="ignore"):
        want = {4: np.sqrt(x), 5: np.float32(1.0) / x}
    d_in = torch.from_numpy(x).cuda()
    for kind, w in want.items():
        d_out = torch.empty_like(d_in)
        L.check(L.lib().lrt_libm_eval_device(kind, d_in.data_ptr(), d_out.data_ptr(), d_in.numel()))
        got = d_out.cpu().numpy()
        same = (got.view(np.uint32) == w.view(np.uint32)) | (np.isnan(got) & np.isnan(w))
        assert same.all(), f"kind {kind}: {int((~same).sum())} mismatches, first x={x[~same][:4]}"


def test_invalid_arguments_fail_loudly(gpu):
    from learnraytracing_amd import LrtError
    with pytest.raises(LrtError):
        _render(gpu, 64, 36, 1, 65)                      # depth > 64
    with pytest.raises(LrtError):
        _render(gpu, 64, 36, 1, 8, x0=10, xc=60)         # window outside the image
    with pytest.raises(LrtError):
        gpu.DrawTest(0.0, 0, 64, 36, np.zeros(10, np.float32))


def test_deterministic_repeat_full_config2(gpu):
    a, ra = _render(gpu, 1280, 720, 4, 8)
    b, rb = _render(gpu, 1280, 720, 4, 8)
    assert ra == rb and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("n,seed", [(17, 3), (200, 5), (1000, 1), (4096, 7)])
@pytest.mark.parametrize("kflags", [2, 256, 512])
def test_bvh_equals_linear_scan(gpu, n, seed, kflags):
    """The BVH closest hit returns the reference's scan result bit for bit: same
    pixels and ray counts as LRT_F_NO_BVH, for every kernel."""
    try:
        gpu.set_scene(*gpu.random_scene(n, seed))
        args = (3840, 2160, 2, 8, 0, 1880, 64, 980, 48)
        a, ra = _render(gpu, *args, flags=kflags)
        b, rb = _render(gpu, *args, flags=kflags | 32)
    finally:
        gpu.set_scene(*gpu.default_scene())
    assert ra == rb
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_bvh_vs_oracle_random_scene(gpu):
    """A 300-sphere scene through the BVH against the C oracle's linear scan."""
    from learnraytracing_amd.scene import scene_arrays
    sph, mat = gpu.random_scene(300, 11)
    s, m = (np.array(v, np.float32) for v in scene_arrays(sph, mat))
    try:
        gpu.set_scene(sph, mat)
        buf, rays = _render(gpu, 640, 360, 3, 8, y0=150, yc=40)
    finally:
        gpu.set_scene(*gpu.default_scene())
    want, wrays = oracle.orc_render(640, 360, 3, 8, y0=150, yc=40, spheres=s, mats=m)
    _assert_bitwise(buf, want[..., :3], "bvh 300 spheres")
    assert rays == wrays


def test_work_counters_across_slots_and_streams(gpu):
    """v0's per-launch tile queues and ray counters live in rotating slots that the
    launch's collect kernel zeroes: > 2 x 64 launches in a row, and launches in flight
    on two streams at once, must all give the same image and ray count."""
    import torch
    want, wr = _render(gpu, 96, 54, 4, 8)
    for _ in range(140):
        got, r = _render(gpu, 96, 54, 4, 8)
        assert r == wr
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    job = gpu.Job(width=320, height=180, frame0=0, frames=4, max_depth=8)
    one, r1 = _render(gpu, 320, 180, 4, 8)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [torch.zeros((180, 320, 4), dtype=torch.float32, device="cuda") for _ in range(8)]
    rays = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(8)]
    for st in streams:   # after the buffers' zero fills (current stream)
        st.wait_stream(torch.cuda.current_stream())
    for i in range(8):
        gpu.render_tensor(job, bufs[i], rays[i], streams[i % 2])
    torch.cuda.synchronize()
    for b, r in zip(bufs, rays):
        assert int(r.item()) == r1
        assert np.array_equal(b.cpu().numpy().view(np.uint32), one.view(np.uint32))


def test_cu_reserved_render_stream(gpu):
    """lrt_stream_create: a CU-masked stream (for overlap with RCCL) renders the same bits
    with a grid sized to the CUs it may use."""
    import torch
    from learnraytracing_amd.renderer import RenderStream
    want, wr = _render(gpu, 320, 180, 4, 8)
    job = gpu.Job(width=320, height=180, frame0=0, frames=4, max_depth=8)
    # num_cus - 1 leaves ONE CU: fewer resident blocks than v0's 16 tile queues, and every
    # queue still needs a block of its own
    for reserved in (8, 200, torch.cuda.get_device_properties(0).multi_processor_count - 1):
        rs = RenderStream(reserved)
        try:
            buf = torch.zeros((180, 320, 4), dtype=torch.float32, device="cuda")
            rays = torch.zeros(1, dtype=torch.int64, device="cuda")
            rs.torch.wait_stream(torch.cuda.current_stream())   # after the zero fills
            gpu.render_tensor(job, buf, rays, rs.torch)
            rs.torch.synchronize()
            assert int(rays.item()) == wr
            assert np.array_equal(buf.cpu().numpy().view(np.uint32), want.view(np.uint32))
        finally:
            rs.close()


V0 = 2     # LRT_F_SIMPLE: the per-pixel loop, frames over lanes
WF = 256   # LRT_F_WAVEFRONT: breadth-first kernels over compacted queues
POOL = 512   # LRT_F_POOL: sample-pool regeneration inside the wave
ALT = pytest.mark.parametrize("kflags", [V0, WF, POOL], ids=["v0", "wavefront", "pool"])


@ALT
def test_kernel_config2_full_frame_vs_oracle(gpu, kflags):
    """Each kernel forced on BASELINE config 2 at full size, bit-exact vs the C oracle."""
    buf, rays = _render(gpu, 1280, 720, 4, 8, flags=kflags)
    want, wrays = oracle.orc_render(1280, 720, 4, 8)
    _assert_bitwise(buf, want[..., :3], f"flags={kflags} config2 full frame")
    assert rays == wrays


@pytest.mark.parametrize("bit", [4, 8, 16, 128, 1 << 20])
def test_removed_and_unknown_flags_are_rejected(gpu, bit):
    """The removed kernels' bits (v1 4, v2s 8, v2 16, v3 128) and any other undefined bit fail
    loudly instead of running another kernel."""
    from learnraytracing_amd import _lib as L
    with pytest.raises(L.LrtError) as e:
        _render(gpu, 16, 8, 1, 8, flags=bit)
    assert e.value.code == L.LRT_E_INVALID


@pytest.mark.parametrize("case", [
    (97, 55, 3, 8, 0, 0, None, 0, None),       # partial 8x8 tiles on both edges
    (640, 360, 5, 20, 2, 13, 301, 7, 45),      # window, frame offset, odd frame count
    (1920, 1080, 16, 50, 0, 0, None, 520, 24), # config 3 band: deep paths, overflow stack
    (33, 9, 1, 8, 0, 0, None, 0, None),        # fewer pixels than one wave per queue
])
@ALT
def test_kernel_windows_vs_oracle(gpu, case, kflags):
    w, h, frames, depth, f0, x0, xc, y0, yc = case
    buf, rays = _render(gpu, w, h, frames, depth, frame0=f0, x0=x0, xc=xc, y0=y0, yc=yc, flags=kflags)
    want, wrays = oracle.orc_render(w, h, frames, depth, frame0=f0, x0=x0, xc=xc, y0=y0, yc=yc)
    _assert_bitwise(buf, want[..., :3], f"flags={kflags} {case}")
    assert rays == wrays


@ALT
def test_kernel_fuzz_and_scene1000(gpu, manifest, images, kflags):
    """Each kernel on the fuzzed scenes (all materials, TIR, 1-3 lights) and the 1000-sphere crops."""
    from learnraytracing_amd import _lib as L
    from learnraytracing_amd.scene import scene_from_arrays
    try:
        for fz in manifest["fuzz"]:
            gpu.set_scene(*scene_from_arrays(fz["spheres"], fz["mats"]))
            cam = L.Camera()
            vals = fz["camera"]
            names = ("origin", "a", "u", "r", "lowerLeftCorner", "horizontalVec", "verticalVec")
            for i, n in enumerate(names):
                setattr(cam, n, L.f3(*vals[3 * i:3 * i + 3]))
            cam.lensRadius = vals[21]
            buf, rays = _render(gpu, fz["w"], fz["h"], fz["frames"], fz["max_depth"], camera=cam, flags=kflags)
            _assert_bitwise(buf, images[fz["name"]], f"flags={kflags} " + fz["name"])
            assert rays == fz["rays"], fz["name"]
        gpu.set_scene(*gpu.random_scene(1000, 1))
        for name in ("scene1000_c4_crop", "scene1000_c5_crop"):
            fx = manifest["fixtures"][name]
            buf, rays = _render(gpu, fx["w"], fx["h"], fx["frames"], fx["max_depth"], 0, fx["x0"], fx["xc"],
                                fx["y0"], fx["yc"], flags=kflags)
            _assert_bitwise(buf, images[name], f"flags={kflags} " + name)
            assert rays == fx["rays"]
    finally:
        gpu.set_scene(*gpu.default_scene())


@ALT
def test_kernel_row_block_cyclic_shard(gpu, kflags):
    """A shard (rows dealt in blocks of 8 over 3 ranks, rank 1) equals the oracle's rows."""
    w, h, rb, period, phase = 320, 180, 8, 3, 1
    rows = [y for y in range(h) if (y // rb) % period == phase]
    job = gpu.Job(width=w, height=h, frames=2, max_depth=8, row_block=rb, row_period=period, row_phase=phase,
                  flags=kflags)
    buf = np.zeros((len(rows), w, 4), np.float32)
    rays = gpu.render_host(job, buf)
    want, wrays = oracle.orc_render(w, h, 2, 8)
    _assert_bitwise(buf, want[rows][..., :3], f"flags={kflags} shard")
    assert rays == sum(oracle.orc_render(w, h, 2, 8, y0=y, yc=1)[1] for y in rows)


@pytest.mark.parametrize("case", [
    (320, 90, 32, 8, 0),      # 2 rounds of 16 lanes per pixel, few tiles: sample mode
    (200, 60, 40, 8, 3),      # 3 rounds, the last one partial, frame offset
    (1280, 720, 32, 8, 0),    # rank 0's shard of 8 at N x spp, as bench --gpus 8 renders it
])
def test_many_frames_sample_mode_vs_oracle(gpu, case):
    """More frames per pixel than lanes per pixel on few pixels runs in sample mode
    (one task per tile and round, frame planes merged afterwards): same bits as the
    oracle's serial per-pixel loop."""
    w, h, frames, depth, f0 = case
    if w == 1280:   # row-block-cyclic shard 0 of 8, blocks of 8 rows
        rows = [y for y in range(h) if (y // 8) % 8 == 0]
        job = gpu.Job(width=w, height=h, frame0=f0, frames=frames, max_depth=depth, row_block=8, row_period=8,
                      row_phase=0)
        buf = np.zeros((len(rows), w, 4), np.float32)
        rays = gpu.render_host(job, buf)
        yc = 24   # check the first three row blocks against the oracle (the rest is the same code)
        want = np.concatenate([oracle.orc_render(w, h, frames, depth, frame0=f0, y0=y, yc=1)[0] for y in rows[:yc]])
        _assert_bitwise(buf[:yc], want[..., :3], f"shard of 8 at {frames} spp")
        assert rays > 0
        return
    buf, rays = _render(gpu, w, h, frames, depth, frame0=f0)
    want, wrays = oracle.orc_render(w, h, frames, depth, frame0=f0)
    _assert_bitwise(buf, want[..., :3], f"{case}")
    assert rays == wrays


EDGE_CASES = {
    "1x1": (1, 1, 3, 8, 0),
    "1x37": (1, 37, 2, 8, 0),
    "37x1": (37, 1, 5, 8, 0),
    "131x3": (131, 3, 4, 8, 0),
    "depth0": (64, 36, 2, 0, 0),           # no scatter event: every hit is its own emissive
    "depth1": (64, 36, 2, 1, 0),
    "depth64": (48, 27, 2, 64, 0),          # the deepest supported budget
    "lerp_table_edge": (64, 36, 4, 8, 65534),  # frames 65534..65537 cross the host-divided table
    "seed_wrap": (64, 36, 2, 8, 3000000),   # f * 26699 wraps uint32 as in the reference seed
    "frames17": (40, 20, 17, 8, 0),         # a 16-lane split plus one frame
}


@pytest.mark.parametrize("kflags", [0, V0, WF, POOL], ids=["auto", "v0", "wavefront", "pool"])
@pytest.mark.parametrize("case", list(EDGE_CASES), ids=list(EDGE_CASES))
def test_edge_cases_vs_oracle(gpu, case, kflags):
    """Degenerate sizes, depth budgets 0/1/64, frame numbers at the lerp table's end and
    past the seed's uint32 wrap, odd frame counts: bits and rays equal the oracle."""
    w, h, frames, depth, f0 = EDGE_CASES[case]
    buf, rays = _render(gpu, w, h, frames, depth, frame0=f0, flags=kflags)
    want, wrays = oracle.orc_render(w, h, frames, depth, frame0=f0)
    _assert_bitwise(buf, want[..., :3], f"{case} flags={kflags}")
    assert rays == wrays


@pytest.mark.parametrize("f0,frames", [(0, 3), (5, 3), (0, 40)])   # 40: few pixels, many frames
def test_non_finite_prev_propagates_like_reference(gpu, f0, frames):
    """The lerp reads prev even at frame 0 (prev * 0 + col, parallel.cpp:282): NaN, +-inf
    and huge values in the caller's buffer propagate exactly as in the reference. NaNs are
    compared as NaN (their payload bits are platform-defined)."""
    w, h = 48, 20
    rng = np.random.default_rng(7)
    init = rng.uniform(0, 2, (h, w, 4)).astype(np.float32)
    specials = np.array([np.nan, np.inf, -np.inf, 3.0e38, -3.0e38, 0.0, -0.0], np.float32)
    mask = rng.random((h, w, 3)) < 0.3
    init[..., :3][mask] = rng.choice(specials, int(mask.sum()))
    got = init.copy()
    want = init.copy()
    rays = gpu.render_host(gpu.Job(width=w, height=h, frame0=f0, frames=frames, max_depth=8), got)
    _, wrays = oracle.orc_render(w, h, frames, 8, frame0=f0, buf=want)
    assert rays == wrays
    g, e = got[..., :3], want[..., :3]
    same = (g.view(np.uint32) == e.view(np.uint32)) | (np.isnan(g) & np.isnan(e))
    assert same.all(), f"{int((~same).sum())} channels differ"
    assert np.isnan(g).sum() >= int(np.isnan(init[..., :3]).sum())
    assert np.array_equal(got[..., 3].view(np.uint32), init[..., 3].view(np.uint32))


GRID = 2048   # LRT_F_GRID: the uniform grid, also for scenes the policy leaves on the linear scan


@pytest.mark.parametrize("kflags", [V0, POOL], ids=["v0", "pool"])
def test_grid_on_small_scenes_vs_oracle(gpu, manifest, images, kflags):
    """The grid forced on the reference's own 9 spheres (configs 1-3) and the fuzzed scenes
    (9 spheres each, 1-3 lights, every material): the same bits as the scan's goldens."""
    from learnraytracing_amd import _lib as L
    from learnraytracing_amd.scene import scene_from_arrays
    buf, rays = _render(gpu, 1280, 720, 4, 8, flags=kflags | GRID)
    info = L.last_launch()
    assert info["acc"] == "grid", info
    want, wrays = oracle.orc_render(1280, 720, 4, 8)
    _assert_bitwise(buf, want[..., :3], f"flags={kflags | GRID} config2 full frame")
    assert rays == wrays
    buf, rays = _render(gpu, 1920, 1080, 16, 50, y0=520, yc=24, flags=kflags | GRID)
    want, wrays = oracle.orc_render(1920, 1080, 16, 50, y0=520, yc=24)
    _assert_bitwise(buf, want[..., :3], f"flags={kflags | GRID} config3 band")
    assert rays == wrays
    try:
        for fz in manifest["fuzz"]:
            gpu.set_scene(*scene_from_arrays(fz["spheres"], fz["mats"]))
            cam = L.Camera()
            vals = fz["camera"]
            names = ("origin", "a", "u", "r", "lowerLeftCorner", "horizontalVec", "verticalVec")
            for i, n in enumerate(names):
                setattr(cam, n, L.f3(*vals[3 * i:3 * i + 3]))
            cam.lensRadius = vals[21]
            buf, rays = _render(gpu, fz["w"], fz["h"], fz["frames"], fz["max_depth"], camera=cam,
                                flags=kflags | GRID)
            _assert_bitwise(buf, images[fz["name"]], f"flags={kflags | GRID} " + fz["name"])
            assert rays == fz["rays"], fz["name"]
    finally:
        gpu.set_scene(*gpu.default_scene())


def test_pool_scratch_over_more_streams_than_slots(gpu):
    """The pool kernel keeps per-stream scratch in 8 slots; rendering on 11 streams in rotation
    (twice round) takes slots over from other streams -- in stream order, behind an event of the
    previous owner's last launch, with no device-wide sync (advisor r5) -- and every render
    still gives the one-stream bits."""
    import torch

    from learnraytracing_amd import _lib as L
    w, h, frames, depth = 1280, 720, 4, 8
    want = np.zeros((h, w, 4), np.float32)
    want_rays = gpu.render_host(gpu.Job(width=w, height=h, frames=frames, max_depth=depth), want)
    streams = [torch.cuda.Stream() for _ in range(11)]
    bufs = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(2 * len(streams))]
    rays = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in bufs]
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)   # the zero fills come first
    job = gpu.Job(width=w, height=h, frames=frames, max_depth=depth)
    for i, b in enumerate(bufs):
        gpu.render_tensor(job, b, rays[i], streams[i % len(streams)])
        assert L.last_launch()["kernel"] == "pool_kernel"
    torch.cuda.synchronize()
    for i, b in enumerate(bufs):
        _assert_bitwise(b.cpu().numpy(), want[..., :3], f"render {i} on stream {i % len(streams)}")
        assert int(rays[i].item()) == want_rays
