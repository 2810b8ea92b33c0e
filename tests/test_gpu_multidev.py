"""GPU tests of round 3's host-side additions, through the C-ABI:

* lrt_initialize_devices: one process splits a host render over several devices
  (row-block-cyclic); each device copies its rows back to the caller's buffer (the direct
  exchange, default) or the shards' RGB is gathered into the first -- by RCCL (ncclCommInitAll +
  grouped ncclGather, rccl.h:745) when the ids are distinct, by device-to-device copies when an
  id repeats. On a one-GPU box RCCL runs with one device; repeated ids rehearse 2-3 shards on
  GPU 0. Every frame must equal the one-device render / the oracle bit for bit
  (parallel.cpp:262,280-286 per pixel; the reference's dispatch over rows, :317-320).
* DrawTest keeps nothing of the caller's buffer between calls: a pageable buffer freed and
  remapped at the same address (main.cpp:40's `new float[]` replaced) renders exactly.
* the pool kernel's heaviest-first tile order on two streams at once (the bench's
  pipelining), on the exact benchmarked state (order=2), for a new camera (borrowed order),
  and on the full config-3 frame.
"""
import contextlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _bitwise(got, want, what):
    g = got[..., :3]
    w = np.ascontiguousarray(want[..., :3])
    if not np.array_equal(g.view(np.uint32), w.view(np.uint32)):
        d = np.abs(g.astype(np.float64) - w.astype(np.float64))
        raise AssertionError(f"{what}: {int((g != w).any(axis=-1).sum())} pixels differ, max |diff| {d.max():.3g}")


@contextlib.contextmanager
def devices(gpu, ids, peer_copy=False, gather=False):
    """Re-initialise the library over `ids` for the block, then back to lrt_initialize."""
    gpu.ShutdownTest()
    try:
        gpu.InitializeDevices(ids, peer_copy=peer_copy, gather=gather)
        yield
    finally:
        gpu.ShutdownTest()
        gpu.InitializeTest()


def _host(gpu, job, buf=None):
    d = job.desc()
    if buf is None:
        buf = np.zeros((d.row_count, d.x_count, 4), np.float32)
    rays = gpu.render_host(job, buf)
    return buf, rays


@pytest.mark.parametrize("ids,peer,gather,exchange", [
    ([0], False, False, "direct"), ([0, 0], False, False, "direct"), ([0, 0, 0], False, False, "direct"),
    ([0], False, True, "rccl"), ([0], True, False, "copy"), ([0, 0], False, True, "copy"),
    ([0, 0, 0], False, True, "copy")],
    ids=["direct-1", "direct-2", "direct-3", "rccl-1", "copy-1", "copy-2", "copy-3"])
def test_multidevice_render_host_equals_oracle(gpu, ids, peer, gather, exchange):
    from learnraytracing_amd import _lib as L
    w, h, frames, depth = 320, 180, 4, 8
    want, wrays = oracle.orc_render(w, h, frames, depth)
    prev = np.random.default_rng(1).uniform(0, 1, (h, w, 4)).astype(np.float32)
    want_prev, _ = oracle.orc_render(w, h, frames, depth, frame0=3, buf=prev.copy())
    with devices(gpu, ids, peer, gather):
        assert gpu.device_count() == len(ids)
        buf, rays = _host(gpu, gpu.Job(width=w, height=h, frames=frames, max_depth=depth))
        info = L.last_launch()
        assert info["devices"] == str(len(ids)) and info["exchange"] == exchange, info
        _bitwise(buf, want, f"{len(ids)} devices ({exchange})")
        assert rays == wrays
        # progressive: the previous values of every shard come from the caller's buffer;
        # alpha is carried through the exchange untouched
        b2 = prev.copy()
        _host(gpu, gpu.Job(width=w, height=h, frame0=3, frames=frames, max_depth=depth), b2)
        _bitwise(b2, want_prev, "progressive multi-device")
        assert np.array_equal(b2[..., 3].view(np.uint32), prev[..., 3].view(np.uint32))


@pytest.mark.parametrize("ids,gather", [([0], True), ([0, 0, 0], True), ([0, 0, 0], False)],
                         ids=["rccl-1", "copy-3", "direct-3"])
def test_multidevice_drawtest_window_bvh(gpu, ids, gather):
    """DrawTest (kMaxDepth 20) progressively, a window with odd sizes, and a BVH scene
    rendered over the devices: all equal the oracle."""
    from learnraytracing_amd.scene import random_scene, scene_arrays
    w, h = 200, 120
    want = np.zeros((h, w, 4), np.float32)
    for f in range(2):
        oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
    wwin, wwr = oracle.orc_render(97, 61, 3, 8, x0=5, xc=83, y0=7, yc=41)
    sph, mat = random_scene(300, 4)
    s, m = (np.array(v, np.float32) for v in scene_arrays(sph, mat))
    wbvh, wbr = oracle.orc_render(160, 90, 5, 8, spheres=s, mats=m)
    with devices(gpu, ids, gather=gather):
        bb = np.zeros(w * h * 4, np.float32)
        for f in range(2):
            assert gpu.DrawTest(0.0, f, w, h, bb) > 0
        _bitwise(bb.reshape(h, w, 4), want, "multi-device DrawTest")
        win, wr = _host(gpu, gpu.Job(width=97, height=61, frames=3, max_depth=8, x0=5, x_count=83, y0=7, row_count=41))
        _bitwise(win, wwin, "multi-device window")
        assert wr == wwr
        gpu.set_scene(sph, mat)   # every device gets the scene
        img, r = _host(gpu, gpu.Job(width=160, height=90, frames=5, max_depth=8))
        _bitwise(img, wbvh, "multi-device BVH scene")
        assert r == wbr


@pytest.mark.parametrize("gather", [False, True], ids=["direct", "gather"])
def test_multidevice_drawtest_1280x720_three_frames(gpu, gather):
    """The reference caller's own shape on two devices (GPU 0 twice on a one-GPU box):
    DrawTest at 1280x720, kMaxDepth 20, frames 0-2 into one pageable buffer, each frame's rows
    split over the devices -- equal to the oracle bit for bit, rays included."""
    from learnraytracing_amd import _lib as L
    w, h = 1280, 720
    want = np.zeros((h, w, 4), np.float32)
    wr = [oracle.orc_render(w, h, 1, 20, frame0=f, buf=want, threads=16)[1] for f in range(3)]
    with devices(gpu, [0, 0], gather=gather):
        bb = np.zeros(w * h * 4, np.float32)
        got = [gpu.DrawTest(0.0, f, w, h, bb) for f in range(3)]
        info = L.last_launch()
    assert info["devices"] == "2" and info["exchange"] == ("copy" if gather else "direct"), info
    assert got == wr
    _bitwise(bb.reshape(h, w, 4), want, "two-device DrawTest 1280x720")


def test_multidevice_caller_shard_stays_on_first_device(gpu):
    """A caller's own row-block-cyclic shard (row_period > 1) is not split again: device 0
    renders it, same rows as the oracle."""
    from learnraytracing_amd import _lib as L
    w, h, rb, period, phase = 160, 90, 8, 3, 2
    rows = [y for y in range(h) if (y // rb) % period == phase]
    want, _ = oracle.orc_render(w, h, 2, 8)
    with devices(gpu, [0, 0]):
        buf, _ = _host(gpu, gpu.Job(width=w, height=h, frames=2, max_depth=8, row_block=rb, row_period=period,
                                    row_phase=phase))
        assert "devices" not in L.last_launch()
    _bitwise(buf, want[rows], "caller shard")


def test_initialize_devices_validation(gpu):
    from learnraytracing_amd import _lib as L
    with pytest.raises(L.LrtError):          # already initialised (the session's lrt_initialize)
        gpu.InitializeDevices([0])
    gpu.ShutdownTest()
    try:
        for bad in ([99], [-1]):
            with pytest.raises(L.LrtError):
                gpu.InitializeDevices(bad)
        assert gpu.device_count() == 0
    finally:
        gpu.InitializeTest()
    assert gpu.device_count() == 1


def _mmap_frame(nbytes, at=None):
    """An anonymous mapping as a float32 array (MAP_FIXED at `at` when given): the way a C
    caller's large `new float[]` gets its pages, and the way freeing it and allocating another
    can return the same address."""
    import ctypes
    import mmap as _m
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    flags = _m.MAP_PRIVATE | _m.MAP_ANONYMOUS | (0x10 if at is not None else 0)   # 0x10: MAP_FIXED
    p = libc.mmap(at, nbytes, _m.PROT_READ | _m.PROT_WRITE, flags, -1, 0)
    assert p not in (None, ctypes.c_void_p(-1).value), "mmap failed"
    arr = np.ctypeslib.as_array((ctypes.c_float * (nbytes // 4)).from_address(p))
    return p, arr, lambda: libc.munmap(p, nbytes)


def test_drawtest_pageable_buffer_freed_and_remapped_at_same_address(gpu):
    """The drop-in contract (parallel.h:8): DrawTest keeps nothing of the caller's buffer
    between calls. Frames 0-1 go into pageable buffer A; the caller frees A and maps a new
    buffer B at the SAME address (munmap + mmap MAP_FIXED) holding A's values, and frames 2-3
    go into B: every frame equals the oracle's (a registration kept from A's calls would make
    the device read and write A's stale pages instead of B's). Each call page-locks the buffer
    for itself only (host=registered-pipelined) and both the remapped and a fresh buffer take
    that path at once."""
    from learnraytracing_amd import _lib as L
    w, h = 320, 180
    nbytes = w * h * 16
    want = np.zeros((h, w, 4), np.float32)
    p, a, free_a = _mmap_frame(nbytes)
    a[:] = 0.0
    paths = []
    for f in range(2):
        gpu.DrawTest(0.0, f, w, h, a)
        paths.append(L.last_launch().get("host"))
        oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
    _bitwise(a.reshape(h, w, 4), want, "buffer A")
    keep = a.copy()
    free_a()
    p2, b, free_b = _mmap_frame(nbytes, at=p)
    try:
        assert p2 == p, "the kernel did not reuse the address"
        b[:] = keep
        for f in range(2, 4):
            gpu.DrawTest(0.0, f, w, h, b)
            paths.append(L.last_launch().get("host"))
            oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
        _bitwise(b.reshape(h, w, 4), want, "buffer B at A's address")
    finally:
        free_b()
    assert paths == ["registered-pipelined"] * 4, paths


def _torch_render(gpu, job, stream, out):
    import torch
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    # `out` and `rays` were zero-filled on the current stream: the render on `stream` must come
    # after those fills (without this a fill could land after the render's stores)
    stream.wait_stream(torch.cuda.current_stream())
    gpu.render_tensor(job, out, rays, stream)
    return rays


def test_pool_order_two_streams_bitwise(gpu):
    """The bench's pipelining: config 2 launched alternately on two streams, each into its own
    buffer, across the recording launch and the switch to the heaviest-first order, with no
    host synchronisation in between: the order is sorted on the device behind the recording
    launch, the second launch (the other stream) records again in that order and sorts into the
    other permutation buffer (order=5), and every later launch, on either stream, waits for the
    latest sort's event. Every frame equals the single-stream render. A launch made while the
    other stream's is still running takes 128-px tiles (a signature, and an order, of its own):
    per tile size, the orders run recording -> refining (5) -> sorted (2)."""
    import torch
    from learnraytracing_amd import _lib as L
    w, h = 1280, 720
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(8)]
    orders, pix = [], []
    cam = gpu.make_camera((0.1, 2, 3), (0, 0, 0), (0, 1, 0), 60, w / h, 0.1, 3)   # a signature of its own
    job2 = gpu.Job(width=w, height=h, frames=4, max_depth=8, camera=cam)
    for k, o in enumerate(outs):
        _torch_render(gpu, job2, streams[k % 2], o)
        info = L.last_launch()
        orders.append(info["order"])
        pix.append(info["pix"])
    torch.cuda.synchronize()
    want, _ = oracle.orc_render(w, h, 4, 8, cam22=cam.to22())
    for k, o in enumerate(outs):
        _bitwise(o.cpu().numpy(), want, f"launch {k} (order {orders[k]})")
    for p in set(pix):
        seq = [o for o, q in zip(orders, pix) if q == p]
        assert seq[0] in ("1", "3", "4") and seq[1:2] in (["5"], []) and seq[2:] == ["2"] * (len(seq) - 2), \
            (orders, pix)
    assert set(pix) <= {"64", "128"} and "128" in pix, (orders, pix)   # the overlapping launches' tiles


def test_config2_benchmarked_state_vs_oracle(gpu):
    """The exact state bench.py times: config 2 through lrt_render_device after a recording
    launch, i.e. pool_kernel with the heaviest-first order (order=2), full frame, bit-exact."""
    import torch
    from learnraytracing_amd import _lib as L
    w, h = 1280, 720
    job = gpu.Job(width=w, height=h, frames=4, max_depth=8)
    s = torch.cuda.current_stream()
    warm = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
    for _ in range(2):   # the recording launch and the refining pass
        _torch_render(gpu, job, s, warm)
    torch.cuda.synchronize()
    out = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
    rays = _torch_render(gpu, job, s, out)
    info = L.last_launch()
    assert info["kernel"] == "pool_kernel" and info["order"] == "2" and info["ns"] == "9", info
    # a launch alone serves its lightest tiles as halves (the split tail, lrt_pool.h)
    assert int(info["split_from"]) < int(info["tasks"]), info
    torch.cuda.synchronize()
    want, wrays = oracle.orc_render(w, h, 4, 8)
    _bitwise(out.cpu().numpy(), want, "config 2, order=2")
    assert int(rays.item()) == wrays == 11669343


def test_new_view_borrows_order_bitwise(gpu):
    """A camera move keeps the geometry: its first launch borrows the previous view's ready
    order (order=3) instead of running in queue order; the pixels are the new view's."""
    from learnraytracing_amd import _lib as L
    w, h = 1280, 720
    # (flags 512: the pool kernel; a host buffer of <= 4 frames otherwise takes the pipelined
    # host path, whose colours v0 renders)
    for _ in range(3):   # view A: recording launch, the refining pass, then its own order
        _host(gpu, gpu.Job(width=w, height=h, frames=4, max_depth=8, flags=512))
    assert L.last_launch()["order"] == "2"
    cam = gpu.make_camera((0.3, 2.1, 3), (0, 0, 0), (0, 1, 0), 60, w / h, 0.1, 3)
    buf, rays = _host(gpu, gpu.Job(width=w, height=h, frames=4, max_depth=8, camera=cam, flags=512))
    assert L.last_launch()["order"] == "3"
    want, wrays = oracle.orc_render(w, h, 4, 8, cam22=cam.to22())
    _bitwise(buf, want, "moved camera, borrowed order")
    assert rays == wrays


def test_probe_ordered_first_launch_vs_oracle(gpu):
    """A geometry with no measured order yet (this window's shape is used by no other test):
    the first launch takes its tiles in the cost probe's order (probe_kernel +
    probe_order_kernel, order=4), the second in its own measured order while it records again
    (order=5), the third in the refined order; all are the restatement's pixels and ray count."""
    from learnraytracing_amd import _lib as L
    kw = dict(width=1280, height=720, frames=4, max_depth=8, x0=100, x_count=312, y0=200, row_count=104)
    want, wrays = oracle.orc_render(1280, 720, 4, 8, 0, 100, 312, 200, 104, threads=16)
    for order in ("4", "5", "2"):
        buf, rays = _host(gpu, gpu.Job(flags=512, **kw))
        info = L.last_launch()
        assert info["kernel"] == "pool_kernel" and info["order"] == order, info
        _bitwise(buf, want, f"order {order}")
        assert rays == wrays


def test_config3_full_frame_vs_oracle(gpu):
    """BASELINE config 3 at full size (1920x1080, 16 spp, 50 bounces, ~106 M rays) on the
    instance and order the benchmark runs (pool kernel, heaviest-first after a recording
    launch): bit-exact vs the C oracle."""
    from learnraytracing_amd import _lib as L
    job = gpu.Job(width=1920, height=1080, frames=16, max_depth=50)
    _host(gpu, job)   # the recording launch
    _host(gpu, job)   # the refining pass
    buf, rays = _host(gpu, job)
    info = L.last_launch()
    assert info["kernel"] == "pool_kernel" and info["maxd"] == "64" and info["order"] == "2", info
    want, wrays = oracle.orc_render(1920, 1080, 16, 50)
    _bitwise(buf, want, "config 3 full frame")
    assert rays == wrays


def test_drawtest_lookahead_hits_and_misses(gpu):
    """lrt_draw_test renders frame f + 1's colours behind call f: DrawTest's colours depend on
    frameCount, the size and the scene only (parallel.cpp:297-323; `time` is unused) and
    main.cpp:165,187 asks for frameCount + 1 next. A call continuing the sequence uses them
    (lookahead=hit); a repeated or skipped frame, a new size or a new scene renders for itself
    (miss). The oracle's bits and ray counts either way."""
    from learnraytracing_amd import _lib as L
    from learnraytracing_amd.scene import scene_arrays

    def run(seq, w, h, bb, want, spheres=None, mats=None):
        for f, expect in seq:
            rays = gpu.DrawTest(0.0, f, w, h, bb)
            ll = L.last_launch()
            assert ll.get("host") == "pipelined" and ll.get("lookahead") == expect, (f, ll)
            _, wr = oracle.orc_render(w, h, 1, 20, frame0=f, buf=want, spheres=spheres, mats=mats)
            assert rays == wr, (f, rays, wr)
            _bitwise(bb.reshape(h, w, 4), want, f"frame {f} ({expect})")

    w, h = 320, 180
    bb = gpu.pinned_backbuffer(w * h * 4)
    bb[:] = 0.0
    want = np.zeros((h, w, 4), np.float32)
    run([(0, "miss"), (1, "hit"), (2, "hit"), (2, "miss"), (3, "hit"), (7, "miss"), (8, "hit")], w, h, bb, want)
    w2, h2 = 200, 117   # a new size: its own look-ahead
    bb2 = gpu.pinned_backbuffer(w2 * h2 * 4)
    bb2[:] = 0.0
    want2 = np.zeros((h2, w2, 4), np.float32)
    run([(9, "miss"), (10, "hit")], w2, h2, bb2, want2)
    sph, mats = gpu.default_scene()
    sph[2].center = L.f3(sph[2].center.x + 0.25, sph[2].center.y, sph[2].center.z)
    gpu.set_scene(sph, mats)   # a new scene between frames 10 and 11: the look-ahead is stale
    try:
        s, m = scene_arrays(sph, mats)
        run([(11, "miss"), (12, "hit")], w2, h2, bb2, want2, spheres=s, mats=m)
    finally:
        gpu.set_scene(*gpu.default_scene())


def test_probe_order_many_tiles_equals_v0(gpu):
    """The probe's counting sort over more tiles than one pass of its workgroup holds
    (1920x704 at 64 px: 21,120 tiles > 16,384): the probe-ordered first launch renders every
    tile exactly once -- its pixels and ray count equal v0's render of the same frame."""
    from learnraytracing_amd import _lib as L
    kw = dict(width=1920, height=704, frames=4, max_depth=8)
    buf, rays = _host(gpu, gpu.Job(flags=512, **kw))
    info = L.last_launch()
    assert info["kernel"] == "pool_kernel" and info["order"] == "4" and int(info["tasks"]) > 16384, info
    want, wrays = _host(gpu, gpu.Job(flags=2, **kw))
    assert L.last_launch()["kernel"] == "trace_kernel"
    _bitwise(buf, want, "probe order over 21,120 tiles vs v0")
    assert rays == wrays


def test_pool_scratch_grows_and_is_reused_bitwise(gpu):
    """The pool kernel's colour slots and overflow stack live in a per-stream scratch buffer kept
    between launches (lrt_render.hip stream_scratch): a small window, then windows that need more
    (more waves' slots; a 20-bounce budget with overflow levels), then the small one again, all on
    one stream: every render is the restatement's."""
    import torch
    from learnraytracing_amd import _lib as L
    s = torch.cuda.Stream()
    cases = [dict(x0=0, x_count=320, y0=0, row_count=64, max_depth=8),
             dict(x0=0, x_count=1280, y0=0, row_count=360, max_depth=8),
             dict(x0=320, x_count=640, y0=100, row_count=200, max_depth=20),
             dict(x0=0, x_count=320, y0=0, row_count=64, max_depth=8)]
    for kw in cases:
        job = gpu.Job(width=1280, height=720, frames=4, flags=512, **kw)
        out = torch.zeros((kw["row_count"], kw["x_count"], 4), dtype=torch.float32, device="cuda")
        rays = _torch_render(gpu, job, s, out)
        info = L.last_launch()
        assert info["kernel"] == "pool_kernel", info
        s.synchronize()
        want, wrays = oracle.orc_render(1280, 720, 4, kw["max_depth"], 0, kw["x0"], kw["x_count"], kw["y0"],
                                        kw["row_count"], threads=16)
        _bitwise(out.cpu().numpy(), want, f"window {kw}")
        assert int(rays.item()) == wrays


def test_kernel_timing_events(gpu):
    """lrt_kernel_timing (lrt_diag.h): events right around each render kernel, read back in launch
    order; off again, nothing more is recorded."""
    import ctypes
    import torch
    from learnraytracing_amd import _lib as L
    s = torch.cuda.current_stream()
    job = gpu.Job(width=320, height=180, frames=4, max_depth=8)
    out = torch.zeros((180, 320, 4), dtype=torch.float32, device="cuda")
    L.check(L.lib().lrt_kernel_timing(1))
    for _ in range(3):
        _torch_render(gpu, job, s, out)
    ms = (ctypes.c_float * 8)()
    n = ctypes.c_int(-1)
    L.check(L.lib().lrt_kernel_times(ms, 8, ctypes.byref(n)))
    assert n.value == 3 and all(0.0 < ms[i] < 1000.0 for i in range(3)), (n.value, list(ms))
    L.check(L.lib().lrt_kernel_timing(0))
    _torch_render(gpu, job, s, out)
    L.check(L.lib().lrt_kernel_times(ms, 8, ctypes.byref(n)))
    assert n.value == 0
