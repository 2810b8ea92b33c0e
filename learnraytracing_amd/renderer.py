"""Host-side mirror of the reference renderer API (src/cpu/parallel.h:6-8) over the
C-ABI, plus the device-resident render used by the benchmark and the multi-GPU path.

Reference API (same names, same argument meaning):
    InitializeTest()                                  parallel.cpp:231-235
    ShutdownTest()                                    parallel.cpp:237-240
    DrawTest(time, frameCount, screenWidth, screenHeight, backbuffer) -> rayCount
                                                      parallel.cpp:297-323
`backbuffer` is a float32 array of screenWidth*screenHeight*4 (RGBA stride, row 0 at
the bottom); DrawTest adds one progressive sample per pixel exactly as the reference's
TraceRowJob does (kMaxDepth 20), but every pixel-sample owns its XorShift32 stream
(seed (x*1973 + y*9277 + frameCount*26699) | 1) instead of the reference's shared,
racy global one (maths.cpp:5), so the output is deterministic.

Error behaviour: the reference returns void and has no argument checks (bad sizes are
undefined behaviour). Here every failure raises LrtError with the library's message.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib as L


# ---- the reference API ---------------------------------------------------------------
def InitializeTest() -> None:
    L.check(L.lib().lrt_initialize())


def ShutdownTest() -> None:
    L.check(L.lib().lrt_shutdown())


def InitializeDevices(device_ids: Optional[Sequence[int]] = None, peer_copy: bool = False,
                      gather: bool = False) -> None:
    """InitializeTest over several GPUs of this process (lrt_initialize_devices): DrawTest and
    render_host then split the rows over all of them; each device copies its rows back to the
    caller's buffer itself, or with gather=True they are gathered into the first device by RCCL
    (device-to-device copies when an id repeats, or with peer_copy). None: every visible GPU."""
    flags = (L.DEV_PEER_COPY if peer_copy else 0) | (L.DEV_GATHER if gather else 0)
    if device_ids is None:
        L.check(L.lib().lrt_initialize_devices(0, None, flags))
        return
    ids = (ctypes.c_int * len(device_ids))(*[int(i) for i in device_ids])
    L.check(L.lib().lrt_initialize_devices(len(device_ids), ctypes.cast(ids, ctypes.c_void_p), flags))


def device_count() -> int:
    return int(L.lib().lrt_device_count())


def DrawTest(time: float, frameCount: int, screenWidth: int, screenHeight: int,
             backbuffer: np.ndarray) -> int:
    """The reference's DrawTest (parallel.h:8): one progressive frame into the caller's
    float RGBA backbuffer (any host memory; a pageable array is page-locked for the call
    only). Returns the rays counted (outRayCount)."""
    _check_host_buffer(backbuffer, screenWidth * screenHeight * 4)
    rays = ctypes.c_int(0)
    L.check(L.lib().lrt_draw_test(float(time), int(frameCount), int(screenWidth), int(screenHeight),
                                  backbuffer.ctypes.data_as(ctypes.c_void_p), ctypes.byref(rays)))
    return rays.value


# ---- extended API -----------------------------------------------------------------------
def default_camera(width: int, height: int) -> L.Camera:
    cam = L.Camera()
    L.check(L.lib().lrt_camera_default(int(width), int(height), ctypes.byref(cam)))
    return cam


def make_camera(look_from, look_at, vup, vfov, aspect, aperture, focus_dist) -> L.Camera:
    cam = L.Camera()
    L.check(L.lib().lrt_camera_make(L.f3(*look_from), L.f3(*look_at), L.f3(*vup), float(vfov),
                                    float(aspect), float(aperture), float(focus_dist), ctypes.byref(cam)))
    return cam


def set_scene(spheres: Sequence[L.Sphere], materials: Sequence[L.Material]) -> None:
    n = len(spheres)
    if n != len(materials):
        raise L.LrtError(L.LRT_E_INVALID, "spheres and materials differ in length")
    sa = (L.Sphere * max(n, 1))(*spheres)
    ma = (L.Material * max(n, 1))(*materials)
    L.check(L.lib().lrt_set_scene(sa, ma, n))


def get_scene():
    """(spheres, materials) the devices hold now (lrt_get_scene)."""
    n = ctypes.c_int(0)
    rc = L.lib().lrt_get_scene(None, None, 0, ctypes.byref(n))
    if rc != 0 and n.value == 0:
        L.check(rc)
    sa = (L.Sphere * max(n.value, 1))()
    ma = (L.Material * max(n.value, 1))()
    L.check(L.lib().lrt_get_scene(sa, ma, n.value, ctypes.byref(n)))
    return list(sa)[: n.value], list(ma)[: n.value]


def shard_rows(height: int, row_block: int, period: int, phase: int) -> int:
    return L.check(L.lib().lrt_shard_rows(int(height), int(row_block), int(period), int(phase)))


@dataclass
class Job:
    """One render call (lrt_render_desc). Rows are local; see include/lrt.h."""
    width: int
    height: int
    frame0: int = 0
    frames: int = 1
    max_depth: int = 8
    x0: int = 0
    x_count: Optional[int] = None
    y0: int = 0
    row_count: Optional[int] = None
    row_block: Optional[int] = None
    row_period: int = 1
    row_phase: int = 0
    camera: Optional[L.Camera] = None
    flags: int = 0

    def desc(self) -> L.RenderDesc:
        d = L.RenderDesc()
        d.camera = self.camera if self.camera is not None else default_camera(self.width, self.height)
        d.width, d.height = self.width, self.height
        d.x0 = self.x0
        d.x_count = self.width - self.x0 if self.x_count is None else self.x_count
        d.y0 = self.y0
        rb = self.row_block if self.row_block is not None else max(1, self.height)
        d.row_block, d.row_period, d.row_phase = rb, self.row_period, self.row_phase
        if self.row_count is None:
            if self.row_period == 1:
                d.row_count = self.height - self.y0
            else:
                d.row_count = shard_rows(self.height - self.y0, rb, self.row_period, self.row_phase)
        else:
            d.row_count = self.row_count
        d.frame0, d.frames, d.max_depth, d.flags = self.frame0, self.frames, self.max_depth, self.flags
        return d


def pinned_backbuffer(n_floats: int) -> np.ndarray:
    """A zeroed float32 host array in page-locked memory (a torch pin_memory tensor viewed
    by numpy; the array keeps the tensor alive). DrawTest / render_host detect such buffers:
    the colours are rendered while the previous values come in by DMA, and the lerp writes
    the result straight into the buffer over PCIe (LRT_HOST_PIPELINE=0: the kernel reads and
    writes the buffer in place; LRT_HOST_ZEROCOPY=0: staged like pageable memory)."""
    import torch
    return torch.zeros(int(n_floats), dtype=torch.float32, pin_memory=True).numpy()


def render_host(job: Job, backbuffer: np.ndarray) -> int:
    """Render `job` into a host float32 buffer (row_count*x_count*4). Returns rays."""
    d = job.desc()
    _check_host_buffer(backbuffer, d.row_count * d.x_count * 4)
    rays = ctypes.c_longlong(0)
    L.check(L.lib().lrt_render_host(ctypes.byref(d), backbuffer.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.byref(rays)))
    return rays.value


def render_host_features(job: Job, backbuffer: np.ndarray, features: dict, max_frame: int = 4) -> int:
    """render_host plus the GL path's first-hit features (lrt_render_host_ex): `features`
    maps names of lrt_features ("normal", "world_pos", "albedo", "color_std", "normal_std",
    "world_pos_std") to host float32 buffers shaped like the backbuffer, updated in place
    for frames <= max_frame (< 0: all). Returns rays."""
    d = job.desc()
    n = d.row_count * d.x_count * 4
    _check_host_buffer(backbuffer, n)
    f = L.Features()
    f.max_frame = int(max_frame)
    for name, buf in features.items():
        if name not in L.FEATURE_NAMES:
            raise L.LrtError(L.LRT_E_INVALID, f"unknown feature {name!r}")
        _check_host_buffer(buf, n)
        setattr(f, name, buf.ctypes.data)
    rays = ctypes.c_longlong(0)
    L.check(L.lib().lrt_render_host_ex(ctypes.byref(d), backbuffer.ctypes.data_as(ctypes.c_void_p),
                                       ctypes.byref(rays), ctypes.byref(f)))
    return rays.value


def render_device(job: Job, buf_ptr: int, rays_ptr: int, stream_ptr: int = 0) -> None:
    """Asynchronous render into device memory (raw pointers, e.g. torch's data_ptr())."""
    d = job.desc()
    L.check(L.lib().lrt_render_device(ctypes.byref(d), ctypes.c_void_p(buf_ptr), ctypes.c_void_p(rays_ptr),
                                      ctypes.c_void_p(stream_ptr)))


def render_tensor(job: Job, buf, rays, stream=None) -> None:
    """torch front end of render_device: buf is a cuda float32 tensor with
    row_count*x_count*4 elements, rays a cuda int64 tensor with >= 1 element
    (incremented by the counted rays), stream a torch.cuda.Stream (default: current)."""
    import torch

    d = job.desc()
    need = d.row_count * d.x_count * 4
    if not (buf.is_cuda and buf.dtype == torch.float32 and buf.is_contiguous() and buf.numel() >= need):
        raise L.LrtError(L.LRT_E_INVALID, f"buf must be a contiguous cuda float32 tensor of >= {need} elements")
    if not (rays.is_cuda and rays.dtype == torch.int64 and rays.numel() >= 1):
        raise L.LrtError(L.LRT_E_INVALID, "rays must be a cuda int64 tensor")
    s = stream if stream is not None else torch.cuda.current_stream(buf.device)
    L.check(L.lib().lrt_render_device(ctypes.byref(d), ctypes.c_void_p(buf.data_ptr()),
                                      ctypes.c_void_p(rays.data_ptr()), ctypes.c_void_p(s.cuda_stream)))


def render_tensor_to_frame(job: Job, buf, rays, frame_ptr: int, stream=None) -> None:
    """render_tensor plus the fused frame exchange (lrt_render_device_to_frame): each finished
    pixel is also stored into the width x height RGBA frame at frame_ptr (a device pointer,
    e.g. rank 0's frame opened over IPC) at its global row."""
    import torch

    d = job.desc()
    need = d.row_count * d.x_count * 4
    if not (buf.is_cuda and buf.dtype == torch.float32 and buf.is_contiguous() and buf.numel() >= need):
        raise L.LrtError(L.LRT_E_INVALID, f"buf must be a contiguous cuda float32 tensor of >= {need} elements")
    if not (rays.is_cuda and rays.dtype == torch.int64 and rays.numel() >= 1):
        raise L.LrtError(L.LRT_E_INVALID, "rays must be a cuda int64 tensor")
    s = stream if stream is not None else torch.cuda.current_stream(buf.device)
    L.check(L.lib().lrt_render_device_to_frame(ctypes.byref(d), ctypes.c_void_p(buf.data_ptr()),
                                               ctypes.c_void_p(rays.data_ptr()), ctypes.c_void_p(int(frame_ptr)),
                                               ctypes.c_void_p(s.cuda_stream)))


class RenderStream:
    """A CU-masked render stream (lrt_stream_create) leaving `reserved_cus` CUs free for
    concurrent work such as RCCL collectives; `.torch` is the torch.cuda.ExternalStream."""

    def __init__(self, reserved_cus: int):
        import torch

        h = ctypes.c_void_p()
        L.check(L.lib().lrt_stream_create(int(reserved_cus), ctypes.byref(h)))
        self.handle = h.value
        self.torch = torch.cuda.ExternalStream(self.handle)

    def close(self) -> None:
        if self.handle:
            L.check(L.lib().lrt_stream_destroy(ctypes.c_void_p(self.handle)))
            self.handle = None


def unshard_tensor(gathered, out, width: int, height: int, row_block: int, period: int, stream=None) -> None:
    """Frame assembly (lrt_unshard_rows) on cuda tensors."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream(out.device)
    L.check(L.lib().lrt_unshard_rows(ctypes.c_void_p(gathered.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     int(width), int(height), int(row_block), int(period),
                                     ctypes.c_void_p(s.cuda_stream)))


def pack_rgb_tensor(rgba, rgb, stream=None) -> None:
    """RGBA quads -> packed RGB triples (lrt_pack_rgb) on cuda tensors: the shard a rank
    sends in the frame exchange."""
    import torch

    if rgba.numel() // 4 != rgb.numel() // 3:
        raise ValueError("pack_rgb: rgba and rgb must hold the same pixels")
    s = stream if stream is not None else torch.cuda.current_stream(rgba.device)
    L.check(L.lib().lrt_pack_rgb(ctypes.c_void_p(rgba.data_ptr()), ctypes.c_void_p(rgb.data_ptr()),
                                 int(rgba.numel() // 4), ctypes.c_void_p(s.cuda_stream)))


def unshard_rgb_tensor(gathered_rgb, out, width: int, height: int, row_block: int, period: int, stream=None) -> None:
    """Frame assembly from packed RGB shards (lrt_unshard_rows_rgb); out's alpha untouched."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream(out.device)
    L.check(L.lib().lrt_unshard_rows_rgb(ctypes.c_void_p(gathered_rgb.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                         int(width), int(height), int(row_block), int(period),
                                         ctypes.c_void_p(s.cuda_stream)))


def present_tensor(rgba, bgra, width: int, height: int, stream=None) -> None:
    """LinearToSRGB + BGRA8 pack (main.cpp:109-141) on cuda tensors."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream(rgba.device)
    L.check(L.lib().lrt_present_bgra8(ctypes.c_void_p(rgba.data_ptr()), ctypes.c_void_p(bgra.data_ptr()),
                                      int(width), int(height), ctypes.c_void_p(s.cuda_stream)))


def _check_host_buffer(buf: np.ndarray, n: int) -> None:
    if not isinstance(buf, np.ndarray) or buf.dtype != np.float32 or not buf.flags.c_contiguous or buf.size < n:
        raise L.LrtError(L.LRT_E_INVALID, f"backbuffer must be a C-contiguous float32 array of >= {n} elements")
