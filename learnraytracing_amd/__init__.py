"""learnraytracing_amd — MI355X-native drop-in for the per-pixel path tracer of
Sefaice/LearnRayTracing's src/cpu renderer (TraceRowJob -> Trace -> HitWorld/HitSphere
-> Scatter -> progressive backbuffer), as a hand-written HIP megakernel for gfx950
behind the C-ABI of include/lrt.h.

Python is the host-side mirror of the reference API; the compute path is
liblrt_hip.so only (no CPU fallback).
"""
from ._lib import LrtError, lib  # noqa: F401
from .renderer import (DrawTest, InitializeDevices, InitializeTest, Job, ShutdownTest,  # noqa: F401
                       default_camera, device_count, make_camera, pinned_backbuffer,
                       get_scene, render_device, render_host, render_host_features, render_tensor,
                       render_tensor_to_frame, set_scene, shard_rows)
from .scene import default_scene, random_scene  # noqa: F401

__version__ = "0.3.0"
