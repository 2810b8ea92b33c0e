#!/usr/bin/env python3
"""First launches of a view at config 2 (1280x720, 4 spp, 8 bounces): each launch timed alone
with HIP events on its stream, and the tile order it ran with (lrt_last_launch `order`:
0 queue order, 1 recording, 2 own sorted order, 3 borrowed from the same geometry).

    python tools/first_launch.py
"""
import sys

sys.path.insert(0, ".")
import torch

import learnraytracing_amd as lrt
from learnraytracing_amd import _lib as L

w, h = 1280, 720
lrt.InitializeTest()
buf = torch.zeros(h * w * 4, dtype=torch.float32, device="cuda")
rays = torch.zeros(1, dtype=torch.int64, device="cuda")
s = torch.cuda.Stream()


def launch(job, tag):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    lrt.render_tensor(job, buf, rays, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    info = L.last_launch()
    print(f"{tag:28s} {e0.elapsed_time(e1):7.3f} ms  kernel={info.get('kernel')} order={info.get('order')}", flush=True)


view_a = lrt.Job(width=w, height=h, frames=4, max_depth=8)
for k in range(4):
    launch(view_a, f"view A launch {k}")
for i, dx in enumerate((0.3, 0.6, 0.9)):
    cam = lrt.make_camera((dx, 2.0 + 0.1 * i, 3), (0, 0, 0), (0, 1, 0), 60, w / h, 0.1, 3)
    job = lrt.Job(width=w, height=h, frames=4, max_depth=8, camera=cam)
    for k in range(3):
        launch(job, f"moved camera {i} launch {k}")
sph, mats = lrt.default_scene()
sph[2].center = L.f3(sph[2].center.x + 0.25, sph[2].center.y, sph[2].center.z)
lrt.set_scene(sph, mats)   # an edited scene: the same geometry key? (sphere count / kind)
for k in range(3):
    launch(view_a, f"edited scene launch {k}")
lrt.ShutdownTest()
