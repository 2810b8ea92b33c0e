#!/usr/bin/env python3
"""Why bench.py's DrawTest leg (0.57-0.59 ms/frame) runs slower than tools/drawtest_rate.py
(0.50-0.52) on the same box: DrawTest timed alone, then again after each thing the bench does
before its leg (config-2 renders on torch streams, pinned torch host buffers, a scene upload,
lrt_initialize_devices / shutdown)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import learnraytracing_amd as lrt  # noqa: E402
from learnraytracing_amd import _lib as L  # noqa: E402

W, H, N = 1280, 720, int(sys.argv[1]) if len(sys.argv) > 1 else 200
torch.cuda.set_device(0)
lrt.InitializeTest()
bb = np.zeros(W * H * 4, np.float32)
frame = [0]


def rate(what):
    for _ in range(2):
        lrt.DrawTest(0.0, frame[0], W, H, bb)
        frame[0] += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        lrt.DrawTest(0.0, frame[0], W, H, bb)
        frame[0] += 1
    dt = (time.perf_counter() - t0) / N
    print(f"{what:48s} {dt * 1e3:.4f} ms/frame  {L.last_launch().get('host')}", flush=True)


rate("alone")
rate("alone again")
job = lrt.Job(width=1280, height=720, frame0=0, frames=4, max_depth=8)
bufs = [torch.zeros((720, 1280, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
rays = torch.zeros(1, dtype=torch.int64, device="cuda")
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
for k in range(40):
    lrt.render_tensor(job, bufs[k % 2], rays, streams[k % 2])
torch.cuda.synchronize()
rate("after 40 config-2 renders on two torch streams")
host = [torch.empty((720, 1280, 4), dtype=torch.float32, pin_memory=True) for _ in range(2)]
for k in range(4):
    host[k % 2].copy_(bufs[k % 2], non_blocking=True)
torch.cuda.synchronize()
rate("after pinned torch host buffers + D2H")
lrt.set_scene(*lrt.default_scene())
rate("after a scene upload")
del host
torch.cuda.synchronize()
rate("after freeing the pinned buffers")
lrt.ShutdownTest()

# bench.py's own leg, in this process (its numbers are the bench line's)
import bench  # noqa: E402

lrt.InitializeTest()
for k in range(2):
    print("bench.drawtest_leg", bench.drawtest_leg(lrt)["ms_per_frame"], flush=True)
rate("rate() after the bench leg")
lrt.ShutdownTest()
