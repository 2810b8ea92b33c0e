#!/usr/bin/env python3
"""The reference API's own throughput: DrawTest(time, frame, 1280, 720, backbuffer) per frame
(host buffer; H2D + D2H of the frame inside every call, kMaxDepth 20; argv[2] "pinned":
a page-locked backbuffer, which the kernel reads and writes in place over PCIe), the way
src/cpu/main.cpp:151-194 measures it (Mrays/s = rays per frame / seconds per frame)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import learnraytracing_amd as lrt

w, h, frames = 1280, 720, int(sys.argv[1]) if len(sys.argv) > 1 else 30
pinned = len(sys.argv) > 2 and sys.argv[2] == "pinned"
if "torch" in sys.argv[2:]:   # as bench.py's process: torch imported, its HIP context up
    import torch
    torch.zeros(1, device="cuda").sum().item()
lrt.InitializeTest()
bb = lrt.pinned_backbuffer(w * h * 4) if pinned else np.zeros(w * h * 4, np.float32)
lrt.DrawTest(0.0, 0, w, h, bb)  # warm-up
t0 = time.perf_counter()
rays = 0
for f in range(1, frames + 1):
    rays += lrt.DrawTest(0.0, f, w, h, bb)
dt = time.perf_counter() - t0
s = dt / frames
print(f"DrawTest host path ({'pinned' if pinned else 'pageable'}): {s * 1e3:.2f}ms ({1 / s:.1f} FPS) {rays / dt * 1e-6:.1f}Mrays/s "
      f"{rays / frames * 1e-6:.2f}Mrays/frame frames {frames}")
lrt.ShutdownTest()
