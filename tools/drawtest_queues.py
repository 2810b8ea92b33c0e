#!/usr/bin/env python3
"""DrawTest's rate against the HIP streams created before the library's own (HIP deals a
process's streams to its hardware queues in turn, GPU_MAX_HW_QUEUES = 4): N extra streams
first, then lrt_initialize and 300 pageable DrawTest frames; then shutdown + initialize again.
    python tools/drawtest_queues.py N"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import learnraytracing_amd as lrt  # noqa: E402
from learnraytracing_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 0
hip = ctypes.CDLL("libamdhip64.so")
extra = []
for _ in range(n):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    extra.append(s)
W, H, N = 1280, 720, 300
bb = np.zeros(W * H * 4, np.float32)


def rate(what):
    for f in range(2):
        lrt.DrawTest(0.0, f, W, H, bb)
    t0 = time.perf_counter()
    ts, hits = [], 0
    for f in range(2, 2 + N):
        t1 = time.perf_counter()
        lrt.DrawTest(0.0, f, W, H, bb)
        ts.append(time.perf_counter() - t1)
        hits += L.last_launch().get("lookahead") == "hit"
    dt = (time.perf_counter() - t0) / N
    q = np.percentile(np.array(ts) * 1e3, [10, 50, 90])
    print(f"streams before: {n}  {what:12s} {dt * 1e3:.4f} ms/frame  p10/50/90 {q[0]:.3f}/{q[1]:.3f}/{q[2]:.3f}  "
          f"look-ahead hits {hits}/{N}  {L.last_launch().get('host')}", flush=True)


lrt.InitializeTest()
rate("first init")
lrt.ShutdownTest()
lrt.InitializeTest()
rate("re-init")
lrt.ShutdownTest()
