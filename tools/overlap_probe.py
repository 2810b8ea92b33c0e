#!/usr/bin/env python3
"""Does work on another stream run beside the persistent render kernel? Launch a config-2
render on the render stream, then (after a short host delay) a device copy of COPY_MB on a
second stream, and report when each finished, with and without a CU-reserved render
stream (lrt_stream_create). Stands in for the RCCL gather of bench.py --gpus N, which
cannot run on one GPU.   python tools/overlap_probe.py [reserved ...]"""
import sys
import time

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import learnraytracing_amd as lrt
from learnraytracing_amd.renderer import RenderStream

COPY_MB = 16


def probe(reserved):
    rs = RenderStream(reserved) if reserved else None
    rstream = rs.torch if rs else torch.cuda.Stream()
    other = torch.cuda.Stream()
    job = lrt.Job(width=1280, height=720, frame0=0, frames=32, max_depth=8)   # ~3 ms: host launch latency negligible
    buf = torch.zeros((720, 1280, 4), device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    src = torch.ones(COPY_MB * 1024 * 256, device="cuda")
    dst = torch.empty_like(src)
    for _ in range(3):
        lrt.render_tensor(job, buf, rays, rstream)
        with torch.cuda.stream(other):
            torch.mul(src, 2.0, out=dst)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    r1 = torch.cuda.Event(enable_timing=True)
    c0 = torch.cuda.Event(enable_timing=True)
    c1 = torch.cuda.Event(enable_timing=True)
    t0.record(rstream)
    lrt.render_tensor(job, buf, rays, rstream)
    r1.record(rstream)
    time.sleep(0.0005)
    with torch.cuda.stream(other):
        other.wait_event(t0)
        c0.record(other)
        torch.mul(src, 2.0, out=dst)
        c1.record(other)
    torch.cuda.synchronize()
    if rs:
        rs.close()
    return t0.elapsed_time(r1), t0.elapsed_time(c0), t0.elapsed_time(c1)


def main():
    lrt.InitializeTest()
    for r in [int(a) for a in sys.argv[1:]] or [0, 8]:
        render_ms, c0, c1 = probe(r)
        print(f"reserved {r:3d}: render ends {render_ms:.3f} ms; other stream: kernel queued at {c0:.3f} ms, done at {c1:.3f} ms")
    lrt.ShutdownTest()


if __name__ == "__main__":
    main()
