"""Does a config-2 launch get faster as the GPU stays busy? (round 6, profiles/r6_c)

Times back-to-back regions of 20 pipelined config-2 steps (two streams, as bench.py) in one
process: right after 5 warmup steps, then region after region; then after 1 s of idle; then
after ~50 ms of other GPU work. Prints ms/step per region."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import learnraytracing_amd as lrt  # noqa: E402

torch.cuda.set_device(0)
lrt.InitializeTest()
W, H = 1280, 720
job = lrt.Job(width=W, height=H, frames=4, max_depth=8)
dev = torch.device("cuda", 0)
bufs = [torch.zeros((H, W, 4), dtype=torch.float32, device=dev) for _ in range(2)]
rays = torch.zeros(1, dtype=torch.int64, device=dev)
s0 = torch.cuda.current_stream(dev)
streams = [s0, torch.cuda.Stream(device=dev)]
streams[1].wait_stream(s0)


import ctypes  # noqa: E402
import os  # noqa: E402
_cp = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libclock_probe.so"))
_cbuf = torch.zeros(2 * 256, dtype=torch.int64, device=dev)


def mhz():
    """The shader clock right now: 256 one-wave blocks spinning 200k cycles (clock_probe.hip)."""
    m = ctypes.c_double(0)
    torch.cuda.synchronize()
    assert _cp.clock_probe_mhz(ctypes.c_void_p(s0.cuda_stream), ctypes.c_void_p(_cbuf.data_ptr()), 256,
                               ctypes.byref(m)) == 0
    return m.value


def region(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        lrt.render_tensor(job, bufs[i % 2], rays, streams[i % 2])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for i in range(5):
    lrt.render_tensor(job, bufs[i % 2], rays, streams[i % 2])
print("clock before the first render (MHz):", f"{mhz():.0f}", flush=True)
print("after 5 warmup steps:", " ".join(f"{region(20):.4f}" for _ in range(12)), flush=True)
print("clock now:", f"{mhz():.0f}", flush=True)
print("region / clock pairs:", " ".join(f"{region(20):.4f}@{mhz():.0f}" for _ in range(6)), flush=True)
time.sleep(1.0)
print("clock after 1 s idle:", f"{mhz():.0f}", flush=True)
print("after 1 s idle:      ", " ".join(f"{region(20):.4f}@{mhz():.0f}" for _ in range(8)), flush=True)
time.sleep(1.0)
a = torch.randn(4096, 4096, device=dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.05:
    a = a @ a.T
    a = a / a.norm()
torch.cuda.synchronize()
print("after 50 ms of GEMMs:", " ".join(f"{region(20):.4f}" for _ in range(12)), flush=True)
print("one region of 200:   ", f"{region(200):.4f}", flush=True)
# what warms it: 50 ms of HBM traffic (1-GB copies), or 50 ms of VALU spinning on every CU
time.sleep(1.0)
big = torch.empty(256 << 20, dtype=torch.float32, device=dev)
big2 = torch.empty_like(big)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.05:
    big2.copy_(big)
    torch.cuda.synchronize()
print("after 50 ms of copies:", " ".join(f"{region(20):.4f}" for _ in range(6)), flush=True)
del big, big2
time.sleep(1.0)
t0 = time.perf_counter()
m = ctypes.c_double(0)
while time.perf_counter() - t0 < 0.05:
    _cp.clock_probe_mhz(ctypes.c_void_p(s0.cuda_stream), ctypes.c_void_p(_cbuf.data_ptr()), 256, ctypes.byref(m))
print("after 50 ms of VALU spin:", " ".join(f"{region(20):.4f}" for _ in range(6)), flush=True)
time.sleep(1.0)
for _ in range(60):
    lrt.render_tensor(job, bufs[0], rays, streams[0])
torch.cuda.synchronize()
print("after 60 renders on one stream:", " ".join(f"{region(20):.4f}" for _ in range(6)), flush=True)
lrt.ShutdownTest()
