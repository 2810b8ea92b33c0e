"""Shader clock and span of consecutive config-2 launches (round 6, profiles/r6_g).

Needs the LRT_EXP_WAVETRACE + LRT_EXP_WAVECLK build (tools/build_variant.sh WC
-DLRT_EXP_WAVETRACE -DLRT_EXP_WAVECLK) as LRT_LIB and LRT_WAVETRACE=<file>: every pool launch
appends each wave's {t0, t1 (100-MHz ticks), hw ids, shader cycles}. Runs N launches one at a
time (the dump synchronises), sleeps 1 s, runs N more, then prints per launch: span (us), the
mean shader clock over the waves' lives (MHz) and the summed wave lives (wave-ms)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import learnraytracing_amd as lrt  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 60
path = os.environ["LRT_WAVETRACE"]
torch.cuda.set_device(0)
lrt.InitializeTest()
job = lrt.Job(width=1280, height=720, frames=4, max_depth=8)
buf = torch.zeros((720, 1280, 4), dtype=torch.float32, device="cuda")
rays = torch.zeros(1, dtype=torch.int64, device="cuda")
for phase in range(2):
    for i in range(N):
        lrt.render_tensor(job, buf, rays)
    torch.cuda.synchronize()
    time.sleep(1.0)
lrt.ShutdownTest()
raw = np.fromfile(path, dtype=np.uint64)
i, k = 0, 0
while i < len(raw):
    n = int(raw[i])
    w = raw[i + 1:i + 1 + 4 * n].reshape(n, 4).astype(np.int64)
    i += 1 + 4 * n
    life = (w[:, 1] - w[:, 0]).astype(np.float64)   # 100-MHz ticks
    span_us = (w[:, 1].max() - w[:, 0].min()) / 100.0
    mhz = w[:, 3].sum() / life.sum() * 100.0
    print(f"launch {k:3d}  span {span_us:8.1f} us  clock {mhz:7.1f} MHz  wave-ms {life.sum() / 1e5:9.1f}  "
          f"cycles/wave {w[:, 3].mean():11.0f}", flush=True)
    k += 1
