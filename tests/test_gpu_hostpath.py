"""The reference API's host-buffer paths (lrt_draw_test / lrt_render_host, parallel.cpp:297-323)
under each of their implementations, in fresh processes (the path switches are read once
per process): the pipelined path for page-locked buffers (colours rendered while the
previous values are copied in by DMA, chunked lerp written straight to the host pixels;
1, 3 and 8 row chunks), zero copy (LRT_HOST_PIPELINE=0), a pageable buffer (page-locked for
each call only, then the pipelined path) and the staged path (LRT_HOST_REGISTER=0). Every one must give the oracle's bits and ray counts over several progressive
frames, with the caller's alpha untouched."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

SCRIPT = r'''
import sys
import numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {oracle!r})
import torch
import learnraytracing_amd as lrt
import oracle
lrt.InitializeTest()
w, h = {w}, {h}
bb = lrt.pinned_backbuffer(w * h * 4) if {pinned} else np.zeros(w * h * 4, np.float32)
bb[:] = 0.0
bb[3::4] = 0.25
want = np.zeros((h, w, 4), np.float32)
for f in range(3):
    rays = lrt.DrawTest(0.0, f, w, h, bb)
    _, wr = oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
    assert rays == wr, (f, rays, wr)
got = bb.reshape(h, w, 4)
assert np.array_equal(got[..., :3].view(np.uint32), want[..., :3].view(np.uint32)), "pixels differ"
assert np.all(got[..., 3] == 0.25), "alpha changed"
lrt.ShutdownTest()
print("ok")
'''


@pytest.mark.parametrize("env,pinned,w,h", [
    ({}, True, 200, 117),                                # pipelined, default chunks (4 with the look-ahead)
    ({"LRT_HOST_CHUNKS": "1"}, True, 160, 90),
    ({"LRT_HOST_CHUNKS": "3"}, True, 200, 117),          # uneven chunks
    ({"LRT_HOST_CHUNKS": "8"}, True, 96, 61),
    ({"LRT_DRAW_LOOKAHEAD": "0"}, True, 200, 117),      # no look-ahead render of the next frame
    ({"LRT_HOST_PIPELINE": "0"}, True, 200, 117),        # zero copy
    ({}, False, 200, 117),                               # pageable: page-locked per call, pipelined
    ({"LRT_HOST_REGISTER": "0"}, False, 200, 117),       # pageable, staged
], ids=["pipe2", "pipe1", "pipe3", "pipe8", "nolookahead", "zerocopy", "pageable", "staged"])
def test_drawtest_host_paths(env, pinned, w, h):
    code = SCRIPT.format(root=ROOT, oracle=os.path.join(ROOT, "oracle"), w=w, h=h, pinned=pinned)
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-3000:]
