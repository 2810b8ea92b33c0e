"""The reference-side binding and the plain-C hosts.

* CPU: integration/parallel_lrt.cpp compiles against the reference's own
  src/cpu/parallel.h, and a translation unit that only sees parallel.h links against it
  (the three declarations of parallel.h:6-8 resolve to the binding). Skipped where the
  reference is absent (the GPU box).
* GPU: the prebuilt headless hosts run the reference's call sequence (main.cpp:40-77,165:
  InitializeTest, DrawTest with frameCount 0, 1, 2, ShutdownTest) -- drawtest_ref_api
  through parallel.h -> parallel_lrt.cpp -> liblrt_hip.so, and learnraytracing_amd/lrt_demo
  (plain C) -- and the PFM each writes equals the oracle bit for bit, rays included.
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (test infrastructure)

REF_H = "/root/reference/src/cpu/parallel.h"
LIBDIR = os.path.join(ROOT, "learnraytracing_amd")


@pytest.mark.skipif(not os.path.exists(REF_H), reason="reference sources absent")
def test_binding_compiles_and_links_against_reference_header(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "liblrt_hip.so")):
        pytest.skip("liblrt_hip.so not built")
    inc = ["-I" + os.path.dirname(REF_H), "-I" + os.path.join(ROOT, "include")]
    obj = tmp_path / "parallel_lrt.o"
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", *inc, "-c", "-o", str(obj),
                    os.path.join(ROOT, "integration", "parallel_lrt.cpp")], check=True)
    # a caller that sees only the reference's header takes the address of each function
    caller = tmp_path / "caller.cpp"
    caller.write_text('#include "parallel.h"\n'
                      "int main() {\n"
                      "  void (*i)() = &InitializeTest; void (*s)() = &ShutdownTest;\n"
                      "  void (*d)(float, int, int, int, float*, int&) = &DrawTest;\n"
                      "  return (i && s && d) ? 0 : 1;\n}\n")
    exe = tmp_path / "caller"
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", *inc, "-o", str(exe), str(caller), str(obj),
                    "-L" + LIBDIR, "-llrt_hip", "-Wl,-rpath," + LIBDIR], check=True)
    syms = subprocess.run(["nm", "-C", str(obj)], capture_output=True, text=True, check=True).stdout
    for s in ("InitializeTest()", "ShutdownTest()", "DrawTest(float, int, int, int, float*, int&)"):
        assert re.search(r" T " + re.escape(s), syms), s


def _read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(v) for v in f.readline().split())
        assert float(f.readline()) < 0   # little-endian
        return np.frombuffer(f.read(), "<f4").reshape(h, w, 3)


def _run_host(exe, w, h, frames, tmp_path, env=None):
    if not os.path.exists(exe):
        pytest.skip(f"{os.path.relpath(exe, ROOT)} not built (build() makes it where the reference is present)")
    out = tmp_path / "out.pfm"
    p = subprocess.run([exe, str(w), str(h), str(frames), str(out)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stderr[-2000:]
    rays = int(re.search(r"rays (\d+)", p.stdout).group(1))
    return _read_pfm(out), rays


def _drawtest_oracle(w, h, frames):
    want = np.zeros((h, w, 4), np.float32)
    rays = 0
    for f in range(frames):   # DrawTest: one frame per call, kMaxDepth 20 (parallel.cpp:12,297-323)
        _, r = oracle.orc_render(w, h, 1, 20, frame0=f, buf=want)
        rays += r
    return want[..., :3], rays


@pytest.mark.gpu
@pytest.mark.parametrize("exe", [os.path.join(ROOT, "integration", "_build", "drawtest_ref_api"),
                                 os.path.join(LIBDIR, "lrt_demo")], ids=["parallel_h_binding", "lrt_demo"])
def test_headless_host_matches_oracle(exe, tmp_path):
    w, h, frames = 160, 90, 3
    img, rays = _run_host(exe, w, h, frames, tmp_path)
    want, wrays = _drawtest_oracle(w, h, frames)
    assert rays == wrays
    assert np.array_equal(img.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["0", "0,0,0"], ids=["rccl-1", "copy-3"])
def test_binding_multi_device_matches_oracle(devices, tmp_path):
    """The unchanged main.cpp-style host through parallel_lrt.cpp with LRT_DEVICES: DrawTest's
    rows split over the listed devices (lrt_initialize_devices; RCCL with one device here, the
    copy exchange for a repeated id) -- the same bits as the oracle."""
    w, h, frames = 160, 90, 3
    img, rays = _run_host(os.path.join(ROOT, "integration", "_build", "drawtest_ref_api"), w, h, frames, tmp_path,
                          env={"LRT_DEVICES": devices})
    want, wrays = _drawtest_oracle(w, h, frames)
    assert rays == wrays
    assert np.array_equal(img.view(np.uint32), want.view(np.uint32))
