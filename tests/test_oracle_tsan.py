"""Race detection on the CPU restatement (the reference shares one RNG state
across its workers, maths.cpp:5,9-13; the restatement must not race). The threaded
renderer of oracle/lrt_oracle.c is built under ThreadSanitizer (`make -C oracle tsan`) and
run with 8 threads: no TSan report, and the same bits and ray count as one thread."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from learnraytracing_amd.scene import default_scene, random_scene, scene_arrays

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
EXE = os.path.join(ORACLE, "_tsan", "tsan_check")


@pytest.fixture(scope="module")
def tsan_exe():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-s", "-C", ORACLE, "tsan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("ThreadSanitizer build failed: " + r.stderr[-400:])
    return EXE


def _write_scene(path, spheres, mats):
    s, m = (np.asarray(v, np.float32) for v in scene_arrays(spheres, mats))
    with open(path, "wb") as f:
        f.write(np.int32(len(s) // 4).tobytes())
        f.write(s.tobytes())
        f.write(m.tobytes())


@pytest.mark.parametrize("scene,w,h,frames,depth", [
    ("default", 64, 36, 2, 8),
    ("default", 48, 27, 1, 50),
    ("r1000", 32, 18, 1, 8),
])
def test_threaded_oracle_race_free(tsan_exe, tmp_path, scene, w, h, frames, depth):
    path = str(tmp_path / "scene.bin")
    _write_scene(path, *(default_scene() if scene == "default" else random_scene(1000, 1)))
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([tsan_exe, path, str(w), str(h), str(frames), str(depth), "8"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
    assert r.returncode == 0 and r.stdout.startswith("identical"), (r.stdout, r.stderr[-500:])
