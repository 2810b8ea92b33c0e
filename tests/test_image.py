"""PFM / PPM writers of the present step (learnraytracing_amd/image.py)."""
import numpy as np

from learnraytracing_amd.image import load_pfm, save_pfm, save_ppm_bgra


def test_pfm_round_trip_bitwise(tmp_path):
    g = np.random.default_rng(0)
    buf = g.random((18, 32, 4), dtype=np.float32) * 40
    p = tmp_path / "f.pfm"
    save_pfm(str(p), buf)
    back = load_pfm(str(p))
    assert np.array_equal(back.view(np.uint32), np.ascontiguousarray(buf[..., :3]).view(np.uint32))


def test_ppm_bgra_order(tmp_path):
    w, h = 3, 2
    bgra = np.array([0x00010203, 0, 0, 0, 0, 0x00ff0000], np.uint32)   # (x0,y0) bottom-left, (x2,y1) top-right
    p = tmp_path / "f.ppm"
    save_ppm_bgra(str(p), bgra, w, h)
    data = p.read_bytes()
    assert data.startswith(b"P6\n3 2\n255\n")
    rgb = np.frombuffer(data[len(b"P6\n3 2\n255\n"):], np.uint8).reshape(h, w, 3)
    assert rgb[0, 2].tolist() == [255, 0, 0]      # top row first: bottom-up rows flipped
    assert rgb[1, 0].tolist() == [1, 2, 3]
