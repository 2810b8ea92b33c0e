"""Image output for the present step (replaces main.cpp:109-141's GDI
blit): PFM for the linear float backbuffer and binary PPM for the sRGB BGRA8 frame that
lrt_present_bgra8 (present_tensor) produces on the GPU. Row 0 of the backbuffer is the
bottom of the image (bottom-up DIB, main.cpp:33)."""
from __future__ import annotations

import numpy as np


def save_pfm(path: str, backbuffer: np.ndarray) -> None:
    """backbuffer: (H, W, 4) float32, row 0 at the bottom -- PFM's own row order."""
    rgb = np.ascontiguousarray(np.asarray(backbuffer, np.float32)[..., :3], dtype="<f4")
    h, w = rgb.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode("ascii"))   # negative scale: little-endian
        f.write(rgb.tobytes())


def load_pfm(path: str) -> np.ndarray:
    """-> (H, W, 3) float32, row 0 at the bottom."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"PF":
            raise ValueError("not a colour PFM")
        w, h = (int(v) for v in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4", count=w * h * 3)
    return data.reshape(h, w, 3).astype(np.float32)


def save_ppm_bgra(path: str, bgra: np.ndarray, width: int, height: int) -> None:
    """bgra: width*height uint32 pixels b | g << 8 | r << 16 (main.cpp:137-139), row 0 at
    the bottom; written top-down as binary PPM."""
    px = np.asarray(bgra, np.uint32).reshape(height, width)[::-1]
    rgb = np.stack([(px >> 16) & 255, (px >> 8) & 255, px & 255], axis=-1).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(f"P6\n{width} {height}\n255\n".encode("ascii"))
        f.write(rgb.tobytes())
