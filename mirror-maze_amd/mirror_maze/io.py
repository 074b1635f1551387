"""Frame files (include/mm_io.h): PPM / PNG writers and host RGBA8 quantisation."""
from __future__ import annotations

import os

import numpy as np

from ._lib import MMError, lib


def _rgba8(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an (H, W, 4) uint8 RGBA8 image")
    return img


def quantize(rgba: np.ndarray) -> np.ndarray:
    """float32 (..., 4) -> uint8 with the texture-write conversion."""
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    out = np.empty(rgba.shape, dtype=np.uint8)
    lib().mm_quantize_rgba8_host(rgba.ctypes.data, out.ctypes.data, rgba.size // 4)
    return out


def write_ppm(path: str | os.PathLike, rgba8: np.ndarray) -> None:
    img = _rgba8(rgba8)
    rc = lib().mm_write_ppm(os.fsencode(path), img.ctypes.data, img.shape[1], img.shape[0])
    if rc:
        raise MMError(rc, f"mm_write_ppm({path}) failed")


def write_png(path: str | os.PathLike, rgba8: np.ndarray) -> None:
    img = _rgba8(rgba8)
    rc = lib().mm_write_png(os.fsencode(path), img.ctypes.data, img.shape[1], img.shape[0])
    if rc:
        raise MMError(rc, f"mm_write_png({path}) failed")
