"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle
(oracle/_build/libmm_oracle.so, a restatement of src/shaders.metal:245-368).
Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never from the product package.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libmm_oracle.so"
# bench.py's same-algorithm CPU baseline (grid_cpu.c): the oracle's path loop with the product's certified
# grid search as the closest-hit query -- not a checker
GRID_LIB_PATH = HERE / "_build" / "libmm_gridcpu.so"


class _U(C.Structure):  # mm_uniform, include/mm_types.h
    _fields_ = [("center", C.c_float * 3), ("focal", C.c_float), ("quat", C.c_float * 4),
                ("viewport", C.c_float * 2), ("view_w", C.c_float), ("view_h", C.c_float),
                ("chunk_w", C.c_uint32), ("time", C.c_uint32)]


class OracleScene(C.Structure):
    _fields_ = [("rects", C.c_void_p), ("n_rects", C.c_uint32), ("nodes", C.c_void_p), ("n_nodes", C.c_uint32),
                ("idx", C.c_void_p), ("is_mirror", C.c_void_p), ("emission", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("rect_tests", C.c_uint64), ("paths", C.c_uint64)]


_lib = None
_grid_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def _bind(path):
    if not path.exists():
        build()
    return _declare(C.CDLL(str(path)))


def grid_lib():
    """The same-algorithm CPU baseline's library (grid_cpu.c; bench.py only)."""
    global _grid_lib
    if _grid_lib is None:
        L = _bind(GRID_LIB_PATH)
        L.gridcpu_build.argtypes = [C.c_void_p]
        L.gridcpu_build.restype = C.c_int
        L.gridcpu_scene.argtypes = []
        L.gridcpu_scene.restype = C.c_void_p
        L.gridcpu_stats.argtypes = [C.c_void_p, C.c_int]
        L.gridcpu_stats.restype = None
        _grid_lib = L
    return _grid_lib


def lib():
    global _lib
    if _lib is None:
        _lib = _bind(LIB_PATH)
    return _lib


def _declare(L):
    """Argument and result types of the oracle entry points."""
    P = C.c_void_p
    L.oracle_trace_chunks.argtypes = [P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, P, P]
    L.oracle_trace_group.argtypes = [P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, P]
    L.oracle_trace_tile.argtypes = [P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, P]
    L.oracle_trace_path.argtypes = [P, P, P, C.c_uint32, C.c_int, C.c_int, P, P]
    L.oracle_rand_pm1.argtypes = [P]
    L.oracle_rand_pm1.restype = C.c_float
    L.oracle_seed_reference.argtypes = [C.c_uint32] * 3
    L.oracle_seed_reference.restype = C.c_uint32
    L.oracle_tile_seed.argtypes = [C.c_uint32] * 3
    L.oracle_tile_seed.restype = C.c_uint32
    L.oracle_primary_dir.argtypes = [P, C.c_uint32, C.c_uint32, P]
    L.oracle_intersect_aabb.argtypes = [P, P, C.c_float, P, P]
    L.oracle_intersect_aabb.restype = C.c_float
    L.oracle_present_blur.argtypes = [P, P, C.c_uint32, C.c_uint32]
    L.oracle_present_blur.restype = None
    L.oracle_quantize.argtypes = [P, P, C.c_uint64]
    L.oracle_quantize.restype = None
    L.oracle_set_fp_mode.argtypes = [C.c_int]
    L.oracle_set_fp_mode.restype = None
    L.oracle_fp_flags.argtypes = [C.c_int]
    L.oracle_fp_flags.restype = C.c_uint
    return L


class Oracle:
    """Holds numpy copies of a scene and calls the oracle on them."""

    def __init__(self, rects, nodes, idx, is_mirror, emission):
        self.rects = np.ascontiguousarray(rects, dtype=np.float32)
        self.nodes = np.ascontiguousarray(nodes)
        self.idx = np.ascontiguousarray(idx, dtype=np.uint32)
        self.is_mirror = np.ascontiguousarray(is_mirror, dtype=np.uint8)
        self.emission = np.ascontiguousarray(emission, dtype=np.float32)
        self.sc = OracleScene(self.rects.ctypes.data, self.rects.shape[0], self.nodes.ctypes.data,
                              self.nodes.shape[0], self.idx.ctypes.data, self.is_mirror.ctypes.data,
                              self.emission.ctypes.data)

        self._lib = lib

    @classmethod
    def from_scene(cls, s, method: str = "walk") -> "Oracle":
        """method "walk": the oracle (the reference BVH walk on every query);
        "grid": the same path loop with the product's certified grid search as
        the query (grid_cpu.c) -- bench.py's same-algorithm CPU baseline."""
        o = cls(s.rects, s.nodes, s.idx, s.is_mirror, s.emission)
        if method == "grid":
            if grid_lib().gridcpu_build(C.byref(o.sc)) != 0:
                raise RuntimeError("gridcpu_build failed")
            o._lib = o._grid_checked
        elif method != "walk":
            raise ValueError(method)
        return o

    def _grid_checked(self):
        """grid_lib(), after checking that the process's one grid is this
        scene's: a later grid Oracle rebuilds it for its own scene, and this
        one's queries would then silently walk the BVH."""
        L = grid_lib()
        if L.gridcpu_scene() != C.addressof(self.sc):
            raise RuntimeError("grid_cpu holds another scene's grid (one grid per process): rebuild with "
                               "Oracle.from_scene(s, method='grid')")
        return L

    @staticmethod
    def grid_stats(reset: bool = False) -> dict:
        """grid_cpu's query counts since the last build: grid answers, walk
        fallbacks, and queries for another scene (walked)."""
        out = (C.c_uint64 * 3)()
        grid_lib().gridcpu_stats(out, 1 if reset else 0)
        return {"grid": out[0], "fallback": out[1], "other_scene": out[2]}

    @staticmethod
    def _u(uniform) -> bytes:
        return bytes(uniform)  # mm_uniform is 56 B, same layout

    def trace_chunks(self, uniform, chunks, fb=None, tg=(32, 32)):
        W, H = int(uniform.view_w), int(uniform.view_h)
        if fb is None:
            fb = np.zeros((H, W, 4), dtype=np.float32)
        ch = np.ascontiguousarray(chunks, dtype=np.uint32).reshape(-1, 2)
        ub = C.create_string_buffer(bytes(uniform), len(bytes(uniform)))
        st = Stats()
        rc = self._lib().oracle_trace_chunks(C.byref(self.sc), ub, ch.ctypes.data, ch.shape[0], tg[0], tg[1],
                                       fb.ctypes.data, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_trace_chunks rc={rc}")
        return fb, st

    def trace_group(self, uniform, chunks, gx, gy, fb, tg=(32, 32)):
        ch = np.ascontiguousarray(chunks, dtype=np.uint32).reshape(-1, 2)
        ub = C.create_string_buffer(bytes(uniform), len(bytes(uniform)))
        st = Stats()
        rc = self._lib().oracle_trace_group(C.byref(self.sc), ub, ch.ctypes.data, ch.shape[0], tg[0], tg[1], gx, gy,
                                      fb.ctypes.data, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_trace_group rc={rc}")
        return st

    def trace_tile(self, uniform, ext, x0, y0, w, h, y_stride=1, out=None):
        if out is None:
            out = np.zeros((h, w, 4), dtype=np.float32)
        ub = C.create_string_buffer(bytes(uniform), len(bytes(uniform)))
        eb = C.create_string_buffer(bytes(ext), len(bytes(ext)))
        st = Stats()
        rc = self._lib().oracle_trace_tile(C.byref(self.sc), ub, eb, x0, y0, w, h, y_stride, out.ctypes.data, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_trace_tile rc={rc}")
        return out, st

    def trace_path(self, ori, d, seed, bounce_limit=5, mirror_limit=15):
        o = np.asarray(ori, dtype=np.float32)
        dd = np.asarray(d, dtype=np.float32)
        rgb = np.zeros(3, dtype=np.float32)
        rays = C.c_uint32()
        rc = self._lib().oracle_trace_path(C.byref(self.sc), o.ctypes.data, dd.ctypes.data, seed, bounce_limit,
                                     mirror_limit, rgb.ctypes.data, C.byref(rays))
        return rgb, rays.value, rc


def present_blur(tex: np.ndarray) -> np.ndarray:
    """One Jacobi blur step of an (H, W, 4) uint8 texture (oracle_present_blur)."""
    tex = np.ascontiguousarray(tex, dtype=np.uint8)
    out = np.empty_like(tex)
    lib().oracle_present_blur(tex.ctypes.data, out.ctypes.data, tex.shape[1], tex.shape[0])
    return out


def quantize(rgba: np.ndarray) -> np.ndarray:
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    out = np.empty(rgba.shape, dtype=np.uint8)
    lib().oracle_quantize(rgba.ctypes.data, out.ctypes.data, rgba.size // 4)
    return out


class DisplayLoop:
    """The reference's per-frame sequence on the RGBA8 screen texture
    (src/main.rs:860-894): compute_shader writes the traced chunks' texels,
    then the fragment_shader blur runs over the whole texture."""

    def __init__(self, oracle: Oracle, W: int, H: int):
        self.o = oracle
        self.tex = np.zeros((H, W, 4), dtype=np.uint8)

    def frame(self, uniform, chunks, present: bool = True) -> np.ndarray:
        H, W = self.tex.shape[:2]
        fb = np.full((H, W, 4), np.nan, dtype=np.float32)
        self.o.trace_chunks(uniform, chunks, fb=fb)
        written = ~np.isnan(fb[..., 0])
        self.tex[written] = quantize(fb[written])
        if present:
            self.tex = present_blur(self.tex)
        return self.tex


# MXCSR sticky-flag bits oracle_fp_flags reports
FP_DENORMAL_OPERAND, FP_UNDERFLOW = 1 << 1, 1 << 4


def set_fp_mode(ftz_daz: bool) -> None:
    """True: the trace entry points run with MXCSR FTZ|DAZ -- the reference's
    `air.compile.denorms_disable` (src/shaders.ir !47); False (default): IEEE
    binary32 with denormals, the HIP kernels' arithmetic."""
    lib().oracle_set_fp_mode(1 if ftz_daz else 0)


def fp_flags(reset: bool = False) -> int:
    """MXCSR sticky flags raised by the trace entry points since the last reset
    (FP_DENORMAL_OPERAND: some operand was denormal; FP_UNDERFLOW: some result
    was tiny and inexact)."""
    return int(lib().oracle_fp_flags(1 if reset else 0))
