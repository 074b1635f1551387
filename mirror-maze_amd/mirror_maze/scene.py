"""Scene construction through the C++ host builder (include/mm_scene.h).

Python face of the reference's host-side scene plumbing: the Kruskal maze and
planes (src/main.rs:356-586), the SAH BVH (src/main.rs:74-263), the camera /
Uniform (src/main.rs:732-755) and the chunk scheduler (src/main.rs:293-326).
Arrays use the reference's byte layouts (Plane 48 B, BVHNode 32 B, ...).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib

NODE_DTYPE = np.dtype([("mn", "<f4", 3), ("mx", "<f4", 3), ("left_first", "<u4"), ("count", "<u4")])
assert NODE_DTYPE.itemsize == 32


@dataclass
class Scene:
    """The five scene buffers compute_shader reads (buffers 1, 2, 3, 5, 6)."""

    maze_n: int
    rects: np.ndarray      # (P, 12) float32: o, v, u, color       == Vec<Plane>
    nodes: np.ndarray      # (M,) NODE_DTYPE                        == Vec<BVHNode>
    idx: np.ndarray        # (P,) uint32                            plane indices
    is_mirror: np.ndarray  # (P,) uint8                             Vec<bool>
    emission: np.ndarray   # (P, 4) float32                         Vec<Float4>
    grid: np.ndarray       # (N, N) uint8 maze cell bitmasks
    bvh_depth: int

    @property
    def n_rects(self) -> int:
        return int(self.rects.shape[0])

    @property
    def n_nodes(self) -> int:
        return int(self.nodes.shape[0])

    @classmethod
    def build(cls, maze_n: int = 10, seed: int = 0) -> "Scene":
        """maze_n=10, seed=0 is the reference's scene (src/main.rs:362-363, 381)."""
        L = lib()
        p = C.POINTER(_lib.mm_scene)()
        check(L.mm_scene_build(maze_n, seed, C.byref(p)))
        try:
            s = p.contents
            P, M = s.n_rects, s.n_nodes
            rects = np.ctypeslib.as_array(C.cast(s.rects, C.POINTER(C.c_float)), (P * 12,)).reshape(P, 12).copy()
            nodes = np.frombuffer(C.string_at(s.nodes, M * 32), dtype=NODE_DTYPE).copy()
            idx = np.ctypeslib.as_array(s.idx, (P,)).copy()
            mats = np.ctypeslib.as_array(s.is_mirror, (P,)).copy()
            emis = np.ctypeslib.as_array(s.emission, (P * 4,)).reshape(P, 4).copy()
            grid = np.ctypeslib.as_array(s.grid, (maze_n * maze_n,)).reshape(maze_n, maze_n).copy()
            return cls(maze_n, rects, nodes, idx, mats, emis, grid, int(s.bvh_depth))
        finally:
            L.mm_scene_free(p)

    @staticmethod
    def bvh(rects: np.ndarray, method: int = _lib.MM_BVH_SWEEP):
        """Rebuild the SAH BVH for an arbitrary (P, 12) float32 rect array.

        method: MM_BVH_SWEEP (sorted sweep, default) or MM_BVH_EXHAUSTIVE (the
        reference's O(n^2) candidate loop); both give the same tree."""
        rects = np.ascontiguousarray(rects, dtype=np.float32)
        P = rects.shape[0]
        nodes = np.zeros(2 * P - 1, dtype=NODE_DTYPE)
        idx = np.zeros(P, dtype=np.uint32)
        n = C.c_uint32()
        check(lib().mm_bvh_build_ex(rects.ctypes.data, P, nodes.ctypes.data, C.byref(n), idx.ctypes.data, method))
        return nodes[: n.value].copy(), idx


def default_uniform(view_w: float, view_h: float, time: int = 0) -> _lib.mm_uniform:
    """Camera + Uniform of src/main.rs:732-755 for a view_w x view_h frame."""
    u = _lib.mm_uniform()
    lib().mm_uniform_default(view_w, view_h, time, C.byref(u))
    return u


def calculate_quaternion(d) -> np.ndarray:
    a = np.asarray(d, dtype=np.float32)
    q = np.zeros(4, dtype=np.float32)
    lib().mm_calculate_quaternion(a.ctypes.data, q.ctypes.data)
    return q


class ChunkScheduler:
    """gen_pixels + random_pixels (src/main.rs:293-326), seeded."""

    def __init__(self, view_w: float, view_h: float, chunk_w: int = 4, seed: int = 0):
        self._p = C.c_void_p()
        check(lib().mm_chunks_create(view_w, view_h, chunk_w, seed, C.byref(self._p)))

    @property
    def total(self) -> int:
        return int(lib().mm_chunks_total(self._p))

    def next(self, n: int) -> np.ndarray:
        out = np.zeros((n, 2), dtype=np.uint32)
        check(lib().mm_chunks_next(self._p, n, out.ctypes.data))
        return out

    def close(self) -> None:
        if self._p:
            lib().mm_chunks_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Player:
    """The reference's interactive camera (src/main.rs:738-842, 922-924):
    WASD moves of 5/fps along the rotated axes, undone when the player box
    (+-0.5, 0.2, 0.5) overlaps a BVH leaf (check_collision, main.rs:265-291),
    mouse deltaX turning the view's half angle.  Drives an offline fly-through
    (``uniform``) exactly as the reference's event loop drives its camera."""

    KEY_A, KEY_S, KEY_D, KEY_W = 0, 1, 2, 13   # macOS key codes the reference matches

    def __init__(self, scene: "Scene", view_w: float = 1024, view_h: float = 768):
        self.scene = scene
        self.view_w, self.view_h = view_w, view_h
        u = default_uniform(view_w, view_h, 0)
        self._p = _lib.mm_player()
        q = np.array(list(u.cam.quat), dtype=np.float32)
        check(lib().mm_player_init(q.ctypes.data, C.byref(self._p)))
        self._nodes = np.ascontiguousarray(scene.nodes)

    @property
    def center(self) -> np.ndarray:
        return np.array(list(self._p.center), dtype=np.float32)

    @property
    def quat(self) -> np.ndarray:
        return np.array(list(self._p.quat), dtype=np.float32)

    def step(self, keys=(), mouse_dx=()):
        """One frame; returns the MM_PLAYER_* flags."""
        k = np.ascontiguousarray(keys, dtype=np.uint16)
        m = np.ascontiguousarray(mouse_dx, dtype=np.float32)
        flags = C.c_uint32()
        check(lib().mm_player_step(C.byref(self._p), k.ctypes.data if k.size else None, k.size,
                                   m.ctypes.data if m.size else None, m.size, self._nodes.ctypes.data,
                                   self._nodes.shape[0], C.byref(flags)))
        return flags.value

    def uniform(self, time: int = 0) -> _lib.mm_uniform:
        u = _lib.mm_uniform()
        check(lib().mm_player_uniform(C.byref(self._p), self.view_w, self.view_h, time, C.byref(u)))
        return u


def check_collision(nodes: np.ndarray, bmin, bmax) -> int:
    """check_collision (src/main.rs:265-291): first leaf overlapping the box, or -1."""
    nodes = np.ascontiguousarray(nodes)
    a = np.asarray(bmin, dtype=np.float32)
    b = np.asarray(bmax, dtype=np.float32)
    r = lib().mm_check_collision(nodes.ctypes.data, nodes.shape[0], a.ctypes.data, b.ctypes.data)
    if r == -2:
        raise ValueError("check_collision: node index out of range")
    return int(r)


def quat_mult(v, q) -> np.ndarray:
    a = np.asarray(v, dtype=np.float32)
    b = np.asarray(q, dtype=np.float32)
    out = np.zeros(3, dtype=np.float32)
    lib().mm_quat_mult(a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out
