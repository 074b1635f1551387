"""ctypes binding of lib/libmirror_maze.so (include/mm_api.h, include/mm_scene.h).

The library is the product: HIP kernels for gfx950, the C-ABI runtime and the
C++ scene builder.  It is loaded eagerly and loudly: there is no CPU fallback.
``import torch`` (when available) happens first so that the HIP runtime torch
ships (libamdhip64.so.7) is the one the library binds to — device pointers
and streams are then shared with torch.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

try:  # share torch's HIP runtime when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host side
    torch = None

PKG_ROOT = Path(__file__).resolve().parent.parent          # mirror-maze_amd/
LIB_PATH = Path(os.environ.get("MIRROR_MAZE_LIB", PKG_ROOT / "lib" / "libmirror_maze.so"))


class MMError(RuntimeError):
    """A negative return code from the C ABI."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


MM_OK, MM_ERR_INVALID, MM_ERR_HIP, MM_ERR_NOMEM = 0, -1, -2, -3
MM_ERR_NO_SCENE, MM_ERR_STACK, MM_ERR_UNSUPPORTED = -4, -5, -6
MM_EXT_COUNT_STATS, MM_EXT_ACCUMULATE, MM_EXT_RGBA8 = 0x1, 0x2, 0x4
MM_PIPE_AUTO, MM_PIPE_MEGAKERNEL, MM_PIPE_WAVEFRONT, MM_PIPE_REFERENCE = 0, 1, 2, 3
MM_OPT_LDS_NODES, MM_OPT_BLOCK, MM_OPT_PERSIST, MM_OPT_TRAVERSAL, MM_OPT_LDS_RECTS = 1, 2, 3, 7, 8
MM_OPT_LDS_SPLIT, MM_OPT_FUSE_RESOLVE, MM_OPT_RESERVE_CUS, MM_OPT_DICT_NODES, MM_OPT_DEFER = 9, 12, 19, 20, 21
MM_OPT_DEFER_MIN, MM_OPT_FAULT_INJECT, MM_OPT_GRID_MERGE, MM_OPT_GRID_CELL = 22, 23, 24, 25
MM_OPT_GRID_WIDE = 26
MM_PENDING = 1
MM_TRAV_AUTO, MM_TRAV_IFIF, MM_TRAV_LEAF_INTERIOR, MM_TRAV_LEAN, MM_TRAV_GRID = -1, 0, 5, 7, 11
MM_INFO_GRID_OK, MM_INFO_GRID_CELLS_X, MM_INFO_GRID_CELLS_Y, MM_INFO_GRID_CELLS_Z = 1, 2, 3, 4
MM_INFO_GRID_GLOBAL, MM_INFO_GRID_BYTES, MM_INFO_GRID_INDEX_BYTES, MM_INFO_LEAN, MM_INFO_DEPTH = 5, 6, 7, 8, 9
MM_INFO_DICT_OK, MM_INFO_LAST_FORM, MM_INFO_LAST_LDS_MODE, MM_INFO_GRID_FACES = 10, 11, 12, 13
MM_INFO_LAST_DEFER, MM_INFO_LAST_VGPRS, MM_INFO_LAST_SCRATCH, MM_INFO_LAST_STATIC_LDS = 14, 15, 16, 17
MM_INFO_GRID_LDS_CAP = 18
MM_PLAYER_COLLIDED, MM_PLAYER_ROTATED, MM_PLAYER_NAN_QUAT = 1, 2, 4
MM_BVH_SWEEP, MM_BVH_EXHAUSTIVE = 0, 1
MM_OWN_STREAM = C.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF).value  # (void*)-1
MM_COMM_ID_BYTES, MM_GATHER_SELF_VIA_RCCL = 128, 1


class mm_rect(C.Structure):
    _fields_ = [("o", C.c_float * 3), ("v", C.c_float * 3), ("u", C.c_float * 3), ("color", C.c_float * 3)]


class mm_node(C.Structure):
    _fields_ = [("mn", C.c_float * 3), ("mx", C.c_float * 3), ("left_first", C.c_uint32), ("count", C.c_uint32)]


class mm_camera(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("focal", C.c_float), ("quat", C.c_float * 4),
                ("viewport", C.c_float * 2)]


class mm_uniform(C.Structure):
    _fields_ = [("cam", mm_camera), ("view_w", C.c_float), ("view_h", C.c_float),
                ("chunk_w", C.c_uint32), ("time", C.c_uint32)]


class mm_ext(C.Structure):
    _fields_ = [("spp", C.c_uint32), ("bounce_limit", C.c_uint32), ("mirror_limit", C.c_uint32),
                ("frame", C.c_uint32), ("flags", C.c_uint32), ("reserved", C.c_uint32)]


class mm_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("rect_tests", C.c_uint64),
                ("paths", C.c_uint64)]


class mm_rng(C.Structure):
    _fields_ = [("key", C.c_uint32 * 8), ("counter", C.c_uint64), ("buf", C.c_uint32 * 64), ("pos", C.c_uint32)]


class mm_player(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("quat", C.c_float * 4), ("half_theta", C.c_float), ("fps", C.c_float)]


class mm_scene(C.Structure):
    _fields_ = [("maze_n", C.c_uint32), ("n_rects", C.c_uint32), ("rects", C.POINTER(mm_rect)),
                ("is_mirror", C.POINTER(C.c_uint8)), ("emission", C.POINTER(C.c_float)),
                ("n_nodes", C.c_uint32), ("nodes", C.POINTER(mm_node)), ("idx", C.POINTER(C.c_uint32)),
                ("grid", C.POINTER(C.c_uint8)), ("n_vert_walls", C.c_uint32), ("n_hori_walls", C.c_uint32),
                ("bvh_depth", C.c_uint32)]


P = C.c_void_p
# name -> (restype, argtypes); every symbol include/mm_api.h and mm_scene.h declare
EXPORTS = {
    # mm_api.h
    "mm_version": (C.c_char_p, []),
    "mm_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "mm_destroy": (None, [P]),
    "mm_last_error": (C.c_char_p, [P]),
    "mm_set_stream": (C.c_int, [P, P]),
    "mm_get_stream": (C.c_int, [P, C.POINTER(P)]),
    "mm_upload_scene": (C.c_int, [P, P, C.c_uint32, P, C.c_uint32, P, P, P]),
    "mm_trace_chunks": (C.c_int, [P, C.POINTER(mm_uniform), P, C.c_uint32]),
    "mm_read_framebuffer": (C.c_int, [P, P, P]),
    "mm_present": (C.c_int, [P]),
    "mm_read_packets": (C.c_int, [P, P, C.c_uint32]),
    "mm_quantize_rgba8": (C.c_int, [P, P, P, C.c_uint64]),
    "mm_trace_tile": (C.c_int, [P, C.POINTER(mm_uniform), C.POINTER(mm_ext), C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint32, C.c_uint32, P, C.POINTER(mm_stats)]),
    "mm_trace_tile_frames": (C.c_int, [P, C.POINTER(mm_uniform), C.POINTER(mm_ext), C.c_uint32, C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, C.POINTER(mm_stats)]),
    "mm_set_pipeline": (C.c_int, [P, C.c_int]),
    "mm_set_option": (C.c_int, [P, C.c_int, C.c_int]),
    "mm_scene_info": (C.c_int, [P, C.c_int, C.POINTER(C.c_double)]),
    "mm_set_wave_timeline": (C.c_int, [P, P, C.c_uint32]),
    "mm_sync": (C.c_int, [P]),
    "mm_last_call": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "mm_call_status": (C.c_int, [P, C.c_uint64]),
    "mm_last_timing": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(C.c_uint32)]),
    "mm_set_profiling": (C.c_int, [P, C.c_int]),
    "mm_kernel_timing": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.c_int]),
    # mm_comm.h
    "mm_comm_unique_id": (C.c_int, [P, P]),
    "mm_comm_init_rank": (C.c_int, [P, C.c_int, C.c_int, P, C.POINTER(P)]),
    "mm_comm_init_all": (C.c_int, [C.c_int, P, P]),
    "mm_comm_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mm_comm_rccl_version": (C.c_int, []),
    "mm_comm_rccl_header_version": (C.c_int, []),
    "mm_comm_destroy": (None, [P]),
    "mm_row_shard": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "mm_gather_rows": (C.c_int, [P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, C.c_uint32]),
    "mm_gather_rows_all": (C.c_int, [C.c_int, P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P,
                                     C.c_uint32]),
    "mm_assemble_rows": (C.c_int, [P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P]),
    # mm_scene.h
    "mm_rng_seed_from_u64": (None, [C.POINTER(mm_rng), C.c_uint64]),
    "mm_rng_from_seed": (None, [C.POINTER(mm_rng), P]),
    "mm_rng_next_u32": (C.c_uint32, [C.POINTER(mm_rng)]),
    "mm_rng_next_u64": (C.c_uint64, [C.POINTER(mm_rng)]),
    "mm_rng_gen_f32": (C.c_float, [C.POINTER(mm_rng)]),
    "mm_rng_gen_range_u32": (C.c_uint32, [C.POINTER(mm_rng), C.c_uint32, C.c_uint32]),
    "mm_chacha_block": (None, [P, C.c_uint64, C.c_uint64, C.c_int, P]),
    "mm_scene_build": (C.c_int, [C.c_uint32, C.c_uint64, C.POINTER(C.POINTER(mm_scene))]),
    "mm_scene_free": (None, [C.POINTER(mm_scene)]),
    "mm_bvh_build": (C.c_int, [P, C.c_uint32, P, C.POINTER(C.c_uint32), P]),
    "mm_bvh_build_ex": (C.c_int, [P, C.c_uint32, P, C.POINTER(C.c_uint32), P, C.c_int]),
    "mm_bvh_depth": (C.c_uint32, [P, C.c_uint32]),
    "mm_calculate_quaternion": (None, [P, P]),
    "mm_uniform_default": (None, [C.c_float, C.c_float, C.c_uint32, C.POINTER(mm_uniform)]),
    "mm_chunks_create": (C.c_int, [C.c_float, C.c_float, C.c_uint32, C.c_uint64, C.POINTER(P)]),
    "mm_chunks_total": (C.c_uint32, [P]),
    "mm_chunks_next": (C.c_int, [P, C.c_uint32, P]),
    "mm_chunks_free": (None, [P]),
    "mm_quat_mult": (None, [P, P, P]),
    "mm_update_quat_angle": (None, [P, C.c_float, P]),
    "mm_check_collision": (C.c_int, [P, C.c_uint32, P, P]),
    "mm_player_init": (C.c_int, [P, C.POINTER(mm_player)]),
    "mm_player_step": (C.c_int, [C.POINTER(mm_player), P, C.c_uint32, P, C.c_uint32, P, C.c_uint32, P]),
    "mm_player_uniform": (C.c_int, [C.POINTER(mm_player), C.c_float, C.c_float, C.c_uint32, C.POINTER(mm_uniform)]),
    # mm_io.h
    "mm_write_ppm": (C.c_int, [C.c_char_p, P, C.c_uint32, C.c_uint32]),
    "mm_write_png": (C.c_int, [C.c_char_p, P, C.c_uint32, C.c_uint32]),
    "mm_quantize_rgba8_host": (None, [P, P, C.c_uint64]),
}

_lib = None


def lib() -> C.CDLL:
    """Load the product library (raises if it is missing — no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"mirror-maze HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, ctx=None) -> None:
    if rc != MM_OK:
        msg = lib().mm_last_error(ctx).decode() if ctx else "error"
        raise MMError(rc, msg)
