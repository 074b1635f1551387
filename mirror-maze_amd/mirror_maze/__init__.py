"""mirror_maze — MI355X-native offline renderer for mirror-maze's ray-trace loop.

Host-side mirror of the reference's operator interface over the C ABI in
include/mm_api.h (HIP path) and include/mm_scene.h (C++ scene builder).
"""
from ._lib import (MM_EXT_ACCUMULATE, MM_EXT_COUNT_STATS, MM_EXT_RGBA8, MM_INFO_DEPTH, MM_INFO_DICT_OK, MM_INFO_GRID_BYTES,  # noqa: F401
                   MM_INFO_GRID_CELLS_X, MM_INFO_GRID_CELLS_Y, MM_INFO_GRID_CELLS_Z, MM_INFO_GRID_GLOBAL,
                   MM_INFO_GRID_FACES, MM_INFO_GRID_INDEX_BYTES, MM_INFO_GRID_OK, MM_INFO_LAST_FORM, MM_INFO_LAST_LDS_MODE, MM_INFO_LEAN, MM_PIPE_AUTO, MM_PIPE_MEGAKERNEL,
                   MM_PIPE_REFERENCE, MM_PIPE_WAVEFRONT, MM_TRAV_AUTO, MM_TRAV_GRID, MM_TRAV_IFIF,
                   MM_TRAV_LEAF_INTERIOR, MM_TRAV_LEAN, MMError, lib, mm_ext, mm_stats, mm_uniform)
from ._lib import (MM_INFO_GRID_LDS_CAP, MM_INFO_LAST_DEFER, MM_INFO_LAST_SCRATCH, MM_INFO_LAST_STATIC_LDS, MM_INFO_LAST_VGPRS,  # noqa: F401
                   MM_OPT_FAULT_INJECT, MM_OPT_GRID_WIDE, MM_PENDING)
from .renderer import Renderer, make_ext  # noqa: F401
from .scene import ChunkScheduler, Player, Scene, calculate_quaternion, check_collision, default_uniform  # noqa: F401

__all__ = ["Renderer", "Scene", "ChunkScheduler", "Player", "check_collision", "default_uniform", "calculate_quaternion", "make_ext",
           "mm_ext", "mm_stats", "mm_uniform", "MMError", "lib"]
