"""Multi-GPU framebuffer sharding: the row split.

One process per GPU.  The frame's rows are interleaved over ranks (rank r
renders rows r, r+N, r+2N, ...), which balances the very uneven per-row cost
(corridor rows vs wall rows) without any scheduling; the RNG is keyed on
(pixel, sample, frame) so the N-GPU image equals the 1-GPU image bit for bit.
The frame-end gather is the library's (include/mm_comm.h: mm_gather_rows,
RCCL send / recv to rank 0 + a de-interleave kernel), driven by
mirror_maze.comm.NativeGatherer in bench.py; `assemble` below is the same
de-interleave on host tensors, for tests.
"""
from __future__ import annotations


def row_shard(height: int, world: int, rank: int):
    """(y0, y_stride, rows) of this rank's interleaved row set."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank, world, len(range(rank, height, world))


def rows_max(height: int, world: int) -> int:
    """Rows every rank sends (the gather needs equal shapes; short ranks pad)."""
    return (height + world - 1) // world


def assemble(gathered, height: int):
    """[world] x (rows_max, W, C) interleaved tiles -> (height, W, C) frame.
    Row i*world + r of the frame is row i of rank r's tile."""
    import torch

    world = len(gathered)
    rm, w, ch = gathered[0].shape
    full = torch.stack(gathered, dim=1).reshape(rm * world, w, ch)
    return full[:height]
