"""Multi-GPU framebuffer sharding.

One process per GPU.  The frame's rows are interleaved over ranks (rank r
renders rows r, r+N, r+2N, ...), which balances the very uneven per-row cost
(corridor rows vs wall rows) without any scheduling; the RNG is keyed on
(pixel, sample, frame) so the N-GPU image equals the 1-GPU image bit for bit.
At frame end one collective moves every tile to rank 0: torch.distributed's
gather (RCCL send/recv over xGMI with the "nccl" backend; gloo on CPU for
tests), then a de-interleave on rank 0.
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


def gather_frame(tile, height: int, dst: int = 0, group=None, out=None):
    """Gather every rank's (rows_max, W, C) tile to `dst` and return the
    assembled frame there (None elsewhere).  `out` may receive the frame."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    gathered = [torch.empty_like(tile) for _ in range(world)] if rank == dst else None
    dist.gather(tile, gathered, dst=dst, group=group)
    if rank != dst:
        return None
    frame = assemble(gathered, height)
    if out is not None:
        out.copy_(frame)
        return out
    return frame


class FrameGatherer:
    """Pipelined frame-end gather for a sequence of frames.

    Two tile buffers alternate: frame k is traced into ``tile(k)`` and its
    gather is issued asynchronously, so it runs on the collective's stream
    while frame k+1 is traced; the assembly of frame k on rank ``dst`` is
    queued after frame k+1's trace (``put`` of frame k+1 waits for gather k
    before assembling it).  ``flush`` completes the last frame.  Stream order
    makes the reuse safe: gather k is awaited (on the current stream) before
    frame k+2 is traced into the same tile, and every gather is launched after
    the current stream's earlier work (the assembly reading its buffers)."""

    def __init__(self, shape, height: int, device, dst: int = 0, group=None, out=None):
        import torch
        import torch.distributed as dist

        self.height, self.dst, self.group, self.out = height, dst, group, out
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.tiles = [torch.zeros(shape, dtype=torch.float32, device=device) for _ in range(2)]
        self.bufs = ([[torch.empty(shape, dtype=torch.float32, device=device) for _ in range(self.world)]
                      for _ in range(2)] if self.rank == dst else [None, None])
        self.k = 0
        self.pending = None

    def tile(self):
        """The buffer the next frame must be traced into."""
        return self.tiles[self.k % 2]

    def put(self):
        """Issue the gather of the frame just traced into ``tile()``."""
        import torch.distributed as dist

        slot = self.k % 2
        work = dist.gather(self.tiles[slot], self.bufs[slot], dst=self.dst, group=self.group, async_op=True)
        prev, self.pending = self.pending, (work, slot)
        self.k += 1
        if prev is not None:
            self._finish(prev)

    def flush(self):
        if self.pending is not None:
            prev, self.pending = self.pending, None
            self._finish(prev)
        return self.out

    def _finish(self, p):
        work, slot = p
        work.wait()
        if self.rank == self.dst:
            frame = assemble(self.bufs[slot], self.height)
            if self.out is None:
                self.out = frame.clone()
            else:
                self.out.copy_(frame)
