"""Multi-GPU framebuffer sharding.

One process per GPU.  The frame's rows are interleaved over ranks (rank r
renders rows r, r+N, r+2N, ...), which balances the very uneven per-row cost
(corridor rows vs wall rows) without any scheduling; the RNG is keyed on
(pixel, sample, frame) so the N-GPU image equals the 1-GPU image bit for bit.
At frame end one collective moves every tile to rank 0: torch.distributed's
gather (RCCL send/recv over xGMI with the "nccl" backend; gloo on CPU for
tests), then a de-interleave on rank 0.  FrameGatherer pipelines one gather
per frame; BatchGatherer issues one gather per multi-frame launch (bench.py's
default issue mode: the launch's frames all finish together).
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

    ``slots`` tile buffers rotate: frame k is traced into ``tile()`` (slot
    k % slots) and ``put()`` issues its gather asynchronously on the current
    stream, so the collective runs while later frames are traced.  The gather
    of frame k is completed -- awaited on the current stream, then assembled
    on rank ``dst`` -- when its slot is handed out again (``tile()`` of frame
    k + slots) or by ``flush()``.  A caller that traces frame k on stream
    s[k % slots] (bench.py: one renderer context per stream, so consecutive
    frames overlap on the GPU) calls ``tile()`` and ``put()`` inside that
    stream; then each stream waits only for the gather that last read its own
    tile before overwriting it, and never for the other stream's trace.
    Completed frames are copied into ``out`` and passed to ``on_frame(k,
    frame)`` (rank ``dst`` only), in frame order.  With ``assembly_stream``
    (CUDA only) the de-interleave runs there instead of on the trace streams:
    a small copy kernel queued ahead of a trace kernel would wait for the CUs
    the other stream's trace holds and delay that trace."""

    def __init__(self, shape, height: int, device, dst: int = 0, group=None, out=None, slots: int = 2,
                 on_frame=None, assembly_stream=None, dtype=None):
        import torch
        import torch.distributed as dist

        self.height, self.dst, self.group, self.out = height, dst, group, out
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.slots = slots
        self.on_frame = on_frame
        dtype = torch.float32 if dtype is None else dtype
        self.tiles = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(slots)]
        self.bufs = ([[torch.empty(shape, dtype=dtype, device=device) for _ in range(self.world)]
                      for _ in range(slots)] if self.rank == dst else [None] * slots)
        self.k = 0
        self.pending = [None] * slots   # (frame index, Work) per slot
        self.asm = assembly_stream
        self.asm_done = [None] * slots  # event: assembly of the slot's last frame done

    def tile(self):
        """The buffer the next frame must be traced into (completes the gather
        that last used it)."""
        slot = self.k % self.slots
        self._finish(slot)
        return self.tiles[slot]

    def put(self):
        """Issue the gather of the frame just traced into ``tile()``."""
        import torch.distributed as dist

        slot = self.k % self.slots
        if self.asm_done[slot] is not None:  # bufs[slot] is free once its last assembly ran
            import torch

            torch.cuda.current_stream().wait_event(self.asm_done[slot])
            self.asm_done[slot] = None
        work = dist.gather(self.tiles[slot], self.bufs[slot], dst=self.dst, group=self.group, async_op=True)
        self.pending[slot] = (self.k, work)
        self.k += 1

    def flush(self):
        """Complete every outstanding gather (oldest first); returns ``out``."""
        for i in range(self.slots):
            self._finish((self.k + i) % self.slots)
        return self.out

    def _finish(self, slot):
        p = self.pending[slot]
        if p is None:
            return
        self.pending[slot] = None
        k, work = p
        work.wait()  # the current stream may now overwrite tiles[slot]
        if self.rank != self.dst:
            return
        if self.asm is None:
            self._assemble(k, slot)
            return
        import torch

        with torch.cuda.stream(self.asm):
            work.wait()
            self._assemble(k, slot)
            ev = torch.cuda.Event()
            ev.record(self.asm)
            self.asm_done[slot] = ev

    def _assemble(self, k, slot):
        frame = assemble(self.bufs[slot], self.height)
        if self.out is None:
            self.out = frame.clone()
        else:
            self.out.copy_(frame)
        if self.on_frame is not None:
            self.on_frame(k, self.out)


class BatchGatherer:
    """One gather per multi-frame launch.

    The frames of one ``mm_trace_tile_frames`` launch all finish when the
    launch does, so gathering them one by one buys no earlier delivery -- only
    n collectives' fixed latency where one would do.  ``tiles(n)`` hands out
    the (n, rows_max, W, C) slice of a slot buffer (completing the gather that
    last used the slot) for the launch's frames; ``put(n)`` issues ONE
    asynchronous gather of the whole slice (every rank passes the same n: the
    launch sizes are deterministic); rank ``dst`` de-interleaves frame by frame
    into ``out`` and calls ``on_frame(k, frame)`` in frame order when the slot
    is reused or on ``flush()``.  ``slots`` buffers rotate (2: the next launch's
    frames are converted while this launch's gather runs)."""

    def __init__(self, shape, height: int, device, max_frames: int, dst: int = 0, group=None, out=None,
                 slots: int = 2, on_frame=None, assembly_stream=None, dtype=None):
        import torch
        import torch.distributed as dist

        self.height, self.dst, self.group, self.out = height, dst, group, out
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.slots, self.max_frames = slots, max_frames
        self.on_frame = on_frame
        dtype = torch.float32 if dtype is None else dtype
        bshape = (max_frames,) + tuple(shape)
        self.tiles_ = [torch.zeros(bshape, dtype=dtype, device=device) for _ in range(slots)]
        self.bufs = ([[torch.empty(bshape, dtype=dtype, device=device) for _ in range(self.world)]
                      for _ in range(slots)] if self.rank == dst else [None] * slots)
        self.k = 0         # frames issued so far
        self.launch = 0    # gathers issued so far
        self.pending = [None] * slots   # (first frame, n, Work) per slot
        self.asm = assembly_stream
        self.asm_done = [None] * slots

    def tiles(self, n: int):
        """The (n, rows_max, W, C) buffer the next launch's frames go into."""
        if not (1 <= n <= self.max_frames):
            raise ValueError(f"batch of {n} frames outside 1..{self.max_frames}")
        slot = self.launch % self.slots
        self._finish(slot)
        return self.tiles_[slot][:n]

    def put(self, n: int):
        """Issue the gather of the n frames just written into ``tiles(n)``."""
        import torch.distributed as dist

        slot = self.launch % self.slots
        if self.asm_done[slot] is not None:
            import torch

            torch.cuda.current_stream().wait_event(self.asm_done[slot])
            self.asm_done[slot] = None
        recv = [b[:n] for b in self.bufs[slot]] if self.bufs[slot] is not None else None
        work = dist.gather(self.tiles_[slot][:n], recv, dst=self.dst, group=self.group, async_op=True)
        self.pending[slot] = (self.k, n, work)
        self.k += n
        self.launch += 1

    def flush(self):
        """Complete every outstanding gather (oldest first); returns ``out``."""
        for i in range(self.slots):
            self._finish((self.launch + i) % self.slots)
        return self.out

    def _finish(self, slot):
        p = self.pending[slot]
        if p is None:
            return
        self.pending[slot] = None
        k, n, work = p
        work.wait()
        if self.rank != self.dst:
            return
        if self.asm is None:
            self._assemble(k, n, slot)
            return
        import torch

        with torch.cuda.stream(self.asm):
            work.wait()
            self._assemble(k, n, slot)
            ev = torch.cuda.Event()
            ev.record(self.asm)
            self.asm_done[slot] = ev

    def _assemble(self, k, n, slot):
        for f in range(n):
            frame = assemble([b[f] for b in self.bufs[slot]], self.height)
            if self.out is None:
                self.out = frame.clone()
            else:
                self.out.copy_(frame)
            if self.on_frame is not None:
                self.on_frame(k + f, self.out)
