"""The multi-GPU frame path over the C ABI (include/mm_comm.h): RCCL
communicators over the renderers' GPUs and the frame-end gather of
interleaved row tiles to rank 0 (north star: "tiles of the framebuffer shard
one-per-GPU ... with a single RCCL gather over xGMI at frame end").

The reference renders on one Metal device (src/main.rs:616) and commits the
frame at src/main.rs:884-894; these are the calls its host makes to drive N
GPUs instead.  Everything here is a thin binding: the transport (RCCL
send/recv, one group per gather), the staging and the de-interleave kernel
are libmirror_maze.so's (csrc/mm_comm.hip).

* one process per GPU: ``Comm.unique_id(renderer)`` on rank 0, shared by the
  caller's rendezvous (bench.py: torch.distributed's gloo broadcast), then
  ``Comm.init_rank(renderer, n, rank, uid)`` on every rank;
* one process for N GPUs: ``Comm.init_all(renderers)`` and
  ``gather_rows_all``.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import check, lib


def row_shard(height: int, n_ranks: int, rank: int):
    """(y0, y_stride, rows, rows_max) of rank's interleaved row set (mm_row_shard)."""
    v = [C.c_uint32() for _ in range(4)]
    rc = lib().mm_row_shard(height, n_ranks, rank, *(C.byref(x) for x in v))
    if rc != _lib.MM_OK:
        raise ValueError(f"mm_row_shard({height}, {n_ranks}, {rank}) failed")
    return tuple(x.value for x in v)


def _stream_of(renderer, stream):
    """hipStream_t handle for a call: `stream` (torch stream or int) if given,
    else the renderer's pinned stream, else torch's current stream."""
    import torch

    if stream is not None:
        return int(getattr(stream, "cuda_stream", stream))
    if renderer._pinned_stream:
        h = C.c_void_p()
        check(lib().mm_get_stream(renderer._ctx, C.byref(h)), renderer._ctx)
        return h.value
    return torch.cuda.current_stream(renderer.device).cuda_stream


class _OnStream:
    """Enqueue the renderer's next C-ABI calls on `handle`, then restore."""

    def __init__(self, renderer, handle):
        self.r, self.h = renderer, handle

    def __enter__(self):
        old = C.c_void_p()
        check(lib().mm_get_stream(self.r._ctx, C.byref(old)), self.r._ctx)
        self.old = old.value
        check(lib().mm_set_stream(self.r._ctx, self.h), self.r._ctx)
        return self

    def __exit__(self, *exc):
        lib().mm_set_stream(self.r._ctx, self.old)


def _tile_shape(t, height: int = 0, n_ranks: int = 0):
    """(n_frames, rows_max, width, bytes_per_px) of a (F, rows_max, W, C) or
    (rows_max, W, C) contiguous CUDA tensor.  With height and n_ranks, the
    tile must hold exactly rows_max = ceil(height / n_ranks) rows: the C side
    sizes every rank's slab from the height alone, so a shorter tile (a
    ragged rank's tile[:rows]) would be read past its end."""
    if not (t.is_cuda and t.is_contiguous()):
        raise ValueError("tiles must be contiguous CUDA tensors")
    shape = tuple(t.shape) if t.dim() == 4 else (1,) + tuple(t.shape)
    if len(shape) != 4:
        raise ValueError("tile must be (frames, rows, width, channels) or (rows, width, channels)")
    if n_ranks:
        rm = row_shard(height, n_ranks, 0)[3]
        if shape[1] != rm:
            raise ValueError(f"tile has {shape[1]} rows; every rank's tile must hold rows_max = {rm} rows "
                             f"(height {height} over {n_ranks} ranks; pad the short ranks' tiles)")
    return shape[0], shape[1], shape[2], shape[3] * t.element_size()


def _check_out(out, tile, nf: int, height: int):
    """rank 0's frame buffer: contiguous CUDA, the tile's dtype, (nf, height, W, C) elements."""
    if not (out.is_cuda and out.is_contiguous() and out.dtype == tile.dtype
            and out.numel() == nf * height * tile.shape[-2] * tile.shape[-1]):
        raise ValueError("out must be a contiguous (frames, height, width, channels) tensor of the tile dtype")


class Comm:
    """An RCCL communicator of the library (mm_comm), bound to one renderer's GPU."""

    def __init__(self, handle: int, renderer):
        self._h = C.c_void_p(handle)
        self.renderer = renderer
        rank, n, dev = C.c_int(), C.c_int(), C.c_int()
        check(lib().mm_comm_info(self._h, C.byref(rank), C.byref(n), C.byref(dev)))
        self.rank, self.n_ranks, self.device = rank.value, n.value, dev.value

    @staticmethod
    def unique_id(renderer) -> bytes:
        buf = (C.c_uint8 * _lib.MM_COMM_ID_BYTES)()
        check(lib().mm_comm_unique_id(renderer._ctx, buf), renderer._ctx)
        return bytes(buf)

    @classmethod
    def init_rank(cls, renderer, n_ranks: int, rank: int, uid: bytes) -> "Comm":
        """Join the communicator `uid` (collective: returns once all n_ranks joined)."""
        if len(uid) != _lib.MM_COMM_ID_BYTES:
            raise ValueError("uid must be MM_COMM_ID_BYTES bytes")
        buf = (C.c_uint8 * _lib.MM_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().mm_comm_init_rank(renderer._ctx, n_ranks, rank, buf, C.byref(h)), renderer._ctx)
        return cls(h.value, renderer)

    @classmethod
    def init_all(cls, renderers) -> list:
        """One communicator per renderer (one process, distinct GPUs); rank i = renderers[i]."""
        n = len(renderers)
        ctxs = (C.c_void_p * n)(*[r._ctx.value for r in renderers])
        hs = (C.c_void_p * n)()
        check(lib().mm_comm_init_all(n, ctxs, hs), renderers[0]._ctx)
        return [cls(hs[i], renderers[i]) for i in range(n)]

    @staticmethod
    def rccl_version() -> int:
        return lib().mm_comm_rccl_version()

    @staticmethod
    def rccl_header_version() -> int:
        return lib().mm_comm_rccl_header_version()

    def gather_rows(self, tile, height: int, out=None, stream=None, self_via_rccl: bool = False):
        """Frame-end gather (mm_gather_rows) of this rank's tile -- (F, rows_max,
        W, C) or (rows_max, W, C), rows rank, rank + N, ... of each frame -- into
        `out` on rank 0, a (F, height, W, C) tensor of the tile's dtype
        (allocated if None); other ranks return None.  Enqueued on `stream`
        (default: the renderer's stream, or torch's current one)."""
        import torch

        nf, rows_max, w, bpp = _tile_shape(tile, height, self.n_ranks)
        if self.rank == 0:
            if out is None:
                out = torch.empty((nf, height) + tuple(tile.shape[-2:]), dtype=tile.dtype, device=tile.device)
            else:
                _check_out(out, tile, nf, height)
        flags = _lib.MM_GATHER_SELF_VIA_RCCL if self_via_rccl else 0
        r = self.renderer
        with _OnStream(r, _stream_of(r, stream)):
            check(lib().mm_gather_rows(r._ctx, self._h, tile.data_ptr(), nf, w, height, bpp,
                                       out.data_ptr() if self.rank == 0 else None, flags), r._ctx)
        return out if self.rank == 0 else None

    def close(self) -> None:
        """Destroy the communicator (explicitly: RCCL teardown from a finaliser
        at interpreter exit could run after the HIP runtime's)."""
        if self._h:
            lib().mm_comm_destroy(self._h)
            self._h = C.c_void_p()


def gather_rows_all(comms, tiles, height: int, out=None, self_via_rccl: bool = False):
    """mm_gather_rows_all: every rank's tile (tiles[i] on comms[i]'s GPU) to
    rank 0's `out` in one RCCL group, from one process.  Each rank's part is
    enqueued on its renderer's stream (pinned, or torch's current stream of
    that device)."""
    import torch

    n = len(comms)
    if len(tiles) != n:
        raise ValueError("one tile per communicator")
    root = [c.rank for c in comms].index(0)
    t = tiles[root]
    nf, rows_max, w, bpp = _tile_shape(t, height, n)
    for i, ti in enumerate(tiles):  # every rank's tile: the root's shape and dtype (the C side assumes it)
        if tuple(ti.shape) != tuple(t.shape) or ti.dtype != t.dtype or ti.device.index != comms[i].renderer.device:
            raise ValueError(f"tile {i}: every rank's tile must have the root tile's shape and dtype, "
                             f"on its communicator's GPU")
        _tile_shape(ti, height, n)
    if out is None:
        out = torch.empty((nf, height) + tuple(t.shape[-2:]), dtype=t.dtype, device=t.device)
    else:
        _check_out(out, t, nf, height)
    rens = [c.renderer for c in comms]
    ctxs = (C.c_void_p * n)(*[r._ctx.value for r in rens])
    hs = (C.c_void_p * n)(*[c._h.value for c in comms])
    ptrs = (C.c_void_p * n)(*[t.data_ptr() for t in tiles])
    guards = [_OnStream(r, _stream_of(r, None)) for r in rens]
    for g in guards:
        g.__enter__()
    try:
        check(lib().mm_gather_rows_all(n, ctxs, hs, ptrs, nf, w, height, bpp, out.data_ptr(),
                                       _lib.MM_GATHER_SELF_VIA_RCCL if self_via_rccl else 0), rens[root]._ctx)
    finally:
        for g in guards:
            g.__exit__()
    return out


def assemble_rows(renderer, tiles, height: int, out=None, stream=None):
    """mm_assemble_rows: (N, F, rows_max, W, C) tiles of N ranks on one GPU ->
    (F, height, W, C) frames (the gather's de-interleave alone)."""
    import torch

    if tiles.dim() != 5 or not (tiles.is_cuda and tiles.is_contiguous()):
        raise ValueError("tiles must be a contiguous (ranks, frames, rows_max, width, channels) CUDA tensor")
    n, nf, rows_max, w, ch = tiles.shape
    if rows_max != row_shard(height, n, 0)[3]:
        raise ValueError(f"tiles hold {rows_max} rows; {n} ranks of a {height}-row frame need rows_max = "
                         f"{row_shard(height, n, 0)[3]}")
    if out is None:
        out = torch.empty((nf, height, w, ch), dtype=tiles.dtype, device=tiles.device)
    else:
        _check_out(out, tiles[0], nf, height)
    with _OnStream(renderer, _stream_of(renderer, stream)):
        check(lib().mm_assemble_rows(renderer._ctx, tiles.data_ptr(), n, nf, w, height, ch * tiles.element_size(),
                                     out.data_ptr()), renderer._ctx)
    return out


class NativeGatherer:
    """bench.py's frame path over the library's gather (one per multi-frame
    launch, or per frame with n = 1): ``tiles(n)`` hands out the (n, rows_max,
    W, C) slice of a rotating slot buffer the launch's frames go into (after
    the gather that last read the slot is done), ``put(n)`` issues the gather
    on ``gather_stream`` once the current stream's work on the tiles is done,
    so the next launch's trace does not wait for it; ``flush()`` makes the
    current stream wait for every gather and returns rank 0's last frame."""

    def __init__(self, comm: Comm, shape, height: int, max_frames: int, device, dtype=None, slots: int = 2,
                 gather_stream=None):
        import torch

        self.comm, self.height, self.max_frames, self.slots = comm, height, max_frames, slots
        dtype = torch.uint8 if dtype is None else dtype
        self.tiles_ = [torch.zeros((max_frames,) + tuple(shape), dtype=dtype, device=device) for _ in range(slots)]
        self.frames = ([torch.empty((max_frames, height) + tuple(shape[1:]), dtype=dtype, device=device)
                        for _ in range(slots)] if comm.rank == 0 else None)
        self.stream = gather_stream if gather_stream is not None else torch.cuda.Stream(device)
        self.done = [None] * slots
        self.launch = 0
        self.k = 0
        self.last = None  # (slot, n) of the last gather issued

    def tiles(self, n: int):
        import torch

        if not (1 <= n <= self.max_frames):
            raise ValueError(f"batch of {n} frames outside 1..{self.max_frames}")
        slot = self.launch % self.slots
        if self.done[slot] is not None:  # the gather that last read this slot
            torch.cuda.current_stream().wait_event(self.done[slot])
        return self.tiles_[slot][:n]

    def put(self, n: int):
        import torch

        slot = self.launch % self.slots
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        self.stream.wait_event(ready)
        out = self.frames[slot][:n] if self.frames is not None else None
        self.comm.gather_rows(self.tiles_[slot][:n], self.height, out=out, stream=self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.done[slot] = ev
        self.last = (slot, n)
        self.launch += 1
        self.k += n

    def flush(self):
        """The current stream waits for every issued gather; rank 0's last
        delivered frame (None before any gather, and on other ranks)."""
        import torch

        for ev in self.done:
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
        if self.frames is None or self.last is None:
            return None
        slot, n = self.last
        return self.frames[slot][n - 1]


class HostComm:
    """Diagnostics transport with Comm's interface, for N ranks that share ONE
    GPU (bench.py --shared-gpu).  RCCL refuses two ranks on one device, so
    here the tiles cross between the ranks' processes as host copies over
    torch.distributed point-to-point (gloo), and rank 0 de-interleaves them
    with the library's mm_assemble_rows -- the kernel mm_gather_rows ends in.
    Everything around it (NativeGatherer's slots and events, the rank >= 1
    branches of bench.py, the exposed-gather clock, the reductions) is the
    product's N-GPU path unchanged, so one GPU box can execute it end to end.
    Not a product transport: its host round trip makes any timing of it
    meaningless."""

    def __init__(self, renderer, n_ranks: int, rank: int, group=None):
        if not (0 <= rank < n_ranks):
            raise ValueError("rank out of range")
        self.renderer, self.n_ranks, self.rank, self.group = renderer, n_ranks, rank, group
        self.device = getattr(renderer, "device", None)

    def exchange(self, host_tile):
        """Every rank's host tile to rank 0 (which gets them in rank order);
        None on the other ranks.  Blocking, torch.distributed send / recv."""
        import torch
        import torch.distributed as dist

        if self.rank != 0:
            dist.send(host_tile, 0, group=self.group)
            return None
        parts = [host_tile] + [torch.empty_like(host_tile) for _ in range(1, self.n_ranks)]
        for r in range(1, self.n_ranks):
            dist.recv(parts[r], r, group=self.group)
        return parts

    def gather_rows(self, tile, height: int, out=None, stream=None, self_via_rccl: bool = False):
        """Comm.gather_rows's contract (same checks, same result on rank 0),
        over the host transport; enqueued on / synchronised with `stream`."""
        import torch

        nf, rows_max, w, bpp = _tile_shape(tile, height, self.n_ranks)
        if self.rank == 0:
            if out is None:
                out = torch.empty((nf, height) + tuple(tile.shape[-2:]), dtype=tile.dtype, device=tile.device)
            else:
                _check_out(out, tile, nf, height)
        t5 = tile if tile.dim() == 4 else tile.unsqueeze(0)
        s = torch.cuda.current_stream(tile.device) if stream is None else stream
        with torch.cuda.stream(s):
            host = t5.cpu()  # (waits for the stream's work on the tile)
        parts = self.exchange(host)
        if self.rank != 0:
            return None
        with torch.cuda.stream(s):
            staged = torch.stack(parts).to(tile.device)  # (N, F, rows_max, W, C)
            assemble_rows(self.renderer, staged, height, out=out.view((nf, height) + tuple(tile.shape[-2:])),
                          stream=s)
        return out

    def close(self) -> None:
        pass
