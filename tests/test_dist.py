"""N>1 framebuffer path on CPU: world_size-2 (and 3) gloo processes shard the
rows, gather to rank 0 and de-interleave; the result must equal the 1-rank
frame exactly.  The tiles are produced by the CPU oracle, so this also checks
that row-interleaved tracing reproduces the full-frame image bit for bit."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, q):
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    sys.path.insert(0, str(repo / "mirror-maze_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.dist import gather_frame, row_shard, rows_max
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    o = Oracle.from_scene(s)
    u = default_uniform(W, H, 0)
    y0, stride, rows = row_shard(H, world, rank)
    tile = np.zeros((rows_max(H, world), W, 4), np.float32)
    o.trace_tile(u, make_ext(2, 3, 15, frame=1), 0, y0, W, rows, y_stride=stride, out=tile[:rows])
    frame = gather_frame(torch.from_numpy(tile), H)
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def _worker_pipelined(rank, world, port, H, W, q, fmt="f32"):
    """Three frames through FrameGatherer (async, double-buffered gathers);
    fmt "rgba8": each rank converts its tile to RGBA8 (the texture format,
    mirror_maze.io.quantize) and the gather moves the uint8 tiles."""
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    sys.path.insert(0, str(repo / "mirror-maze_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.dist import FrameGatherer, row_shard, rows_max
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    o = Oracle.from_scene(s)
    u = default_uniform(W, H, 0)
    y0, stride, rows = row_shard(H, world, rank)
    frames = {}
    g = FrameGatherer((rows_max(H, world), W, 4), H, "cpu", dtype=torch.uint8 if fmt == "rgba8" else None,
                      on_frame=lambda k, fr: frames.__setitem__(k, fr.numpy().copy()))
    for f in range(3):
        t = g.tile().numpy()
        if fmt == "rgba8":
            ft = np.zeros((rows, W, 4), dtype=np.float32)
            o.trace_tile(u, make_ext(2, 3, 15, frame=f), 0, y0, W, rows, y_stride=stride, out=ft)
            t[:rows] = quantize(ft)
        else:
            o.trace_tile(u, make_ext(2, 3, 15, frame=f), 0, y0, W, rows, y_stride=stride, out=t[:rows])
        g.put()
        if rank == 0:
            assert sorted(frames) == list(range(max(0, f - 1)))  # frame k completes when its slot is reused
    out = g.flush()
    if rank == 0:
        assert sorted(frames) == [0, 1, 2] and np.array_equal(out.numpy(), frames[2])
        q.put(np.stack([frames[k] for k in range(3)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fmt", ["f32", "rgba8"])
def test_gloo_pipelined_gather_three_frames(fmt):
    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    world, H, W = 2, 9, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, H, W, q, fmt)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    o = Oracle.from_scene(Scene.build(10, 0))
    for f in range(3):
        ref, _ = o.trace_tile(default_uniform(W, H, 0), make_ext(2, 3, 15, frame=f), 0, 0, W, H)
        if fmt == "rgba8":
            assert frames[f].dtype == np.uint8 and np.array_equal(frames[f], quantize(ref)), f
        else:
            assert np.array_equal(frames[f].view(np.uint32), ref.view(np.uint32)), f


@pytest.mark.parametrize("world,H", [(2, 12), (3, 10)])
def test_gloo_row_sharded_frame_equals_single_rank(world, H):
    import sys
    from pathlib import Path

    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    W = 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref, _ = Oracle.from_scene(Scene.build(10, 0)).trace_tile(default_uniform(W, H, 0), make_ext(2, 3, 15, frame=1),
                                                               0, 0, W, H)
    assert frame.shape == (H, W, 4)
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def test_row_shard_covers_every_row_once():
    from mirror_maze.dist import row_shard, rows_max

    for H in (1, 7, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                y0, st, n = row_shard(H, world, r)
                seen += [y0 + i * st for i in range(n)]
                assert n <= rows_max(H, world)
            assert sorted(seen) == list(range(H))


def _worker_batched(rank, world, port, H, W, q, sizes):
    """Frames in launches of `sizes` frames, one BatchGatherer gather per launch
    (bench.py's multi-frame path); RGBA8 tiles as bench.py delivers them."""
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    sys.path.insert(0, str(repo / "mirror-maze_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.dist import BatchGatherer, row_shard, rows_max
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    o = Oracle.from_scene(s)
    u = default_uniform(W, H, 0)
    y0, stride, rows = row_shard(H, world, rank)
    frames = {}
    g = BatchGatherer((rows_max(H, world), W, 4), H, "cpu", max(sizes), dtype=torch.uint8,
                      on_frame=lambda k, fr: frames.__setitem__(k, fr.numpy().copy()))
    f0 = 0
    for n in sizes:
        tl = g.tiles(n).numpy()
        for f in range(n):
            ft = np.zeros((rows, W, 4), dtype=np.float32)
            o.trace_tile(u, make_ext(2, 3, 15, frame=f0 + f), 0, y0, W, rows, y_stride=stride, out=ft)
            tl[f, :rows] = quantize(ft)
        g.put(n)
        f0 += n
    out = g.flush()
    if rank == 0:
        assert sorted(frames) == list(range(f0)) and np.array_equal(out.numpy(), frames[f0 - 1])
        q.put(np.stack([frames[k] for k in range(f0)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, (3, 3, 2)), (3, (4, 1))])
def test_gloo_batch_gather_per_launch(world, sizes):
    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    H, W = 11, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_batched, args=(r, world, port, H, W, q, sizes)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    o = Oracle.from_scene(Scene.build(10, 0))
    assert frames.shape == (sum(sizes), H, W, 4)
    for f in range(sum(sizes)):
        ref, _ = o.trace_tile(default_uniform(W, H, 0), make_ext(2, 3, 15, frame=f), 0, 0, W, H)
        assert frames[f].dtype == np.uint8 and np.array_equal(frames[f], quantize(ref)), f


@pytest.mark.parametrize("height,world", [(1080, 8), (1080, 7), (2160, 3), (5, 8), (1, 1)])
def test_row_shard_c_abi_matches_python(height, world):
    """mm_row_shard (include/mm_comm.h, the split a Rust host would call) and
    mirror_maze.dist.row_shard / rows_max name the same rows for every rank,
    and the ranks' row sets partition the frame."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "mirror-maze_amd"))
    from mirror_maze.comm import row_shard as c_shard
    from mirror_maze.dist import row_shard, rows_max

    seen = []
    for rank in range(world):
        y0, stride, rows, rm = c_shard(height, world, rank)
        assert (y0, stride, rows) == row_shard(height, world, rank) and rm == rows_max(height, world)
        seen += list(range(y0, height, stride))[:rows]
        assert rows <= rm
    assert sorted(seen) == list(range(height))
