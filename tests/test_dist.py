"""N>1 framebuffer path on CPU, world_size 2 and 3 gloo processes: the row
split every rank renders (mirror_maze.dist.row_shard, mm_row_shard) and the
host transport of bench.py's --shared-gpu diagnostics mode
(mirror_maze.comm.HostComm.exchange: every rank's tiles reach rank 0 intact,
in rank order).  The tiles are the CPU oracle's interleaved row sets, as
bench.py's N-rank launches write them (F frames per launch, RGBA8); rank 0's
de-interleave of what arrived must equal the 1-rank frames bit for bit.  The
device side of the path (NativeGatherer's slots and events, mm_gather_rows /
mm_assemble_rows, bench.py's rank >= 1 branches) runs on the GPU box:
tests/test_gpu_rccl.py (bench.py --shared-gpu at N = 2 and 8)."""
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


def _worker_exchange(rank, world, port, H, W, q, sizes):
    """Frames in launches of `sizes` frames; each launch's (n, rows_max, W, 4)
    RGBA8 tile goes to rank 0 through HostComm.exchange (one exchange per
    launch, as bench.py's NativeGatherer issues one gather per launch)."""
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    sys.path.insert(0, str(repo / "mirror-maze_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.comm import HostComm
    from mirror_maze.dist import assemble, row_shard, rows_max
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    o = Oracle.from_scene(s)
    u = default_uniform(W, H, 0)
    y0, stride, rows = row_shard(H, world, rank)
    hc = HostComm(None, world, rank)
    frames, f0 = [], 0
    for n in sizes:
        tile = np.zeros((n, rows_max(H, world), W, 4), np.uint8)
        for f in range(n):
            ft = np.zeros((rows, W, 4), dtype=np.float32)
            o.trace_tile(u, make_ext(2, 3, 15, frame=f0 + f), 0, y0, W, rows, y_stride=stride, out=ft)
            tile[f, :rows] = quantize(ft)
        parts = hc.exchange(torch.from_numpy(tile))
        if rank == 0:
            assert len(parts) == world and all(tuple(p.shape) == tile.shape for p in parts)
            assert np.array_equal(parts[0].numpy(), tile)  # its own tile, untouched
            frames += [assemble([p[f] for p in parts], H).numpy() for f in range(n)]
        else:
            assert parts is None
        f0 += n
    if rank == 0:
        q.put(np.stack(frames))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,sizes", [(2, 12, (3, 3, 2)), (3, 10, (4, 1)), (3, 11, (1,))])
def test_gloo_host_transport_delivers_every_rank_tile(world, H, sizes):
    from mirror_maze import Scene, default_uniform, make_ext
    from mirror_maze.io import quantize
    from oracle.oracle import Oracle

    W = 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_exchange, args=(r, world, port, H, W, q, sizes)) for r in range(world)]
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


def test_host_transport_rank_checks():
    from mirror_maze.comm import HostComm

    with pytest.raises(ValueError):
        HostComm(None, 2, 2)
    with pytest.raises(ValueError):
        HostComm(None, 2, -1)


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
