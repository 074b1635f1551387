"""The multi-GPU frame path of the C ABI (include/mm_comm.h) on the MI355X,
through ctypes: RCCL communicators (one process per GPU, and one process for
all GPUs), the frame-end gather and the de-interleave.  The reference has one
Metal device (src/main.rs:616) and commits each frame at src/main.rs:884-894;
an N-GPU frame assembled here must equal trace_tile's 1-GPU frame bit for bit
(the RNG is keyed on (pixel, sample, frame)).

One box has one GPU, so the transport runs at one rank (RCCL allows one rank
per GPU): MM_GATHER_SELF_VIA_RCCL routes rank 0's own tile through ncclSend /
ncclRecv so the RCCL data path is exercised; the N-rank row bookkeeping is
checked by tracing N ranks' tiles on the one GPU and assembling them with
mm_assemble_rows (the same kernel the gather ends in)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame_setup(cfg):
    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    maze_n, W, H, spp, bl, ml, _ = CONFIGS[cfg]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    return r, default_uniform(W, H, 0), make_ext(spp, bl, ml, frame=3), W, H


@pytest.mark.parametrize("cfg,n_ranks", [("c1", 8), ("c1", 7), ("c2", 8), ("c2", 3)])
def test_assembled_rank_tiles_equal_the_whole_frame(gpu, cfg, n_ranks):
    """Each of N ranks' interleaved row sets traced into its own tile (rows
    rank, rank + N, ...; ragged when H % N != 0), the N tiles de-interleaved
    by mm_assemble_rows: float and RGBA8 frames equal trace_tile's whole frame
    bit for bit."""
    import torch

    from mirror_maze.comm import assemble_rows, row_shard

    r, u, e, W, H = _frame_setup(cfg)
    rm = row_shard(H, n_ranks, 0)[3]
    tiles = torch.zeros((n_ranks, 1, rm, W, 4), dtype=torch.float32, device="cuda")
    for k in range(n_ranks):
        y0, stride, rows, _ = row_shard(H, n_ranks, k)
        r.trace_tile(u, e, 0, y0, W, rows, y_stride=stride, out=tiles[k, 0, :rows])
    got = assemble_rows(r, tiles, H)
    want, _ = r.trace_tile(u, e, 0, 0, W, H)
    torch.cuda.synchronize()
    assert torch.equal(got[0].view(torch.int32), want.view(torch.int32))
    got8 = assemble_rows(r, r.quantize(tiles), H)
    assert torch.equal(got8[0], r.quantize(want))
    r.close()


@pytest.mark.parametrize("self_via_rccl", [False, True])
def test_comm_init_rank_gather_equals_trace_tile(gpu, self_via_rccl):
    """One process per GPU at N = 1: mm_comm_unique_id + mm_comm_init_rank,
    then mm_gather_rows of a 3-frame RGBA8 tile (one multi-frame launch) into
    rank 0's frames -- with the root's tile straight from its buffer, and
    through RCCL send/recv to itself."""
    import torch

    from mirror_maze import make_ext
    from mirror_maze.comm import Comm

    r, u, e, W, H = _frame_setup("c2")
    comm = Comm.init_rank(r, 1, 0, Comm.unique_id(r))
    assert (comm.rank, comm.n_ranks, comm.device) == (0, 1, 0)
    assert Comm.rccl_version() >= 22600
    frames, _ = r.trace_tile_frames(u, make_ext(e.spp, e.bounce_limit, e.mirror_limit, frame=5), 3, 0, 0, W, H)
    tile8 = r.quantize(frames)
    out = comm.gather_rows(tile8, H, self_via_rccl=self_via_rccl)
    torch.cuda.synchronize()
    assert out.shape == (3, H, W, 4)
    for f in range(3):
        want, _ = r.trace_tile(u, make_ext(e.spp, e.bounce_limit, e.mirror_limit, frame=5 + f), 0, 0, W, H)
        assert torch.equal(out[f], r.quantize(want)), f
    comm.close()
    r.close()


def test_comm_init_all_and_gather_rows_all(gpu):
    """One process driving the node's GPUs (here its one): mm_comm_init_all
    over the contexts, mm_gather_rows_all in one RCCL group, float tiles
    (16 B/px) through RCCL's self send/recv."""
    import torch

    from mirror_maze.comm import Comm, gather_rows_all

    r, u, e, W, H = _frame_setup("c1")
    comms = Comm.init_all([r])
    assert [(c.rank, c.n_ranks) for c in comms] == [(0, 1)]
    tile, _ = r.trace_tile(u, e, 0, 0, W, H)
    for via in (False, True):
        out = gather_rows_all(comms, [tile], H, self_via_rccl=via)
        torch.cuda.synchronize()
        assert torch.equal(out[0].view(torch.int32), tile.view(torch.int32)), via
    for c in comms:
        c.close()
    r.close()


def test_gather_argument_errors_are_codes(gpu):
    """Shape and communicator mistakes come back as MM_ERR_INVALID with a
    message, before any RCCL call."""
    import ctypes as C

    import torch

    from mirror_maze import MMError, lib
    from mirror_maze.comm import Comm

    r, u, e, W, H = _frame_setup("c1")
    comm = Comm.init_rank(r, 1, 0, Comm.unique_id(r))
    tile = torch.zeros((1, H, W, 4), dtype=torch.uint8, device="cuda")
    from mirror_maze._lib import check

    with pytest.raises(MMError) as ei:
        check(lib().mm_gather_rows(r._ctx, comm._h, tile.data_ptr(), 1, W, H, 4, None, 0), r._ctx)
    assert "rank 0 needs frame_dev" in str(ei.value)
    assert lib().mm_gather_rows(r._ctx, comm._h, tile.data_ptr(), 0, W, H, 4, tile.data_ptr(), 0) == -1
    assert lib().mm_gather_rows(r._ctx, None, tile.data_ptr(), 1, W, H, 4, tile.data_ptr(), 0) == -1
    assert lib().mm_comm_init_rank(r._ctx, 2, 2, (C.c_uint8 * 128)(), C.byref(C.c_void_p())) == -1
    comm.close()
    r.close()
