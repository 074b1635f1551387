"""The frame-end gather's parts that one GPU can time (VERDICT r04 "what's
weak" 6: multi-GPU efficiency inferred, the gather never timed).

  * the de-interleave kernel alone (mm_assemble_rows) at the SCALE run's shape:
    rank 0 assembling N = 8 ranks' RGBA8 tiles of 20 C3 frames (166 MB read,
    166 MB written);
  * mm_gather_rows through an RCCL communicator at one rank with the root's
    tile routed through ncclSend / ncclRecv to itself
    (MM_GATHER_SELF_VIA_RCCL): RCCL's launch and copy cost for one rank's
    20-frame RGBA8 tile (20.7 MB at N = 8) -- a device-local copy, not xGMI;
  * the same gather without RCCL (the root's own rows only: what rank 0 does
    for its own tile at any N).

HIP events on the stream the work is queued on; median of 10 after 2 warm-ups.
Prints one JSON object (profiles/r05/gather_probe.json).

    python scripts/gather_probe.py
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))


def timed(fn, stream, reps=10, warm=2):
    import torch

    out = []
    for i in range(warm + reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        if i >= warm:
            out.append(e0.elapsed_time(e1))
    return statistics.median(out), min(out)


def main():
    import torch

    from mirror_maze import Renderer
    from mirror_maze.comm import Comm, assemble_rows, row_shard

    W, H, F, N = 1920, 1080, 20, 8
    rm = row_shard(H, N, 0)[3]
    r = Renderer(0)
    s = torch.cuda.Stream()
    res = {"shape": f"{N} ranks x {F} frames x {rm} rows x {W} px x 4 B (C3, RGBA8)"}
    with torch.cuda.stream(s):
        tiles = torch.randint(0, 255, (N, F, rm, W, 4), dtype=torch.uint8, device="cuda")
        frames = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
        med, best = timed(lambda: assemble_rows(r, tiles, H, out=frames, stream=s), s)
        nbytes = 2 * F * H * W * 4
        res["assemble_ms"] = round(med, 4)
        res["assemble_gbs"] = round(nbytes / (best * 1e-3) / 1e9, 1)
        # bit check of the assembly against the row rule
        f, y = 7, 517
        assert torch.equal(frames[f, y], tiles[y % N, f, y // N])
        comm = Comm.init_rank(r, 1, 0, Comm.unique_id(r))
        tile = tiles[0].contiguous()          # one rank's 20-frame tile (20.7 MB)
        out1 = torch.empty((F, rm, W, 4), dtype=torch.uint8, device="cuda")
        med_r, best_r = timed(lambda: comm.gather_rows(tile, rm, out=out1, stream=s, self_via_rccl=True), s)
        med_l, best_l = timed(lambda: comm.gather_rows(tile, rm, out=out1, stream=s, self_via_rccl=False), s)
        assert torch.equal(out1, tile)
        tb = tile.numel()
        res["rccl_self_gather_ms"] = round(med_r, 4)
        res["rccl_self_gather_gbs"] = round(tb / (best_r * 1e-3) / 1e9, 1)
        res["local_gather_ms"] = round(med_l, 4)
        res["rccl_version"] = Comm.rccl_version()
        torch.cuda.synchronize()
        comm.close()
    r.close()
    res["note"] = ("rank 0 at N = 8 receives 7 tiles of the rccl_self size over 7 xGMI links in parallel, then "
                   "runs the assemble; the xGMI transfer itself is the first SCALE run's to measure")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
