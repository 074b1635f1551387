"""Render frames through the multi-GPU path: rows interleaved over the ranks
of a torch.distributed.run job, every frame gathered to rank 0 by the
library's RCCL communicator (mm_comm_init_rank + mm_gather_rows,
include/mm_comm.h -- the single frame-end collective of SURVEY.md §8e,
replacing the reference's single device, src/main.rs:616).  torch.distributed
(gloo) only carries the communicator's unique id.  Rank 0's own tile goes
through RCCL's self send/recv too (MM_GATHER_SELF_VIA_RCCL), so one rank on
one GPU exercises the transport.  Rank 0 writes the assembled frames to --out
(.npy, float32 [F, H, W, 4]) and the RCCL library it mapped to --out +
".maps.txt".

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P scripts/rccl_frames.py --config c1 --frames 2 --out f.npy
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze.comm import Comm, row_shard

    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    maze_n, W, H, spp, bl, ml, _ = CONFIGS[a.config]
    scene = Scene.build(maze_n, 0)
    r = Renderer(local)
    r.upload_scene(scene)
    uid = [Comm.unique_id(r) if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = Comm.init_rank(r, world, rank, uid[0])
    u = default_uniform(W, H, 0)
    y0, stride, rows, rm = row_shard(H, world, rank)
    frames = []
    tile = torch.zeros((rm, W, 4), dtype=torch.float32, device=dev)
    for f in range(a.frames):
        r.trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, y0, W, rows, y_stride=stride, out=tile[:rows])
        out = comm.gather_rows(tile, H, self_via_rccl=True)
        if rank == 0:
            frames.append(out[0].cpu().numpy().copy())
    torch.cuda.synchronize()
    if rank == 0:
        np.save(a.out, np.stack(frames))
        maps = [ln.split()[-1] for ln in open("/proc/self/maps") if "rccl" in ln]
        Path(a.out + ".maps.txt").write_text("\n".join(sorted(set(maps))) + "\n")
    dist.barrier()
    comm.close()
    r.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
