#!/usr/bin/env python
"""Single-GPU probe of the strong-scaling split: time the trace of rank 0's
row set (rows 0, N, 2N, ...) for N = 1, 2, 4, 8 and report the per-rank
kernel time against T1 / N.  Everything except the frame-end gather (tens of
microseconds over xGMI) is what one rank of `bench.py --gpus N` executes.

    python scripts/scaling_probe.py [--config c3] [--frames 5]
"""
import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze.dist import row_shard, rows_max

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--ranks", default="1,2,4,8")
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    print(f"# {desc}")
    t1 = None
    for n in (int(x) for x in a.ranks.split(",")):
        y0, stride, rows = row_shard(H, n, 0)
        out = torch.zeros((rows_max(H, n), W, 4), dtype=torch.float32, device="cuda")
        r.trace_tile(u, make_ext(spp, bl, ml, frame=99), 0, y0, W, rows, y_stride=stride, out=out[:rows])
        torch.cuda.synchronize()
        r.set_profiling(True)
        r.kernel_timing(reset=True)
        t0 = time.perf_counter()
        for f in range(a.frames):
            r.trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, y0, W, rows, y_stride=stride, out=out[:rows])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        kms, kn = r.kernel_timing(reset=True)
        r.set_profiling(False)
        k = kms / max(kn, 1)
        if t1 is None:
            t1 = wall
        print(f"N={n}: rank-0 rows {rows:5d}  trace {k:8.3f} ms  wall {wall:8.3f} ms  "
              f"ideal {t1 / n:8.3f} ms  efficiency {t1 / (n * wall):.3f}", flush=True)
    r.close()


if __name__ == "__main__":
    main()
