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
    ap.add_argument("--overlap", nargs="?", const="prio", default=None, choices=["prio", "own"],
                    help="alternate frames over two contexts on two streams (tail of frame k overlaps frame k+1)")
    ap.add_argument("--gate", type=int, default=1, help="with --overlap own: MM_OPT_TAIL_GATE")
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    if a.overlap:
        return overlap(a, r, maze_n, W, H, spp, bl, ml, desc)
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


def overlap(a, r0, maze_n, W, H, spp, bl, ml, desc):
    import torch

    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze.dist import row_shard, rows_max

    r1 = Renderer(0)
    r1.upload_scene(Scene.build(maze_n, 0))
    rens = [r0, r1]
    if a.overlap == "own":  # the contexts' own library streams (equal priority)
        streams = [r.own_stream() for r in rens]
        if a.gate:
            for r in rens:
                r.set_option(13, 1)  # MM_OPT_TAIL_GATE
    else:
        streams = [torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=0)]
    u = default_uniform(W, H, 0)
    print(f"# {desc} -- frames alternate over two contexts / streams")
    t1 = None
    for n in (int(x) for x in a.ranks.split(",")):
        y0, stride, rows = row_shard(H, n, 0)
        outs = [torch.zeros((rows_max(H, n), W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
        for k in range(2):
            with torch.cuda.stream(streams[k]):
                rens[k].trace_tile(u, make_ext(spp, bl, ml, frame=99), 0, y0, W, rows, y_stride=stride, out=outs[k][:rows])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(a.frames):
            k = f & 1
            with torch.cuda.stream(streams[k]):
                rens[k].trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, y0, W, rows, y_stride=stride, out=outs[k][:rows])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        if t1 is None:
            t1 = wall
        print(f"N={n}: rank-0 rows {rows:5d}  wall {wall:8.3f} ms/frame  ideal {t1 / n:8.3f} ms  "
              f"efficiency {t1 / (n * wall):.3f}", flush=True)
    r1.close()
    r0.close()


if __name__ == "__main__":
    main()
