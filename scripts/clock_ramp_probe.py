"""Is rank 0 of an N-way split slower per ray than 1/N of the whole frame
because of what precedes its launch?  (the emulated N=8
efficiency; profiles/r04/tail_probe: rank 0 of 8's chunks run 5 % longer than
N=1's.)  Times one 20-frame launch of a tile in three settings:

  idle      after 100 ms with the GPU idle
  busy      right after ~50 ms of GEMMs on the device (synchronised, then launched)
  queued    the mean of 4 launches queued back to back (the first after idle)

for rank 0 of 1 and of 8 (interleaved rows, as bench.py --gpus 8).  HIP-event
kernel time per launch (mm_kernel_timing).

    python scripts/clock_ramp_probe.py [--config c3] [--frames 20] [--reps 3]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mirror-maze_amd"))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze.dist import row_shard

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ranks", default="1,8")
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    print(f"# {desc}; {a.frames} frames per launch; kernel ms per launch (HIP events)", flush=True)
    for n in [int(v) for v in a.ranks.split(",")]:
        y0, stride, rows = row_shard(H, n, 0)
        out = torch.zeros((a.frames, rows, W, 4), dtype=torch.float32, device="cuda")

        def launch():
            r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, y0, W, rows, y_stride=stride, out=out)

        launch()  # sizes the context's buffers
        r.sync()
        r.set_profiling(True)
        res = {"idle": [], "busy": [], "queued": []}
        for _ in range(a.reps):
            time.sleep(0.1)
            r.kernel_timing(reset=True)
            launch()
            r.sync()
            res["idle"].append(r.kernel_timing(reset=True)[0])
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.05:
                for _ in range(4):
                    x @ x
                torch.cuda.synchronize()
            launch()
            r.sync()
            res["busy"].append(r.kernel_timing(reset=True)[0])
            time.sleep(0.1)
            for _ in range(4):
                launch()
            r.sync()
            ms, k = r.kernel_timing(reset=True)
            res["queued"].append(ms / k)
        line = "  ".join(f"{m} {statistics.median(v):8.3f} ms ({statistics.median(v) / a.frames:.4f}/frame)"
                         for m, v in res.items())
        print(f"rank 0 of {n} ({rows} rows): {line}", flush=True)
        r.set_profiling(False)
        del out


if __name__ == "__main__":
    main()
