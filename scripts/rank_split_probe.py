"""Per-rank launch time of an 8-way C3 split on one GPU, for every rank, with
the interleaved row sets bench.py uses (rows r, r+8, ...) and with contiguous
bands (rows r*135 .. r*135+134) -- is rank 0 of 8 slower per ray than 1/8 of
the frame because of the rows it holds, the split's shape, or the launch's
length?  (profiles/r04/tail_probe: rank 0 of 8's chunks run ~5 % longer than
N=1's.)  HIP-event kernel time per 20-frame launch, after a warm-up launch.

    python scripts/rank_split_probe.py [--config c3] [--frames 20] [--reps 2]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mirror-maze_amd"))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    N = a.ranks
    band = (H + N - 1) // N
    out = torch.zeros((a.frames, band, W, 4), dtype=torch.float32, device="cuda")
    full = torch.zeros((a.frames, H, W, 4), dtype=torch.float32, device="cuda")

    def run(y0, rows, stride, buf):
        r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, y0, W, rows, y_stride=stride, out=buf)

    run(0, H, 1, full)  # warm-up, sizes the context's buffers
    r.sync()
    r.set_profiling(True)

    def timed(y0, rows, stride, buf):
        ms = []
        for _ in range(a.reps):
            r.kernel_timing(reset=True)
            run(y0, rows, stride, buf)
            r.sync()
            ms.append(r.kernel_timing(reset=True)[0])
        return statistics.median(ms)

    print(f"# {desc}; {a.frames} frames per launch; kernel ms per launch (median of {a.reps})", flush=True)
    t1 = timed(0, H, 1, full)
    print(f"N=1: {t1:.3f} ms; / {N} = {t1 / N:.3f}", flush=True)
    for kind in ("interleaved", "contiguous"):
        ts = []
        for k in range(N):
            if kind == "interleaved":
                y0, stride, rows = k, N, len(range(k, H, N))
            else:
                y0, stride, rows = k * band, 1, max(0, min(band, H - k * band))
            ts.append(timed(y0, rows, stride, out))
        print(f"{kind:11s}: " + " ".join(f"{t:.3f}" for t in ts) +
              f"  | max {max(ts):.3f} (eff {t1 / N / max(ts):.3f}), sum / N = {sum(ts) / N:.3f} "
              f"(sum / N=1 {sum(ts) / t1:.3f})", flush=True)


if __name__ == "__main__":
    main()
