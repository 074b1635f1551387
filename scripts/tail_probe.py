#!/usr/bin/env python
"""Per-wave timeline of the mirror-tail kernel (diagnostics build
-DMM_TAIL_TIMELINE): when its waves start, finish and how many 64-path
chunks each ran, for one multi-frame launch.

    bash scripts/build_variant.sh tailtl wt -DMM_TAIL_TIMELINE
    MIRROR_MAZE_LIB=exp/tailtl/lib.so python scripts/tail_probe.py [--config c3] [--frames 3]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))


def main():
    import numpy as np
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.set_option(22, 0)  # deferral on any launch size
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    out = torch.zeros((a.frames, H, W, 4), dtype=torch.float32, device="cuda")
    r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=0), a.frames, 0, 0, W, H, out=out)
    ts = torch.zeros((65536, 4), dtype=torch.int64, device="cuda")
    r.set_wave_timeline(ts)
    r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, 0, W, H, out=out)
    torch.cuda.synchronize()
    r.set_wave_timeline(None)
    t = ts.cpu().numpy()
    t = t[t[:, 2] > 0].astype(np.float64)
    t0 = t[:, 0].min()
    start, staged, end, chunks = (t[:, 0] - t0) / 100, (t[:, 1] - t0) / 100, (t[:, 2] - t0) / 100, t[:, 3]
    print(f"# {desc}: tail kernel, {len(t)} waves, {a.frames} frames; times in us from the first wave's start")
    for q in (0, 10, 50, 90, 100):
        print(f"  p{q:3d}: start {np.percentile(start, q):8.1f}  staged {np.percentile(staged, q):8.1f}  "
              f"end {np.percentile(end, q):8.1f}  chunks|iters {np.percentile(chunks, q):6.1f}")
    print(f"  sum of chunks {chunks.sum():.0f}; busy share (sum of wave lives / (waves x span)) "
          f"{(end - start).sum() / (len(t) * end.max()):.3f}")
    r.close()


if __name__ == "__main__":
    main()
