#!/usr/bin/env python
"""Where a wave's time goes (diagnostics build: -DMM_PHASE_CLOCKS, see
scripts/build_variant.sh): per wave of the main trace kernel, wall_clock64 ticks (100 MHz)
inside closest-hit queries, inside shading, and the wave's whole life; the
remainder is chunk setup, primary rays, deferral and the resolve.

    bash scripts/build_variant.sh phase wt -DMM_PHASE_CLOCKS
    MIRROR_MAZE_LIB=exp/phase/lib.so python scripts/phase_probe.py [--config c3]
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
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    out = torch.zeros((a.frames, H, W, 4), dtype=torch.float32, device="cuda")
    r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=0), a.frames, 0, 0, W, H, out=out)  # warm
    ts = torch.zeros((65536, 4), dtype=torch.int64, device="cuda")
    r.set_wave_timeline(ts)
    r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, 0, W, H, out=out)
    torch.cuda.synchronize()
    r.set_wave_timeline(None)
    t = ts.cpu().numpy()
    t = t[t[:, 2] > 0]
    life = (t[:, 2] - t[:, 0]).astype(np.float64)
    q, s = t[:, 1].astype(np.float64), t[:, 3].astype(np.float64)
    print(f"# {desc}: {len(t)} waves, {a.frames} frames in one launch; first rows {t[:3].tolist()}")
    print(f"wave life  mean {life.mean():.4g} cycles")
    print(f"queries    {q.sum() / life.sum():.3f} of wave time")
    print(f"shading    {s.sum() / life.sum():.3f}")
    print(f"other      {1 - (q.sum() + s.sum()) / life.sum():.3f}")
    r.close()


if __name__ == "__main__":
    main()
