#!/usr/bin/env python
"""Where the idle lanes sit (diagnostics build -DMM_LANE_STATS): per phase of
the bounce loop of the main trace kernel, the wave-iterations that run it and
the lanes active in them, over one multi-frame launch.  Lane utilisation of a
phase = active lanes / (64 x wave-iterations).

    bash scripts/build_variant.sh lanes wt -DMM_LANE_STATS
    MIRROR_MAZE_LIB=exp/lanes/lib.so python scripts/lane_probe.py [--config c3] [--json out.json]
"""
import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))

# mm_device.h LanePhase, in order
PHASES = ["chunk", "bounce", "global_rect", "grid_iter", "rect_test", "cell_step", "certificate",
          "bvh_fallback", "shade", "diffuse", "trial", "mirror"]
RECORD = 49152  # mm_device.h kLaneStatRecord


def main():
    import numpy as np
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    out = torch.zeros((a.frames, H, W, 4), dtype=torch.float32, device="cuda")
    ts = torch.zeros((65536, 4), dtype=torch.int64, device="cuda")
    r.set_wave_timeline(ts)
    r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, 0, W, H, out=out)
    torch.cuda.synchronize()
    r.set_wave_timeline(None)
    w = ts.cpu().numpy().reshape(-1)[4 * RECORD: 4 * RECORD + 2 * len(PHASES)].astype(np.float64)
    waves, lanes = w[0::2], w[1::2]
    rays = a.frames * W * H * spp
    res = {"config": a.config, "frames": a.frames, "phases": {}}
    print(f"# {desc}: {a.frames} frames in one launch; per phase: wave-iterations, active lanes, "
          f"utilisation, wave-iterations per path")
    for i, name in enumerate(PHASES):
        util = lanes[i] / (64.0 * waves[i]) if waves[i] else 0.0
        res["phases"][name] = {"wave_iters": int(waves[i]), "lane_iters": int(lanes[i]), "util": round(util, 4)}
        print(f"{name:13s} {waves[i]:14.0f} {lanes[i]:16.0f}  util {util:6.3f}  per path "
              f"{waves[i] * 64 / rays:7.3f}")
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1) + "\n")
    r.close()


if __name__ == "__main__":
    main()
