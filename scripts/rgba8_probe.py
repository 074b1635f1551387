"""The fused RGBA8 store (MM_EXT_RGBA8) against the float frames + one
mm_quantize_rgba8 per launch that bench.py ran before it, on the driver's
launch shape (C3, 20 frames in one mm_trace_tile_frames launch), same library,
interleaved repetitions; HIP events on the renderer's stream around the whole
launch (trace + resolve + conversion).  Checks the bytes are equal.

    python scripts/rgba8_probe.py [--config c3] [--frames 20] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    s = torch.cuda.Stream()
    n = a.frames
    f32 = torch.zeros((n, H, W, 4), dtype=torch.float32, device="cuda")
    q8 = torch.zeros((n, H, W, 4), dtype=torch.uint8, device="cuda")
    u8 = torch.zeros((n, H, W, 4), dtype=torch.uint8, device="cuda")
    u = default_uniform(W, H, 0)
    times = {"float+quantize": [], "rgba8": []}
    with torch.cuda.stream(s):
        for rep in range(a.reps + 1):
            e = make_ext(spp, bl, ml, frame=100 * rep)
            for arm in ("float+quantize", "rgba8"):
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(s)
                if arm == "rgba8":
                    r.trace_tile_frames(u, e, n, 0, 0, W, H, out=u8)
                else:
                    r.trace_tile_frames(u, e, n, 0, 0, W, H, out=f32)
                    r.quantize(f32, out=q8)
                t1.record(s)
                t1.synchronize()
                if rep:  # rep 0 warms up (staging buffers, tail queue)
                    times[arm].append(t0.elapsed_time(t1) / n)
            assert torch.equal(u8, q8), "RGBA8 frames differ from the quantized float frames"
    r.close()
    out = {"config": desc, "frames_per_launch": n, "reps": a.reps, "bit_identical": True}
    for arm, v in times.items():
        out[arm] = {"ms_per_frame_median": round(statistics.median(v), 4), "all": [round(x, 4) for x in v]}
    out["saving_pct"] = round(100 * (1 - out["rgba8"]["ms_per_frame_median"] / out["float+quantize"]["ms_per_frame_median"]), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
