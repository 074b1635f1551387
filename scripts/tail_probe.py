"""Tail-split diagnostics (MM_OPT_TAIL_SPLIT): one C3 frame (or rank 0's rows
of an N-way split) with the split on; prints the hand-over counters and the
launch's timeline from mm_tail_counters.

    python scripts/tail_probe.py [--ranks N] [--frames F]
"""
import argparse
import ctypes
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze._lib import lib

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    r.set_option(18, 1)
    u = default_uniform(W, H, 0)
    h = (H + a.ranks - 1) // a.ranks
    out = torch.zeros((h, W, 4), dtype=torch.float32, device="cuda")
    buf = (ctypes.c_uint32 * 192)()
    print(f"# {desc}, rank 0 of {a.ranks}")
    for f in range(a.frames):
        r.trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, 0, W, h, y_stride=a.ranks, out=out)
        torch.cuda.synchronize()
        assert lib().mm_tail_counters(r._ctx, buf, 192) == 0
        d = list(buf)
        t0 = d[160 + 17]
        print(f"f{f}: done {d[32]} reserved {d[64]} claimed {d[65]} slots {d[96]} takers {d[128]} idle {d[0]}  "
              f"queue dry at {(d[160 + 14] - t0) / 100:.1f} us, all done {(d[160 + 18] - t0) / 100:.1f} us, "
              f"last exit {(d[160 + 15] - t0) / 100:.1f} us",
              flush=True)
    r.close()


if __name__ == "__main__":
    main()
