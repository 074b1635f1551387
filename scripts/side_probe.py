"""Does side work on another stream get CUs while a batched trace launch runs?
Stand-in for the per-frame RCCL gathers of a multi-GPU run: a device copy of
the size rank 0 receives for a batch of frames (5 frames x 7/8 of a C3 frame),
issued on a second stream at the moment the trace launch starts.  Reports the
trace launch time and when the copy finished, for MM_OPT_RESERVE_CUS = 0 / 4 / 8.

    python scripts/side_probe.py [--ranks 8] [--frames 5]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=5)
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS["c3"]
    h = (H + a.ranks - 1) // a.ranks
    u = default_uniform(W, H, 0)
    n_bytes = a.frames * (H * W * 16) * (a.ranks - 1) // a.ranks
    src = torch.ones(n_bytes // 4, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)
    s_tr, s_side = torch.cuda.Stream(), torch.cuda.Stream()
    print(f"# {desc}: rank 0 of {a.ranks}, {a.frames} frames per launch; side copy {n_bytes / 1e6:.0f} MB")
    for reserve in (0, 4, 8):
        r = Renderer(0)
        r.upload_scene(Scene.build(maze_n, 0))
        r.set_option(19, reserve)
        out = torch.zeros((a.frames, h, W, 4), dtype=torch.float32, device="cuda")
        alone = []
        for rep in range(4):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            with torch.cuda.stream(s_tr):
                ev[0].record(s_tr)
                r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=8 * rep), a.frames, 0, 0, W, h, y_stride=a.ranks,
                                    out=out)
                ev[1].record(s_tr)
            if rep >= 2:  # side copy starts with the launch
                s_side.wait_event(ev[0])
                with torch.cuda.stream(s_side):
                    dst.copy_(src)
                    ev[2].record(s_side)
            torch.cuda.synchronize()
            tr = ev[0].elapsed_time(ev[1])
            if rep < 2:
                alone.append(tr)
            else:
                side = ev[0].elapsed_time(ev[2])
                print(f"reserve {reserve}: trace alone {min(alone):7.3f} ms, with side copy {tr:7.3f} ms, "
                      f"copy done at {side:7.3f} ms ({'during' if side < tr else 'AFTER'} the launch)", flush=True)
        r.close()


if __name__ == "__main__":
    main()
