"""A/B timing of throughput-mode variants on one GPU (C3 unless told
otherwise).  Every variant must produce the bit-identical frame; prints one
line per variant with the HIP-event time of the trace kernel.  Each variant
traces --frames frames in one multi-frame launch (bench.py's issue mode) when
the fused resolve applies, else one launch per frame.

    python scripts/ab_bench.py [--config c3] [--frames 5] [--reps 2] [variant ...]
A different build of the library: MIRROR_MAZE_LIB=/path/lib.so (scripts/ab.py).
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))

# name -> (pipeline, {MM_OPT_*: value}); include/mm_api.h
VARIANTS = {
    "default": (1, {}),
    "grid": (1, {7: 11}),
    "grid-index-lds": (1, {7: 11}),        # same as grid where the image fits (C3)
    "grid-global": (1, {7: 11, 1: 0}),
    "bvh-lean": (1, {7: 7}),
    "bvh-li": (1, {7: 5}),
    "nofuse": (1, {12: 0}),
    "nodefer": (1, {21: 0}),
    "defer8": (1, {21: 8}),
    "defer16": (1, {21: 16}),
    "defer24": (1, {21: 24}),
    "defer32": (1, {21: 32}),
    "defer40": (1, {21: 40}),
    "defer48": (1, {21: 48}),
    "defer56": (1, {21: 56}),
    "defer64": (1, {21: 64}),       # every path deferred at bounce 1: the tail rings run the rest
    "defer-min0": (1, {22: 0}),     # deferral on launches of any size
    "wave": (2, {}),
    "ref": (3, {}),
    "cell60": (1, {25: 60}), "cell70": (1, {25: 70}), "cell80": (1, {25: 80}), "cell90": (1, {25: 90}),
    "cell110": (1, {25: 110}), "cell125": (1, {25: 125}), "cell140": (1, {25: 140}), "cell160": (1, {25: 160}),
    "reserve64": (1, {19: 64}),     # MM_OPT_RESERVE_CUS: resident blocks on 192 of 256 CUs' worth
    "reserve128": (1, {19: 128}),   # 128 of 256
    "plain": (1, {26: 0}),          # MM_OPT_GRID_WIDE 0: plain 32-bit cell words (whole list per cell)
    "nomerge": (1, {24: 0}),        # MM_OPT_GRID_MERGE 0: cells along y by the rect size (round 2's grid)
    "grid-global-nomerge": (1, {1: 0, 24: 0}),
}


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ranks", type=int, default=1, help="trace rank 0's rows of an N-way split (0, N, 2N, ...)")
    ap.add_argument("variants", nargs="*", default=["default", "bvh-lean"])
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    scene = Scene.build(maze_n, 0)
    u = default_uniform(W, H, 0)
    h = (H + a.ranks - 1) // a.ranks
    base = None
    print(f"# {desc}: {scene.n_rects} rects, {scene.n_nodes} nodes, depth {scene.bvh_depth}", flush=True)
    for rep in range(a.reps):
        for name in a.variants:
            pipe, opts = VARIANTS[name]
            r = Renderer(0)
            r.set_pipeline(pipe)
            for k, v in opts.items():
                r.set_option(k, v)
            r.upload_scene(scene)
            multi = pipe in (0, 1) and opts.get(3, 2) == 2 and (opts.get(21, 0) or (opts.get(12, 1) and 64 % spp == 0))
            out = torch.zeros((a.frames, h, W, 4), dtype=torch.float32, device="cuda")
            _, st = r.trace_tile(u, make_ext(spp, bl, ml, frame=0), 0, 0, W, h, y_stride=a.ranks, out=out[0],
                                 stats=True)  # warm; rays of frame 0
            torch.cuda.synchronize()
            r.set_profiling(True)
            r.kernel_timing(reset=True)
            t0 = time.perf_counter()
            if multi:
                r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=1), a.frames, 0, 0, W, h, y_stride=a.ranks, out=out)
            else:
                for f in range(a.frames):
                    r.trace_tile(u, make_ext(spp, bl, ml, frame=f + 1), 0, 0, W, h, y_stride=a.ranks, out=out[f])
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / a.frames * 1e3
            kms, kn = r.kernel_timing(reset=True)
            k = kms / a.frames
            same = "base"
            if base is None:
                base = out.clone()
            else:
                same = "bit-identical" if torch.equal(base.view(torch.int32), out.view(torch.int32)) else "MISMATCH"
            # checksum of the frames' bits, to compare builds (MIRROR_MAZE_LIB) across processes
            bits = out.view(torch.int32).to(torch.int64)
            ck = int((bits * torch.arange(1, bits.numel() + 1, device=bits.device).view(bits.shape) % 1000003)
                     .sum().item())
            gi = "grid %dx%dx%d %s %.0fKB lds%d" % (
                r.scene_info(2), r.scene_info(3), r.scene_info(4), "faces" if r.scene_info(13) else "plain",
                r.scene_info(6) / 1024, r.scene_info(12)) if r.scene_info(1) else "no grid"
            print(f"{name:16s} rep {rep} trace {k:8.3f} ms/frame  wall {wall:8.3f} ms/frame  "
                  f"{st.rays / k / 1e3:9.1f} Mrays/s  launches {kn}  {same}  ck {ck:x}  {gi}", flush=True)
            r.close()


if __name__ == "__main__":
    main()
