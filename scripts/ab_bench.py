"""A/B timing of the throughput-mode variants on one GPU (C3 unless told
otherwise).  Every variant must produce the bit-identical frame; prints one
line per variant with the HIP-event time of the trace kernel.

    python scripts/ab_bench.py [--config c3] [--frames 3] [variant ...]
variants: ref  mega-global  mega-lds  mega-lds-b512 ... (see VARIANTS)
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))

VARIANTS = {
    "ref": dict(pipe=3),
    "mega-global": dict(pipe=1, persist=0, lds=0, block=256),
    "mega-lds": dict(pipe=1, persist=0, lds=1, block=256),
    "mega-lds-b128": dict(pipe=1, persist=0, lds=1, block=128),
    "mega-lds-b512": dict(pipe=1, persist=0, lds=1, block=512),
    "mega-lds-b1024": dict(pipe=1, persist=0, lds=1, block=1024),
    "mega-global-b64": dict(pipe=1, persist=0, lds=0, block=64),
    "wave": dict(pipe=2),
    "wave-global": dict(pipe=2, lds=0),
    "wave-b256": dict(pipe=2, block=256),
}
for _b, _w in ((512, 6), (512, 8), (1024, 1), (1024, 8)):
    for _k in (8, 16, 32):
        VARIANTS[f"lb{_k}-ldsrec-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=1, ww=_k)
        VARIANTS[f"lb{_k}-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=0, ww=_k)
    VARIANTS[f"ww-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, ww=1)
    VARIANTS[f"ww-ldsstack-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=1, ww=1)
    VARIANTS[f"wp-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w)
    VARIANTS[f"wp-global-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=0, block=_b, mw=_w)
    VARIANTS[f"wp-ldsstack-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=1)
    VARIANTS[f"wp-lds-b{_b}-w{_w}"]["ls"] = 0
    VARIANTS[f"wp-lds-b{_b}-w{_w}"]["lr"] = 0
    VARIANTS[f"wp-ldsrec-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=1)
for _b, _w in ((512, 6), (1024, 8), (1024, 1)):
    VARIANTS[f"lean-ldsrec-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=1, ww=2)
    VARIANTS[f"lean-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=0, ww=2)
    VARIANTS[f"lean-ldsstack-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=1, lr=0, ww=2)
    VARIANTS[f"lean-split1-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, split=1, ww=2)
for _b, _w in ((512, 6), (1024, 8), (1024, 1)):
    VARIANTS[f"rt-ldsrec-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=1, ww=3)
    VARIANTS[f"rt-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=0, ww=3)
for _b, _w in ((512, 6), (512, 8), (1024, 8), (1024, 1)):
    VARIANTS[f"cold-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=0, cold=1)
for _b, _w in ((512, 6), (1024, 8), (1024, 1)):
    VARIANTS[f"br-ldsrec-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=1, ww=4)
    VARIANTS[f"br-lds-b{_b}-w{_w}"] = dict(pipe=1, persist=2, lds=1, block=_b, mw=_w, ls=0, lr=0, ww=4)
VARIANTS["br-split1"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=1, ww=4)
VARIANTS["split1-gr0"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=1, gr=0)
VARIANTS["split1-gr1"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=1, gr=1)
VARIANTS["lds-gr1"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, ls=0, lr=0, gr=1)
VARIANTS["lds-gr0"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, ls=0, lr=0, gr=0)
VARIANTS["rt-split1"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=1, ww=3)
VARIANTS["default"] = dict(pipe=1)  # library defaults (auto loop form, fused resolve)
VARIANTS["nofuse"] = dict(pipe=1, fuse=0)
for _f in (1,):
    VARIANTS[f"fair{_f}"] = dict(pipe=1, fair=_f)
for _g in (2, 4, 8):
    VARIANTS[f"grab{_g}"] = dict(pipe=1, grab=_g)
VARIANTS["li-b768-w6"] = dict(pipe=1, persist=2, lds=1, block=768, mw=6, ls=0, lr=1, ww=5)
VARIANTS["brli-ldsrec"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, ls=0, lr=1, ww=6)
VARIANTS["blocksync"] = dict(pipe=1, bsync=1)
VARIANTS["lean7"] = dict(pipe=1, ww=7)
VARIANTS["order1"] = dict(pipe=1, order=1)
VARIANTS["dict"] = dict(pipe=1, dict=1)
VARIANTS["dict-li"] = dict(pipe=1, dict=1, ww=5)
VARIANTS["dict2"] = dict(pipe=1, dict=2)
VARIANTS["cons9"] = dict(pipe=1, ww=9)
VARIANTS["li-ldsstack-grec"] = dict(pipe=1, ls=2)
VARIANTS["li-ldsstack"] = dict(pipe=1, ls=1, lr=0)
VARIANTS["li-lds-grec"] = dict(pipe=1, lr=0, gr=1)
VARIANTS["li-ldsrec"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, ls=0, lr=1, ww=5)
VARIANTS["li-lds"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, ls=0, lr=0, ww=5)
VARIANTS["li-split1"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=1, ww=5)
for _kb in (0, 1, 16, 32, 48, 64, 80):
    VARIANTS[f"wp-split{_kb}"] = dict(pipe=1, persist=2, lds=1, block=1024, mw=8, split=_kb)
    VARIANTS[f"wp-split{_kb}-b512-w6"] = dict(pipe=1, persist=2, lds=1, block=512, mw=6, split=_kb)
for _b, _w in ((512, 6), (1024, 1), (1024, 8)):
    for _th in (0, 8, 16, 24, 32, 40, 48):
        VARIANTS[f"persist-lds-b{_b}-w{_w}-t{_th}"] = dict(pipe=1, persist=1, lds=1, block=_b, mw=_w, th=_th, lr=0)
        VARIANTS[f"persist-ldsrec-b{_b}-w{_w}-t{_th}"] = dict(pipe=1, persist=1, lds=1, block=_b, mw=_w, th=_th, lr=1)
        VARIANTS[f"persist-global-b{_b}-w{_w}-t{_th}"] = dict(pipe=1, persist=1, lds=0, block=_b, mw=_w, th=_th)


def main():
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze._lib import MM_OPT_BLOCK, MM_OPT_LDS_NODES, MM_OPT_MIN_WAVES, MM_OPT_PERSIST, MM_OPT_THRESHOLD

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--ranks", type=int, default=1, help="trace rank 0's rows of an N-way split (0, N, 2N, ...)")
    ap.add_argument("variants", nargs="*", default=["ref", "mega-global", "mega-lds"])
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    scene = Scene.build(maze_n, 0)
    u = default_uniform(W, H, 0)
    base = None
    print(f"# {desc}: {scene.n_rects} rects, {scene.n_nodes} nodes, depth {scene.bvh_depth}", flush=True)
    for name in a.variants:
        v = VARIANTS[name]
        r = Renderer(0)
        r.upload_scene(scene)
        r.set_pipeline(v["pipe"])
        if "lds" in v:
            r.set_option(MM_OPT_LDS_NODES, v["lds"])
        if "block" in v:
            r.set_option(MM_OPT_BLOCK, v["block"])
        if "persist" in v:
            r.set_option(MM_OPT_PERSIST, v["persist"])
        if "lr" in v:
            r.set_option(8, v["lr"])
        if "ww" in v:
            r.set_option(7, v["ww"])
        elif v.get("persist") == 2:
            r.set_option(7, 0)  # historical wp-* variants: the if-if loop
        if "bsync" in v:
            r.set_option(16, v["bsync"])
        if "grab" in v:
            r.set_option(15, v["grab"])
        if "dict" in v:
            r.set_option(20, v["dict"])
        if "order" in v:
            r.set_option(17, v["order"])
        if "fair" in v:
            r.set_option(14, v["fair"])
        if "fuse" in v:
            r.set_option(12, v["fuse"])
        if "ls" in v:
            r.set_option(6, v["ls"])
        if "mw" in v:
            r.set_option(MM_OPT_MIN_WAVES, v["mw"])
        if "gr" in v:
            r.set_option(11, v["gr"])
        if "cold" in v:
            r.set_option(10, v["cold"])
        if "split" in v:
            r.set_option(9, v["split"])
        if "th" in v:
            r.set_option(MM_OPT_THRESHOLD, v["th"])
        h = (H + a.ranks - 1) // a.ranks
        out = torch.zeros((h, W, 4), dtype=torch.float32, device="cuda")
        _, st = r.trace_tile(u, make_ext(spp, bl, ml, frame=0), 0, 0, W, h, y_stride=a.ranks, out=out,
                             stats=True)  # warm
        torch.cuda.synchronize()
        r.set_profiling(True)
        r.kernel_timing(reset=True)
        t0 = time.perf_counter()
        for f in range(a.frames):  # frames 1.. (the per-frame RNG differs from the warm frame's)
            r.trace_tile(u, make_ext(spp, bl, ml, frame=f + 1), 0, 0, W, h, y_stride=a.ranks, out=out)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        kms, kn = r.kernel_timing(reset=True)
        k = kms / max(kn, 1)
        same = "base"
        if base is None:
            base = out.clone()
        else:
            same = "bit-identical" if torch.equal(base.view(torch.int32), out.view(torch.int32)) else "MISMATCH"
        print(f"{name:18s} trace {k:8.3f} ms  wall {wall:8.3f} ms/frame  {st.rays / k / 1e3:9.1f} Mrays/s  "
              f"rays/frame {st.rays}  {same}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
