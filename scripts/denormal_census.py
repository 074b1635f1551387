#!/usr/bin/env python
"""Denormal census of the path.

The reference AIR is compiled with `air.compile.denorms_disable`
(/root/reference/src/shaders.ir metadata !47): the Apple GPU flushes denormal
operands and results to zero.  The HIP kernels and the oracle run IEEE
binary32 with denormals.  The two agree on every input on which no operation
sees a denormal operand or produces a denormal result.  This script runs the
oracle (test infrastructure) over the workloads the parity suite and bench
cover, with the x86 MXCSR sticky flags cleared at every entry point:

  DE (bit 1)  some operand was denormal
  UE (bit 4)  some result was tiny (below 2^-126) and inexact

and, on every workload, again with FTZ|DAZ set (the reference's semantics),
comparing the two outputs bit for bit.  A tiny *exact* result raises no UE
but cannot go unseen either: every value the path produces is an operand of a
later operation (a comparison, sqrt, the sample sum), which raises DE.

    python scripts/denormal_census.py [--quick] [--out profiles/r03/denormal_census.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "mirror-maze_amd")]


def tile(o, u, e, x0, y0, w, h, stride=1, threads=8):
    out = np.zeros((h, w, 4), np.float32)
    band = max(1, -(-h // (4 * threads)))
    jobs = [(j0, min(band, h - j0)) for j0 in range(0, h, band)]

    def run(job):
        j0, n = job
        _, st = o.trace_tile(u, e, x0, y0 + j0 * stride, w, n, y_stride=stride, out=out[j0:j0 + n])
        return st.rays

    with ThreadPoolExecutor(threads) as ex:
        rays = sum(ex.map(run, jobs))
    return out, rays


def workloads(quick):
    from mirror_maze import Scene, calculate_quaternion, default_uniform, make_ext

    s10, s16, s32, s64 = (Scene.build(n, 0) for n in (10, 16, 32, 64))
    W = [
        ("C1 whole frame (16x16 maze, 256x256, 1 spp, 1 bounce)", s16, default_uniform(256, 256, 0),
         make_ext(1, 1, 15), (0, 0, 256, 256, 1)),
        ("C2 whole frame (16x16, 1920x1080, 1 spp, 4/15)", s16, default_uniform(1920, 1080, 0),
         make_ext(1, 4, 15), (0, 0, 1920, 1080, 1)),
    ]
    if not quick:
        W += [("C3 whole frame 0 (32x32, 1920x1080, 8 spp, 8/8)", s32, default_uniform(1920, 1080, 0),
               make_ext(8, 8, 8, frame=0), (0, 0, 1920, 1080, 1)),
              ("C3 whole frame 1", s32, default_uniform(1920, 1080, 0), make_ext(8, 8, 8, frame=1),
               (0, 0, 1920, 1080, 1)),
              ("C4 rank 0 of 8 (32x32, 3840x2160, 16 spp, 8/15)", s32, default_uniform(3840, 2160, 0),
               make_ext(16, 8, 15), (0, 0, 3840, 270, 8))]
    else:
        W += [("C3 rows 500..531", s32, default_uniform(1920, 1080, 0), make_ext(8, 8, 8), (0, 500, 1920, 32, 1))]
    for (x0, y0) in [(0, 0), (1904, 1064), (3808, 2144), (700, 1500), (2900, 300), (1200, 40)][:2 if quick else 6]:
        W.append((f"C5 window ({x0}, {y0}) 32x16 (64x64, 3840x2160, 64 spp, 16/16)", s64,
                  default_uniform(3840, 2160, 0), make_ext(64, 16, 16, frame=7), (x0, y0, 32, 16, 1)))
    # cameras inside the maze (closed corridors, mirrors at close range)
    rng = np.random.default_rng(3)
    for n, sc, bl, ml in ((32, s32, 8, 8), (64, s64, 16, 16), (10, s10, 5, 15))[:1 if quick else 3]:
        for k in range(2 if quick else 6):
            u = default_uniform(320, 180, 0)
            base = -10.0 * (n / 2)
            cx, cz = rng.integers(0, n, size=2)
            u.cam.center[0] = base + 10.0 * cx + 5.0
            u.cam.center[1] = float(rng.uniform(-6.0, 1.5))
            u.cam.center[2] = base + 10.0 * cz + 5.0
            q = calculate_quaternion(rng.normal(size=3).astype(np.float32))
            for i in range(4):
                u.cam.quat[i] = float(q[i])
            W.append((f"camera in the {n}x{n} maze #{k} (320x180, 8 spp, {bl}/{ml})", sc, u,
                      make_ext(8, bl, ml, frame=int(rng.integers(0, 1000))), (0, 0, 320, 180, 1)))
    return W


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default=str(REPO / "profiles" / "r03" / "denormal_census.json"))
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 4))
    args = ap.parse_args()
    from oracle.oracle import FP_DENORMAL_OPERAND, FP_UNDERFLOW, Oracle, fp_flags, set_fp_mode

    rows, t_all = [], time.time()
    for name, sc, u, e, (x0, y0, w, h, st) in workloads(args.quick):
        o = Oracle.from_scene(sc)
        t0 = time.time()
        set_fp_mode(False)
        fp_flags(reset=True)
        ieee, rays = tile(o, u, e, x0, y0, w, h, st, args.threads)
        flags = fp_flags(reset=True)
        set_fp_mode(True)
        ftz, _ = tile(o, u, e, x0, y0, w, h, st, args.threads)
        set_fp_mode(False)
        same = bool(np.array_equal(ieee.view(np.uint32), ftz.view(np.uint32)))
        row = {"workload": name, "rays": int(rays), "denormal_operand": bool(flags & FP_DENORMAL_OPERAND),
               "underflow": bool(flags & FP_UNDERFLOW), "mxcsr_flags": hex(flags),
               "ftz_daz_output_identical": same, "seconds": round(time.time() - t0, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    rec = {"what": ("oracle (IEEE binary32, the HIP kernels' arithmetic) with MXCSR sticky flags per entry point, "
                    "and the same workloads under FTZ|DAZ (the reference's air.compile.denorms_disable, "
                    "src/shaders.ir !47), outputs compared bit for bit"),
           "workloads": len(rows), "rays": sum(r["rays"] for r in rows),
           "any_denormal_operand": any(r["denormal_operand"] for r in rows),
           "any_underflow": any(r["underflow"] for r in rows),
           "all_ftz_identical": all(r["ftz_daz_output_identical"] for r in rows),
           "seconds": round(time.time() - t_all, 1), "rows": rows}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: v for k, v in rec.items() if k != "rows"}))


if __name__ == "__main__":
    main()
