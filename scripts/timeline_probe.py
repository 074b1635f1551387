#!/usr/bin/env python
"""Per-wave timeline of the wave-persistent kernel (diagnostics): for rank 0's
row set at N = 1, 2, 4, 8 (rows 0, N, 2N, ...) record every wave's entry,
LDS-staged and exit times and its chunk count (mm_set_wave_timeline), and
report where a launch's time goes: dispatch ramp, staging, steady state, and
the tail between the first and the last wave to run out of work.

    python scripts/timeline_probe.py [--config c3] [--ranks 1,2,4,8]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mirror-maze_amd"))


TIMELINE_WAVES = 32768  # trace_kernels.hip kTimelineWaves: the second record of wave w is at w + 32768


def tail_report(raw, t0, np):
    """Launch tail (MM_TAIL_CLOCKS build): per wave its exit, XCD, last chunk
    (start, new or tail), longest chunk, chunks over 100 us and the moment it
    saw the global queue out."""
    n = TIMELINE_WAVES
    wid = np.nonzero(raw[:n, 2] > 0)[0]
    ext = (raw[wid, 2] - t0) / 100.0
    r2, r3 = raw[n + wid], raw[2 * n + wid]
    last_raw = r2[:, 0].astype(np.uint64)
    is_tail = (last_raw >> np.uint64(63)).astype(bool)
    last = (last_raw & np.uint64((1 << 63) - 1)).astype(np.int64)
    ok = last > 0
    xcc = r2[:, 1]
    dur = np.where(ok, (raw[wid, 2] - last) / 100.0, np.nan)
    longest = r3[:, 0] / 100.0
    over100 = r3[:, 1]
    qout = np.where(r3[:, 2] > 0, (r3[:, 2] - t0) / 100.0, np.nan)
    span, first_out = ext.max(), ext.min()
    q0 = np.nanmin(qout)
    print(f"    tail {span - first_out:.1f} us (first wave out {first_out:.1f}); global queue first seen out at "
          f"{q0:.1f}, by the last wave at {np.nanmax(qout):.1f}", flush=True)
    print(f"    longest chunk per wave p50 {np.median(longest):.1f} p90 {np.percentile(longest, 90):.1f} max "
          f"{longest.max():.1f} us; chunks over 100 us: {int(over100.sum())} in {int((over100 > 0).sum())} waves "
          f"(of {int(raw[wid, 3].sum())} chunks)", flush=True)
    print(f"    last chunk: {int(is_tail.sum())} waves ended on a tail chunk; duration p50 {np.nanmedian(dur):.1f} "
          f"p90 {np.nanpercentile(dur, 90):.1f} max {np.nanmax(dur):.1f} us", flush=True)
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        e = ext[m]
        print(f"    XCD {x}: {m.sum():5d} waves, exit min/p50/p90/max {e.min():7.1f}/{np.median(e):7.1f}/"
              f"{np.percentile(e, 90):7.1f}/{e.max():7.1f}", flush=True)
    k = max(1, len(ext) // 50)
    idx = np.argsort(ext)[-k:]
    lstart = np.where(ok, (last - t0) / 100.0, np.nan)
    print(f"    last {k} waves out (exit {ext[idx].min():.1f}..{ext[idx].max():.1f}): last chunk started p10/p50/p90 "
          f"{np.nanpercentile(lstart[idx], 10):.1f}/{np.nanmedian(lstart[idx]):.1f}/{np.nanpercentile(lstart[idx], 90):.1f}"
          f", {int(is_tail[idx].sum())} were tail chunks, lasted p50 {np.nanmedian(dur[idx]):.1f} max "
          f"{np.nanmax(dur[idx]):.1f} us; saw the queue out at p50 {np.nanmedian(qout[idx]):.1f}; "
          f"XCDs {np.bincount(xcc[idx].astype(int), minlength=8).tolist()}", flush=True)
    r4 = raw[3 * n + wid].astype(np.uint64)
    if r4[:, 0].any():
        for kind, col in (("new", 0), ("tail", 1)):
            tot = (r4[:, col] >> np.uint64(32)).astype(np.float64) / 100.0
            cnt = (r4[:, col] & np.uint64(0xFFFFFFFF)).astype(np.float64)
            lng = r4[:, 2 + col].astype(np.float64) / 100.0
            print(f"    {kind} chunks: {int(cnt.sum())}, mean {tot.sum() / max(cnt.sum(), 1):.1f} us, longest per wave "
                  f"p50 {np.median(lng):.1f} p90 {np.percentile(lng, 90):.1f} max {lng.max():.1f} us; share of wave "
                  f"time {tot.sum() / (ext.sum() + 1e-9):.1%}", flush=True)
    # per SIMD (HW_REG_HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13], with the XCD): the waves sharing
    # it, ordered by launch (wave id), their chunks and exits -- does the issue arbiter's age order set a
    # wave's speed, and are the last waves out the young ones?
    hw = r2[:, 2].astype(np.int64)
    simd = ((xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) |
            (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3))
    chunks = raw[wid, 3].astype(np.float64)
    order = np.lexsort((wid, simd))
    s_sorted = simd[order]
    starts = np.r_[0, np.nonzero(np.diff(s_sorted))[0] + 1]
    age = np.empty(len(wid), dtype=np.int64)  # 0: the SIMD's first-launched wave
    for a, b in zip(starts, np.r_[starts[1:], len(order)]):
        age[order[a:b]] = np.arange(b - a)
    per = np.bincount(simd_idx := np.unique(simd, return_inverse=True)[1])
    print(f"    SIMDs {len(per)}, waves per SIMD {np.bincount(per).nonzero()[0].tolist()}", flush=True)
    rows = []
    for g in range(int(age.max()) + 1):
        m = age == g
        rows.append(f"{g}:{chunks[m].mean():.0f}/{np.median(ext[m]) - first_out:.0f}")
    print("    by launch order on the SIMD (order: mean chunks / median exit after the first wave out, us): "
          + " ".join(rows), flush=True)
    rk = np.empty(len(wid), dtype=np.int64)  # 0: the SIMD's busiest wave
    for a, b in zip(starts, np.r_[starts[1:], len(order)]):
        o = order[a:b]
        rk[o[np.argsort(-chunks[o], kind="stable")]] = np.arange(b - a)
    print(f"    last {k} waves out: launch order on their SIMD {np.bincount(age[idx], minlength=age.max() + 1).tolist()}"
          f", chunk rank on their SIMD (0 = most) {np.bincount(rk[idx], minlength=rk.max() + 1).tolist()}; their "
          f"chunks p50 {np.median(chunks[idx]):.0f} (all waves p50 {np.median(chunks):.0f})", flush=True)
    # each wave's last new chunk (from the global queue): when it started and ended against the queue running out
    # (q0), and the tail chunks the wave ran after it -- is the drain the last new chunks or the rings' tails?
    r5 = raw[4 * n + wid].astype(np.uint64)
    if r5[:, 0].any():
        ls = (r5[:, 0].astype(np.int64) - t0) / 100.0
        ld = r5[:, 1].astype(np.float64) / 100.0
        le = np.where(ld > 0, ls + ld, ext)  # 0: the last new chunk ran until the exit
        nt = r5[:, 2].astype(np.int64)
        print(f"    last new chunk ended after the queue ran out: p50 {np.median(le) - q0:.1f} p90 "
              f"{np.percentile(le, 90) - q0:.1f} max {le.max() - q0:.1f} us; tail chunks after it p50 "
              f"{np.median(nt):.0f} p90 {np.percentile(nt, 90):.0f} max {nt.max()}", flush=True)
        print(f"    last {k} waves out: their last new chunk started {np.median(ls[idx]) - q0:.1f} (p50) / "
              f"{np.min(ls[idx]) - q0:.1f} (min) and ended {np.median(le[idx]) - q0:.1f} (p50) / "
              f"{np.max(le[idx]) - q0:.1f} (max) us after the queue ran out; tail chunks after it p50 "
              f"{np.median(nt[idx]):.0f} max {nt[idx].max()}", flush=True)
        for g in range(int(age.max()) + 1):
            m = age == g
            print(f"      launch order {g}: last new chunk ends p50 {np.median(le[m]) - q0:.1f} p90 "
                  f"{np.percentile(le[m], 90) - q0:.1f} us after q0, lasted p50 "
                  f"{np.median(np.where(ld[m] > 0, ld[m], ext[m] - ls[m])):.1f} us; tail chunks after p50 "
                  f"{np.median(nt[m]):.0f}; exit p50 {np.median(ext[m]) - q0:.1f}", flush=True)
    # waves still running a chunk that started before the queue ran out: how long did those chunks take?
    pre = ok & (lstart < q0)
    if pre.any():
        print(f"    last chunks started before the queue ran out ({int(pre.sum())} waves): lasted p50 "
              f"{np.nanmedian(dur[pre]):.1f} p90 {np.nanpercentile(dur[pre], 90):.1f} max {np.nanmax(dur[pre]):.1f} us",
              flush=True)


def main():
    import numpy as np
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext
    from mirror_maze.dist import row_shard

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="MM_OPT key:value (repeatable)")
    ap.add_argument("--batch", type=int, default=1, help="frames per launch (mm_trace_tile_frames), as bench.py")
    ap.add_argument("--tail", action="store_true",
                    help="attribute the launch tail (needs a -DMM_TAIL_CLOCKS build via MIRROR_MAZE_LIB): per XCD "
                         "(HW_REG_XCC_ID) exit times, and each wave's last chunk duration")
    a = ap.parse_args()
    maze_n, W, H, spp, bl, ml, desc = CONFIGS[a.config]
    r = Renderer(0)
    for kv in a.opt:
        k, v = kv.split(":")
        r.set_option(int(k), int(v))
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    ts = torch.zeros((5 * TIMELINE_WAVES, 4), dtype=torch.int64, device="cuda")
    print(f"# {desc}; times in us (wall_clock64, 100 MHz)")
    for n in [int(x) for x in a.ranks.split(",")]:
        y0, stride, rows = row_shard(H, n, 0)
        out = torch.zeros((a.batch, rows, W, 4), dtype=torch.float32, device="cuda")

        def launch(frame):
            if a.batch > 1:
                r.trace_tile_frames(u, make_ext(spp, bl, ml, frame=frame), a.batch, 0, y0, W, rows, y_stride=stride,
                                    out=out)
            else:
                r.trace_tile(u, make_ext(spp, bl, ml, frame=frame), 0, y0, W, rows, y_stride=stride, out=out[0])
        launch(99)
        for f in range(a.frames):
            ts.zero_()
            r.set_wave_timeline(ts)
            launch(f)
            torch.cuda.synchronize()
            r.set_wave_timeline(None)
            t = ts.cpu().numpy()[:TIMELINE_WAVES]
            t = t[t[:, 2] > 0]
            t0 = t[:, 0].min()
            ent, stg, ext, ch = ((t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0, t[:, 3])
            span = ext.max()
            busy = (ext - np.maximum(stg, ent)).sum()
            print(f"N={n} f{f}: waves {len(t)} span {span:8.1f}  entry p50/max {np.median(ent):6.1f}/{ent.max():6.1f}  "
                  f"staged p50/max {np.median(stg):6.1f}/{stg.max():6.1f}  exit min/p10/p50/p90/max "
                  f"{ext.min():7.1f}/{np.percentile(ext, 10):7.1f}/{np.median(ext):7.1f}/{np.percentile(ext, 90):7.1f}/"
                  f"{ext.max():7.1f}  tail {span - ext.min():6.1f} ({(span - ext.min()) / span:.1%})  "
                  f"chunks/wave {ch.mean():.2f} [{ch.min()}-{ch.max()}]  wave-busy {busy / (len(t) * span):.1%}",
                  flush=True)
            # what balancing the last chunks' paths inside each block could reach: a block's waves
            # finish together at their mean exit (blocks = consecutive 16-wave groups by wave id)
            wid = np.nonzero(ts.cpu().numpy()[:TIMELINE_WAVES, 2] > 0)[0]
            blk = wid // 16
            bmean = np.array([ext[blk == b].mean() for b in np.unique(blk)])
            print(f"    block-balanced bound: last block mean exit {bmean.max():7.1f} (vs last wave {span:7.1f}); "
                  f"chip mean exit {ext.mean():7.1f}", flush=True)
            if a.tail:
                tail_report(ts.cpu().numpy(), t0, np)
    r.close()


if __name__ == "__main__":
    main()
