#!/usr/bin/env python
"""bench.py — Mrays/s + ms/frame of mirror-maze's ray-trace loop on MI355X.

Headline workload (BASELINE.json configs[2], "C3"): 32x32 maze, 1920x1080,
8 spp, bounce_limit 8, mirror_limit 8.  A "step" is one full frame: every
pixel x sample path traced through the HIP kernels (no work skipped), frame
index = step number (fresh RNG every step).  A "ray" is one closest-hit BVH
query (src/shaders.metal:307).

N GPUs: one process per GPU.  `bench.py --gpus N` started on its own starts
`python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a
child and relays rank 0's line (so --gpus always means N GPUs); under a
launcher (WORLD_SIZE set, as the driver runs it) WORLD_SIZE must equal --gpus.
The frame's rows are interleaved over ranks (rank r renders rows r, r+N, ...),
and rank 0 receives every rank's tiles with one RCCL gather per multi-frame
launch through the library's C ABI (mm_gather_rows: ncclSend/ncclRecv + a
de-interleave kernel, include/mm_comm.h), issued on its own stream (north
star: "tiles of the framebuffer shard one-per-GPU ... single RCCL gather at
frame end"); torch.distributed (gloo, on the CPU) carries only the
rendezvous, barriers and the timing reductions.  Total work is fixed as N
grows -> "scaling": "strong".

Prints ONE JSON line on rank 0 (driver contract), with the roofline of the
dominant kernel (HIP-event timed inside the timed region) and a CPU baseline
(the oracle restatement on a bounded row sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "mirror-maze_amd"))
sys.path.insert(0, str(REPO))

CONFIGS = {
    # id: (maze_n, W, H, spp, bounce_limit, mirror_limit, description)
    "c1": (16, 256, 256, 1, 1, 15, "C1: 16x16 maze, 256x256, 1 spp, 1 bounce"),
    "c2": (16, 1920, 1080, 1, 4, 15, "C2: 16x16 maze, 1920x1080, 1 spp, 4 bounces"),
    "c3": (32, 1920, 1080, 8, 8, 8, "C3: 32x32 maze, 1920x1080, 8 spp, 8 mirror bounces"),
    "c4": (32, 3840, 2160, 16, 8, 15, "C4: 32x32 maze, 3840x2160, 16 spp, 8 bounces"),
    "c5": (64, 3840, 2160, 64, 16, 16, "C5 frame: 64x64 maze, 3840x2160, 64 spp, 16/16 bounces"),
    "c5s": (64, 1920, 1080, 8, 16, 16, "C5 scene at C3 size: 64x64 maze, 1920x1080, 8 spp, 16/16 bounces"),
}
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 78.6          # 256 CU x 4 SIMD x 32 lanes/cycle x 2.4 GHz, non-packed fp32 lane-ops
BYTES_PER_RAY = 136            # SoA path state read+write + hit record
BYTES_PER_PIXEL = 16           # float4 output
OPS_PER_AABB, OPS_PER_RECT = 25, 71  # SURVEY.md §8(d) VALU model of the reference BVH walk
SRC_GLOBS = ("mirror-maze_amd/csrc/*", "mirror-maze_amd/Makefile", "include/*.h")


def src_hash() -> str:
    """sha256 (16 hex) of the product sources the trace kernels are built from;
    a PMC profile under profiles/ is used only when it carries the same hash."""
    import hashlib

    h = hashlib.sha256()
    for pat in SRC_GLOBS:
        for f in sorted(REPO.glob(pat)):
            if f.is_file():
                h.update(str(f.relative_to(REPO)).encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


def usable_cpus():
    """CPUs this process may run on: its affinity set, capped by the cgroup's
    cpu.max quota (a GPU box gives each GPU a share of its host's CPUs).
    Returns (count, basis)."""
    import math

    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n, basis = aff, f"sched_getaffinity {aff} of {os.cpu_count()} online CPUs"
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            q = max(1, math.ceil(int(quota) / int(period)))
            if q < n:
                n = q
                basis += f", cgroup cpu.max quota {quota}/{period} = {q} CPUs"
    except (OSError, ValueError):
        pass
    return n, basis


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--launcher", default="auto", choices=["auto", "torchrun"],
                   help="auto: N > 1 GPUs without a launcher start torchrun as a child; torchrun: also at N = 1 "
                        "(the multi-GPU frame path -- RCCL communicator, gather -- on one rank)")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--pipeline", default="auto", choices=["auto", "mega", "wave"])
    p.add_argument("--contexts", type=int, default=0,
                   help="renderer contexts (one stream each) that consecutive frames alternate over; "
                        "0 = 1 on one GPU, 2 when the frame is split over ranks")
    p.add_argument("--batch", type=int, default=32,
                   help="frames per launch at most (mm_trace_tile_frames: the frames share one work queue, so "
                        "the launch's drain and its tail kernel are paid once per launch, not per frame); 1 = one "
                        "frame per launch (then --contexts applies); 0 = time 1 context / 2 contexts / batches of "
                        "8 after warmup and keep the fastest")
    p.add_argument("--frame-format", default="rgba8", choices=["rgba8", "f32"],
                   help="format of the frame each step delivers on rank 0: rgba8 = the reference's output "
                        "texture format (RGBA8Unorm, src/main.rs:702-709; the texture-write conversion "
                        "written by the trace itself, MM_EXT_RGBA8, then the gather moves 4 B/px), f32 = the float tile "
                        "(16 B/px).  Accumulated runs (--accumulate) gather their f32 running sum.")
    p.add_argument("--accumulate", action="store_true",
                   help="temporal accumulation (C5): every frame adds into one running sum per rank "
                        "(MM_EXT_ACCUMULATE) and the frame is gathered once, after the last step")
    p.add_argument("--shared-gpu", action="store_true",
                   help="diagnostics: the N ranks all use GPU 0 and their tiles reach rank 0 as host copies over "
                        "torch.distributed (gloo) into mm_assemble_rows (mirror_maze.comm.HostComm; RCCL allows "
                        "one rank per GPU) -- the rest of the N-GPU path runs unchanged; its timing is not a "
                        "measurement (VERDICT r05 item 2)")
    p.add_argument("--emulate-ranks", type=int, default=0,
                   help="diagnostics on one GPU: trace only rank 0's row set of an N-rank split")
    p.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                   help="mm_set_option on every context (MM_OPT_* numbers, include/mm_api.h); results never change")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (approx)")
    p.add_argument("--src-hash", action="store_true", help="print the product source hash and exit")
    p.add_argument("--save-frame", default="", help="rank 0 saves the last timed frame as it was delivered "
                                                    "(.npy; tests/test_gpu_rccl.py checks it)")
    return p.parse_args()


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(args, env, argv, port=None):
    """How this invocation runs: ("run", None) in this process, ("child", cmd)
    to start one process per GPU under torch.distributed.run (this script, the
    same arguments), or ("error", message).  Decided before torch is imported
    or any GPU is touched (--gpus N must mean N GPUs)."""
    ws = env.get("WORLD_SIZE")
    if args.gpus < 1:
        return "error", f"--gpus {args.gpus}: need at least one GPU"
    if ws is not None:
        if int(ws) != args.gpus:
            return "error", (f"bench.py --gpus {args.gpus} under a launcher with WORLD_SIZE={ws}: the GPU count and "
                             f"the number of ranks must agree (one process per GPU)")
        return "run", None
    if args.gpus > 1 or args.launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()),
               str(REPO / "bench.py")] + list(argv)
        return "child", cmd
    return "run", None


def relay_child(cmd) -> int:
    """Run the per-GPU ranks as a child process (never exec: see the harness
    rules); rank 0's one JSON line goes to stdout, everything else to stderr.
    Returns the exit status to leave with."""
    import subprocess

    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in p.stdout.splitlines():
        try:
            obj = json.loads(ln)
        except ValueError:
            obj = None
        if isinstance(obj, dict) and "metric" in obj:
            line = ln
        elif ln.strip():
            print(ln, file=sys.stderr)
    if line is not None:
        print(line, flush=True)
    if p.returncode:
        return p.returncode
    return 0 if line is not None else 1


def launch_sizes(count: int, per_launch: int) -> list:
    """Frames per launch for `count` consecutive frames, at most `per_launch`
    each: ceil(count / per_launch) launches of sizes as equal as possible."""
    if count <= 0:
        return []
    n = -(-count // per_launch)
    sizes, left = [], count
    for j in range(n):
        sizes.append(left // (n - j))
        left -= sizes[-1]
    return sizes


def _cpu_rate(o, u, ext, W, H, budget_s, threads):
    """Rays/s of Oracle `o` over a bounded row sample of the frame: calibrated
    on one row, then every stride-th row on `threads` threads (GIL released in
    C).  Returns (rays, seconds, sample text, seconds per row)."""
    t0 = time.perf_counter()
    o.trace_tile(u, ext, 0, H // 2, W, 1)
    row_s = max(time.perf_counter() - t0, 1e-6)
    rows = int(max(threads, min(H, budget_s * threads / row_s)))
    stride = max(1, H // rows)
    sample_rows = list(range(0, H, stride))[:rows]
    totals = [0] * threads
    lock = threading.Lock()
    work = list(sample_rows)

    def worker(i):
        while True:
            with lock:
                if not work:
                    return
                y = work.pop()
            _, s = o.trace_tile(u, ext, 0, y, W, 1)
            totals[i] += s.rays

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    rays = sum(totals)
    return rays, dt, f"{len(sample_rows)} of {H} rows (every {stride}th) x {W} px x {ext.spp} spp, " \
                     f"{rays} rays in {dt:.1f} s", row_s


def cpu_baseline(scene, u, ext, W, H, budget_s):
    """Two CPU baselines on the host cores, each on a bounded row sample of the
    same workload, one thread per core:
    * the oracle (oracle/mm_oracle.c, scalar C -O2): the reference's algorithm,
      the BVH walk on every query (kind "port"), plus its single-core rate;
    * same_algorithm (oracle/grid_cpu.c): the oracle's path loop with the
      product's certified grid search as the query -- the GPU's algorithm on the
      CPU, so the GPU / CPU ratio can be read with the algorithm held fixed.
    Both return the reference walk's answers (identical images)."""
    from oracle.oracle import Oracle

    o = Oracle.from_scene(scene)
    threads, basis = usable_cpus()
    rays, dt, sample, row_s = _cpu_rate(o, u, ext, W, H, budget_s, threads)
    # the same loop on one core (SURVEY 8d asks for both), ~budget/4 seconds of rows
    n1 = int(max(1, min(H, budget_s / 4 / row_s)))
    t0 = time.perf_counter()
    rays1 = 0
    for y in range(0, H, max(1, H // n1))[:n1]:
        _, s1 = o.trace_tile(u, ext, 0, y, W, 1)
        rays1 += s1.rays
    dt1 = time.perf_counter() - t0
    og = Oracle.from_scene(scene, method="grid")
    grays, gdt, gsample, _ = _cpu_rate(og, u, ext, W, H, budget_s / 2, threads)
    gst = Oracle.grid_stats()
    if gst["other_scene"]:
        raise RuntimeError(f"same-algorithm CPU baseline walked {gst['other_scene']} queries of another scene")
    gsample += (f"; {gst['grid']} queries answered by the grid, {gst['fallback']} by the reference walk "
                f"(ties, failed certificates, rays outside the guards)")
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "cores_basis": basis,
            "kind": "port",
            "sample": f"{sample}; scalar C oracle -O2 -ffp-contract=off (the reference BVH walk per query)",
            "single_core": {"value": round(rays1 / dt1 / 1e6, 3), "unit": "Mrays/s",
                            "sample": f"{n1} rows, {rays1} rays in {dt1:.1f} s"},
            "same_algorithm": {"value": round(grays / gdt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
                               "kind": "same-algorithm",
                               "sample": f"{gsample}; oracle/grid_cpu.c: the certified grid search (the GPU's "
                                         f"query method) in the oracle's path loop, scalar C -O2"},
            "host_cpus": os.cpu_count()}


def pmc_record_name(config: str, ranks: int) -> str:
    """profiles/pmc_<name>.json of a launch shape: the configuration's whole
    frames at N = 1, rank 0's row set of an N-way split otherwise (the shape
    rank 0 runs at world = N, and --emulate-ranks N on one GPU)."""
    return config + (f"_r{ranks}" if ranks > 1 else "")


def pmc_profile(args, frames_per_launch, k_avg_s, world, shared=False):
    """Measured counters of the dominant kernel from profiles/pmc_<name>.json
    (scripts/pmc_record.py over rocprofv3 --pmc passes of bench.py's own
    launch), used only when its source hash is this tree's.  The record is
    the launch shape rank 0 runs: pmc_<config>.json at N = 1,
    pmc_<config>_r<N>.json at world = N > 1 and for --emulate-ranks N, so the
    N-GPU lines' headline is the same quantity as N = 1's (VERDICT r05 item
    1).  Returns (measured dict, HBM bytes per launch or None)."""
    if shared:
        return {"source": None, "note": "diagnostics (--shared-gpu): N ranks share one GPU, no roofline"}, None
    ranks = world if world > 1 else (args.emulate_ranks if args.emulate_ranks > 1 else 1)
    f = REPO / "profiles" / f"pmc_{pmc_record_name(args.config, ranks)}.json"
    if not f.exists() or args.pipeline != "auto" or args.opt:
        return {"source": None, "note": f"no PMC record for this launch shape ({f.relative_to(REPO)}, default "
                                        f"options)"}, None
    rec = json.loads(f.read_text())
    here = src_hash()
    if rec.get("src_hash") != here:
        # other kernel sources: only its executed lane-ops per frame, scaled to this run's frames per launch, is
        # offered (labelled) beside a null headline; its HBM bytes are not used
        stale = {"source": str(f.relative_to(REPO)), "stale": True, "profile_src_hash": rec.get("src_hash"),
                 "src_hash": here, "note": "profile of other kernel sources: HBM bytes not used"}
        if rec.get("valu_lane_ops_per_launch") and rec.get("frames_per_launch"):
            per_frame = rec["valu_lane_ops_per_launch"] / rec["frames_per_launch"]
            stale["stale_valu_lane_ops_tops"] = round(per_frame * frames_per_launch / k_avg_s / 1e12, 3)
        return stale, None
    scale = frames_per_launch / rec["frames_per_launch"]
    hbm = rec["hbm_bytes_per_launch"] * scale
    m = {"source": str(f.relative_to(REPO)), "src_hash": here, "git_head": rec.get("git_head"),
         "hbm_bytes_per_launch": round(hbm), "hbm_gbs": round(hbm / k_avg_s / 1e9, 1),
         "hbm_frac": round(hbm / k_avg_s / 1e9 / HBM_PEAK_GBS, 5),
         "valu_issue_share": rec.get("valu_issue_share"), "lane_utilisation": rec.get("lane_utilisation"),
         "valu_lane_ops_tops": (round(rec["valu_lane_ops_per_launch"] * scale / k_avg_s / 1e12, 3)
                                if rec.get("valu_lane_ops_per_launch") else None),
         "profile_kernel_avg_ms": rec.get("kernel_avg_ms"),
         # the record alone: its lane-ops per launch / its own mean launch time / peak
         "profile_frac": (round(rec["valu_lane_ops_per_launch"] / (rec["kernel_avg_ms"] / 1e3) / 1e12
                                / VALU_PEAK_TOPS, 4)
                          if rec.get("valu_lane_ops_per_launch") and rec.get("kernel_avg_ms") else None),
         "note": ("rocprofv3 --pmc passes: HBM = 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE; lane "
                  "utilisation = SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU); issue share = SQ_INSTS_VALU / "
                  "(1024 SIMDs x cycles / 2); per launch, scaled to this run's frames per launch")}
    return m, round(hbm)


def roofline(ops, alg_bytes, k_avg_s, k_launches, frames_per_launch, measured, traffic, contexts, kern_res):
    """The dominant kernel's roofline object.  Headline (achieved / frac): the
    hardware's executed VALU lane-ops per launch (fp32, integer, compare and
    select alike) from the same-source PMC record of this launch shape
    (SQ_INSTS_VALU x 64 x lane utilisation) / this run's mean launch time,
    against 78.6 T lane-ops/s.  Without such a record
    achieved / frac are null and "basis" says why -- never a model (VERDICT
    r05 item 1).  The reference-walk VALU model and the 136 B/ray HBM model
    are labelled sub-objects with a "model_ratio" (a model's count over the
    peak, which can pass 1 -- not a measured fraction)."""
    ref_tops = ops / k_avg_s / 1e12
    lane_tops = measured.get("valu_lane_ops_tops") if isinstance(measured, dict) else None
    stale_tops = measured.get("stale_valu_lane_ops_tops") if isinstance(measured, dict) else None
    hw = lane_tops is not None
    return {
        "bound": "valu", "achieved": round(lane_tops, 3) if hw else None, "peak": VALU_PEAK_TOPS,
        "unit": "T lane-ops/s",
        "frac": round(lane_tops / VALU_PEAK_TOPS, 4) if hw else None, "traffic": traffic,
        "stale": (not hw) and stale_tops is not None,
        "basis": ("executed VALU lane-ops (PMC: SQ_INSTS_VALU x 64 x SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU), "
                  f"{measured.get('source')} of these sources, this launch shape) per launch / mean launch time"
                  if hw else
                  "none: " + (measured.get("note") or "no PMC record of these sources") +
                  " -- achieved / frac null (the models below are not measurements)"),
        "stale_profile": ({"valu_lane_ops_tops": stale_tops, "model_ratio": round(stale_tops / VALU_PEAK_TOPS, 4),
                           "note": "executed lane-ops per frame of the PMC record of OTHER kernel sources "
                                   "(measured.profile_src_hash) x this run's frames per launch / mean launch "
                                   "time -- not measured on these sources"}
                          if (not hw) and stale_tops is not None else None),
        "peak_basis": "256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz (MI355X_MICROARCH.md)",
        "kernel": "k_trace_wavepersist", "kernel_avg_ms": round(k_avg_s * 1e3, 3),
        "launches": k_launches, "frames_per_launch": round(frames_per_launch, 3),
        "timing": ("HIP events around each launch on its stream" +
                   ("; 2 contexts: consecutive launches overlap, so a launch's "
                    "span includes time shared with its neighbours" if contexts > 1 else "")),
        "kernel_resources": kern_res,
        "reference_equivalent": {
            "lane_ops_tops": round(ref_tops, 3), "model_ratio": round(ref_tops / VALU_PEAK_TOPS, 4),
            "ops": ("VALU lane-ops the reference BVH walk would execute on the timed frames (SURVEY 8d "
                    "model: 25 per AABB test + 71 per rect test, counted by the BVH loop form) per launch / "
                    "mean launch time: useful work per second, not what this kernel executes (it passes 1 "
                    "where the grid search does far less work than the walk)")},
        "model_hbm": {"bytes_per_ray": BYTES_PER_RAY, "bytes_per_launch": round(alg_bytes),
                      "gbs": round(alg_bytes / k_avg_s / 1e9, 1), "peak_gbs": HBM_PEAK_GBS,
                      "model_ratio": round(alg_bytes / k_avg_s / 1e9 / HBM_PEAK_GBS, 4),
                      "note": ("SURVEY 8(d) accounting model of a SoA wavefront (136 B/ray + 16 "
                               "B/px), not traffic: the megakernel keeps path state in registers and never "
                               "moves these bytes (measured traffic: roofline.traffic / measured)")},
        "measured": measured,
    }


def main():
    args = parse()
    if args.src_hash:
        print(src_hash())
        return
    how, what = launch_plan(args, os.environ, sys.argv[1:])
    if how == "error":
        print(f"bench.py: {what}", file=sys.stderr)
        sys.exit(2)
    if how == "child":
        sys.exit(relay_child(what))
    # Exactly one JSON line on stdout: anything else written to fd 1 (e.g. the
    # RCCL banner at communicator init) is sent to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import numpy as np
    import torch
    import torch.distributed as dist

    from mirror_maze import MM_PIPE_AUTO, MM_PIPE_MEGAKERNEL, MM_PIPE_WAVEFRONT, Renderer, Scene
    from mirror_maze import MM_EXT_ACCUMULATE, default_uniform, make_ext

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.shared_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    # under torchrun (even with one rank) the frame goes through the RCCL gather path; torch.distributed (gloo,
    # CPU) is only the rendezvous, the barriers and the timing reductions -- the frames move through the
    # library's own RCCL communicator (include/mm_comm.h)
    distributed = "WORLD_SIZE" in os.environ and "MASTER_PORT" in os.environ
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    maze_n, W, H, spp, bl, ml, desc = CONFIGS[args.config]
    scene = Scene.build(maze_n, 0)
    # Issue modes.  Every launch ends in a ~0.4 ms tail in which the last waves
    # finish their last chunks (profiles/r01/timeline_probe.txt) -- 4 % of a
    # C3 frame, 25 % of a rank's frame at N = 8.  Default (--batch 32): frames
    # are independent, so up to 32 consecutive frames share ONE launch's work
    # queue (mm_trace_tile_frames) and the tail is paid once per launch.
    # --batch 1: one frame per launch, optionally alternating over two
    # renderer contexts on their own streams so frame k+1's blocks fill the
    # CUs frame k's tail leaves idle (two frames sharing the GPU run ~7 %
    # slower, profiles/r01/overlap_probe.txt; --contexts 0 times both).
    n_ctx = (1 if args.accumulate else args.contexts if args.contexts > 0 else 1 if args.batch > 1 else 2)
    rens = []
    for _ in range(n_ctx):
        r = Renderer(local)
        r.set_pipeline({"auto": MM_PIPE_AUTO, "mega": MM_PIPE_MEGAKERNEL, "wave": MM_PIPE_WAVEFRONT}[args.pipeline])
        r.upload_scene(scene)
        for kv in args.opt:
            k, v = kv.split("=")
            r.set_option(int(k), int(v))
        rens.append(r)
    streams = [r.own_stream() for r in rens]
    u = default_uniform(W, H, 0)
    comm = None
    if distributed and args.shared_gpu:  # diagnostics: every rank on GPU 0, tiles over gloo (HostComm)
        from mirror_maze.comm import HostComm

        comm = HostComm(rens[0], world, rank)
    elif distributed:  # the library's RCCL communicator: rank 0's unique id over the gloo rendezvous
        from mirror_maze.comm import Comm

        uid = [Comm.unique_id(rens[0]) if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm.init_rank(rens[0], world, rank, uid[0])

    # rows r, r+world, ... (mirror_maze/dist.py); pad so every rank sends the same shape
    from mirror_maze.comm import NativeGatherer
    from mirror_maze.dist import row_shard, rows_max

    y0, y_stride, my_rows = row_shard(H, world, rank)
    if args.emulate_ranks > 1 and world == 1:
        y0, y_stride, my_rows = row_shard(H, args.emulate_ranks, 0)
    # the frame each step delivers: RGBA8 (the reference's texture format) or f32
    rgba8 = args.frame_format == "rgba8" and not args.accumulate
    fdt = torch.uint8 if rgba8 else torch.float32
    frame_buf = torch.empty((H, W, 4), dtype=fdt, device=dev) if rank == 0 else None
    # multi-frame launches need the wave-persistent kernel's fused resolve (64 % spp == 0)
    # (with the mirror-tail deferral -- MM_OPT_DEFER, or spp that does not divide 64 -- samples are staged per
    # frame, any spp)
    batchable = not args.accumulate
    fb_max = (min(args.batch, max(args.steps, args.warmup, 8)) if args.batch > 0 else 8) if batchable else 1
    # ONE gather per launch (a multi-frame launch's frames all finish together; per frame with --batch 1),
    # mm_gather_rows on its own stream into rotating tile slots, so the next launch never waits on it
    # (mirror_maze.comm.NativeGatherer)
    asm_stream = torch.cuda.Stream(dev) if distributed else None
    gatherer = (NativeGatherer(comm, (rows_max(H, world), W, 4), H, fb_max, dev, dtype=fdt,
                               slots=max(2, len(rens)), gather_stream=asm_stream)
                if distributed else None)
    bgather = gatherer if distributed and fb_max > 1 else None
    tiles1 = None if distributed else [torch.zeros((H, W, 4), dtype=fdt, device=dev) for _ in rens]
    last = [0]
    active = [len(rens)]  # contexts the frames alternate over
    batch = [1]           # frames per launch (mm_trace_tile_frames), single context
    # per context: the launch's float frames (and their RGBA8 conversions on one GPU)
    batch_bufs = [torch.zeros((fb_max, my_rows, W, 4), dtype=torch.float32, device=dev)
                  if fb_max > 1 and not rgba8 else None for _ in rens]
    batch_bufs8 = [torch.zeros((fb_max, my_rows, W, 4), dtype=torch.uint8, device=dev)
                   if fb_max > 1 and rgba8 else None for _ in rens]
    progress_t = [time.perf_counter()]

    def progress(msg):
        # long runs (C5) print a line to stderr every ~20 s so a watchdog sees progress
        now = time.perf_counter()
        if now - progress_t[0] > 20.0:
            progress_t[0] = now
            print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)

    acc_tile = (torch.zeros((rows_max(H, world), W, 4), dtype=torch.float32, device=dev)
                if args.accumulate else None)
    trace_end = [torch.cuda.Event(enable_timing=True)] if distributed else None

    def step(k, frame, stats=False):
        slot = k % active[0]
        with torch.cuda.stream(streams[slot]):
            if acc_tile is not None:  # running sum of per-frame means; gathered once by drain()
                _, st = rens[slot].trace_tile(u, make_ext(spp, bl, ml, frame=frame, flags=MM_EXT_ACCUMULATE),
                                              0, y0, W, my_rows, y_stride=y_stride, out=acc_tile[:my_rows],
                                              stats=stats)
                if trace_end is not None:
                    trace_end[0].record(streams[slot])
                return st
            tile = gatherer.tiles(1)[0] if gatherer else tiles1[slot]
            # (an RGBA8 tile: the library writes the texture-write conversion itself, MM_EXT_RGBA8)
            _, st = rens[slot].trace_tile(u, make_ext(spp, bl, ml, frame=frame), 0, y0, W, my_rows,
                                          y_stride=y_stride, out=tile[:my_rows], stats=stats)
            if trace_end is not None:
                trace_end[0].record(streams[slot])
            if gatherer:
                gatherer.put(1)
        last[0] = slot
        return st

    def step_batch(k, frame, n, slot=0, stats=False):
        """n frames (frame, frame+1, ...) in one launch of context `slot`; each frame's tile then
        goes to the gatherer (converted / copied into its rotating tile) or stays in the batch buffer."""
        # the launch's frames (RGBA8: written by the library in the texture-write conversion, MM_EXT_RGBA8)
        buf = batch_bufs8[slot] if rgba8 else batch_bufs[slot]
        with torch.cuda.stream(streams[slot]):
            tl = bgather.tiles(n) if bgather else None
            # straight into the gatherer's tile when the rank's rows fill it, else into the batch buffer
            direct = tl is not None and my_rows == tl.shape[1]
            _, st = rens[slot].trace_tile_frames(u, make_ext(spp, bl, ml, frame=frame), n, 0, y0, W, my_rows,
                                                 y_stride=y_stride, out=tl if direct else buf[:n], stats=stats)
            if trace_end is not None:  # the launch's end on its stream (exposed-gather clock, N > 1)
                trace_end[0].record(streams[slot])
            if bgather:
                if not direct:
                    for f in range(n):
                        tl[f][:my_rows].copy_(buf[f])
                bgather.put(n)
        last[0] = slot
        return st

    def run_frames(k0, frame0, count):
        """count frames starting at frame0 in the current issue mode"""
        if batch[0] > 1:
            i = n = 0
            # launches alternate over the active contexts (their streams): with two, a launch's
            # drain and tail kernel overlap the next launch
            per = batch[0] if active[0] == 1 else min(batch[0], -(-count // active[0]))
            for li, n in enumerate(launch_sizes(count, per)):
                step_batch(k0 + i, frame0 + i, n, slot=li % active[0])
                i += n
            if not bgather and count > 0:  # the last frame, for frame_buf
                sl = last[0]
                with torch.cuda.stream(streams[sl]):
                    tiles1[sl][:my_rows].copy_(batch_bufs8[sl][n - 1] if rgba8 else batch_bufs[sl][n - 1])
        else:
            for i in range(count):
                step(k0 + i, frame0 + i)

    def gather_accumulated():
        with torch.cuda.stream(streams[0]):
            if gatherer:
                gatherer.tiles(1)[0].copy_(acc_tile)
                gatherer.put(1)
            else:
                tiles1[0].copy_(acc_tile[:H])
                last[0] = 0

    def flush_gathers():
        return gatherer.flush() if gatherer else None

    def drain():
        if acc_tile is not None:
            gather_accumulated()
        f = flush_gathers()  # rank 0's last delivered frame (the current stream waits for the gathers)
        if gatherer is None:
            torch.cuda.synchronize(dev)
            frame_buf.copy_(tiles1[last[0]])
        elif f is not None:
            frame_buf.copy_(f)
        torch.cuda.synchronize(dev)

    if fb_max > 1 and args.batch > 1:  # warm up the issue mode that is timed
        active[0], batch[0] = len(rens), fb_max
        # at least one launch of the timed launches' size: the context sizes its staging buffers
        # and tail queue on the first launch that needs them (hipMalloc inside the timed region
        # otherwise: 0.6 ms of a 6.4 ms 10-frame launch at C3 / rank 0 of 8)
        run_frames(0, 10_000, max(args.warmup, min(args.steps, fb_max), len(rens)))
    else:
        for i in range(args.warmup):
            step(i, 10_000 + i)
    drain()
    calib = None
    if fb_max > 1 and args.batch > 1:
        active[0], batch[0] = len(rens), fb_max
    elif (args.batch == 0 or args.contexts == 0) and not args.accumulate:
        # issue modes: one context, two alternating contexts, one context with batches of frames
        modes = [("1", 1, 1), ("2", 2, 1)] + ([(f"batch{fb_max}", 1, fb_max)] if args.batch == 0 and fb_max > 1
                                             else [])
        calib = {}
        for rep in range(2):
            for name, m, fb in modes:
                active[0], batch[0] = m, fb
                if distributed:
                    dist.barrier()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                run_frames(0, 20_000 + 16 * rep, 8)
                drain()
                dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                if distributed:
                    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
                calib[name] = min(calib.get(name, 1e9), float(dt.item()) / 8 * 1e3)
        # the fastest mode; overlap or batching only for a clear (>1 %) gain over one context
        best = min(modes, key=lambda md: calib[md[0]])
        active[0], batch[0] = (best[1], best[2]) if calib[best[0]] < 0.99 * calib["1"] else (1, 1)
    for r in rens[:active[0]]:
        r.set_profiling(True)
        r.kernel_timing(reset=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if acc_tile is not None:
        with torch.cuda.stream(streams[0]):
            acc_tile.zero_()
    if batch[0] > 1:
        run_frames(0, 0, args.steps)
    else:
        for i in range(args.steps):
            step(i, i)
            if args.steps > 20 and i % 8 == 7:
                progress(f"timed frame {i + 1}/{args.steps} queued")
    if acc_tile is not None:
        gather_accumulated()  # C5: one gather of the accumulated frame, inside the timed region
    flush_gathers()  # the last frames' gathers + assembly are inside the timed region
    assembled = None
    if distributed:  # the frame is on rank 0 (assembled) / this rank's gather done: exposed-gather clock
        assembled = torch.cuda.Event(enable_timing=True)
        assembled.record(asm_stream)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    drain()
    for r in rens:  # errors the timed launches raised on the GPU (naming the call), outside the timing
        r.sync()
    exposed_ms = float(trace_end[0].elapsed_time(assembled)) if distributed else None
    # code-object facts of the timed kernel (hipFuncGetAttributes), before the counting re-runs below
    from mirror_maze import MM_INFO_LAST_DEFER, MM_INFO_LAST_SCRATCH, MM_INFO_LAST_STATIC_LDS, MM_INFO_LAST_VGPRS

    kern_res = {"vgprs_per_lane": int(rens[0].scene_info(MM_INFO_LAST_VGPRS)),
                "scratch_bytes_per_lane": int(rens[0].scene_info(MM_INFO_LAST_SCRATCH)),
                "static_lds_bytes_per_block": int(rens[0].scene_info(MM_INFO_LAST_STATIC_LDS)),
                "tail_rings": bool(rens[0].scene_info(MM_INFO_LAST_DEFER)),
                "source": "hipFuncGetAttributes of the timed instance (scripts/kernel_resources.py: spill counts)"}
    k_ms = k_launches = 0
    for r in rens[:active[0]]:
        ms, n = r.kernel_timing(reset=True)
        r.set_profiling(False)
        k_ms += ms
        k_launches += n

    # count the rays of exactly the timed frames (deterministic re-run, untimed), and the reference BVH
    # walk's work on the same frames (node visits = 2 AABB tests each, rect tests) with the BVH loop form,
    # whose counts equal the oracle's (tests/test_gpu_parity.py) -- the SURVEY 8(d) VALU model's inputs
    rays = paths = 0
    for i in range(args.steps):
        st = step(i, i, stats=True)
        rays += st.rays; paths += st.paths
        progress(f"counting rays: frame {i + 1}/{args.steps}")
    drain()
    from mirror_maze import MM_INFO_LEAN, MM_TRAV_LEAF_INTERIOR, MM_TRAV_LEAN
    from mirror_maze import MMError

    counter = Renderer(local)
    counter.upload_scene(scene)
    counter.set_option(7, MM_TRAV_LEAN if counter.scene_info(MM_INFO_LEAN) else MM_TRAV_LEAF_INTERIOR)
    visits = rtests = ref_rays = 0
    cnt_out = torch.empty((my_rows, W, 4), dtype=torch.float32, device=dev)
    with torch.cuda.stream(counter.own_stream()):
        for i in range(args.steps):
            try:
                _, st = counter.trace_tile(u, make_ext(spp, bl, ml, frame=i), 0, y0, W, my_rows,
                                           y_stride=y_stride, out=cnt_out, stats=True)
            except MMError:  # form 7 needs the tree + records in LDS (N=64: form 5, the same counts)
                counter.set_option(7, MM_TRAV_LEAF_INTERIOR)
                _, st = counter.trace_tile(u, make_ext(spp, bl, ml, frame=i), 0, y0, W, my_rows,
                                           y_stride=y_stride, out=cnt_out, stats=True)
            visits += st.node_visits; rtests += st.rect_tests; ref_rays += st.rays
            progress(f"counting reference work: frame {i + 1}/{args.steps}")
    torch.cuda.synchronize(dev)
    counter.close()
    assert ref_rays == rays or args.accumulate, (ref_rays, rays)
    counts = torch.tensor([rays, paths, visits, rtests], dtype=torch.float64)
    t_el = torch.tensor([elapsed], dtype=torch.float64)
    dist_info = None
    if distributed:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_el, op=dist.ReduceOp.MAX)
        # per-rank kernel time and exposed gather (so a SCALE shortfall splits into trace imbalance vs gather)
        k_lo = torch.tensor([k_ms, exposed_ms], dtype=torch.float64)
        k_hi = k_lo.clone()
        dist.all_reduce(k_lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(k_hi, op=dist.ReduceOp.MAX)
        n_gathers = gatherer.launch
        from mirror_maze.comm import Comm

        dist_info = {
            "rccl_world": None if args.shared_gpu else comm.n_ranks,
            "rccl_version": None if args.shared_gpu else Comm.rccl_version(),
            "rccl_header_version": Comm.rccl_header_version(),
            "shared_gpu": bool(args.shared_gpu),
            "backend": (("DIAGNOSTICS (--shared-gpu): every rank on GPU 0; tiles to rank 0 as host copies over "
                         "torch.distributed gloo send/recv, de-interleaved by mm_assemble_rows (mirror_maze.comm."
                         "HostComm) -- the rest of the N-GPU path unchanged; timings not a measurement")
                        if args.shared_gpu else
                        ("RCCL through libmirror_maze.so (mm_comm_init_rank + mm_gather_rows: ncclSend/ncclRecv "
                         "to rank 0, de-interleave kernel); torch.distributed " + str(dist.get_backend()) +
                         " for the rendezvous, barriers and timing reductions")),
            "torch_distributed_world": dist.get_world_size(),
            "kernel_ms_per_rank": {"rank0": round(k_ms, 3), "min": round(float(k_lo[0]), 3),
                                   "max": round(float(k_hi[0]), 3)},
            "exposed_gather_ms": {"rank0": round(exposed_ms, 3), "max": round(float(k_hi[1]), 3),
                                  "what": ("end of the last timed trace launch -> the frame assembled on rank 0 "
                                           "(other ranks: their gather done), HIP events on the device; includes "
                                           "waiting for the slowest rank's launch")},
            "frames_per_gather": (round(args.steps / max(k_launches, 1), 2) if batch[0] > 1 else 1),
            "gathers_total": n_gathers,
            "bytes_per_rank_per_frame": rows_max(H, world) * W * (4 if rgba8 else 16),
        }
    rays_all, paths_all, visits_all, rtests_all = (float(x) for x in counts.tolist())
    elapsed = float(t_el.item())

    if rank == 0:
        img = frame_buf.cpu().numpy()
        if args.save_frame:
            np.save(args.save_frame, img)
        assert np.isfinite(img).all() and img.any(), "non-finite or empty frame"
        value = rays_all / elapsed / 1e6
        # roofline of the dominant kernel (ray trace), rank 0's launches
        k_avg_s = (k_ms / 1e3) / max(k_launches, 1)
        per_launch = 1.0 / max(k_launches, 1)
        ops = (OPS_PER_AABB * 2 * visits + OPS_PER_RECT * rtests) * per_launch   # reference-walk VALU model
        alg_bytes = (BYTES_PER_RAY * rays + BYTES_PER_PIXEL * my_rows * W * args.steps) * per_launch
        frames_per_launch = args.steps * per_launch
        measured, traffic = pmc_profile(args, frames_per_launch, k_avg_s, world, shared=args.shared_gpu)
        line = {
            "metric": "Mrays/sec + ms/frame at 1920x1080, 8 spp, 8 bounces; 1/2/4/8-GPU scaling",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "samples_per_s": round(paths_all / elapsed, 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: Kruskal maze seed 0 (host C++ restatement), default camera, RNG keyed (pixel,sample,frame)",
            "config": {"workload": desc, "maze_n": maze_n, "width": W, "height": H, "spp": spp,
                       "bounce_limit": bl, "mirror_limit": ml, "pipeline": args.pipeline,
                       "parallelism": ((f"rows interleaved x{world} ranks on ONE GPU + host gather (diagnostics)"
                                        if args.shared_gpu else f"rows interleaved x{world} + RCCL gather")
                                       if distributed else "1 GPU") +
                                      (f" (emulating rank 0 of {args.emulate_ranks})" if args.emulate_ranks > 1 else ""),
                       "frame_contexts": active[0],
                       "frame_format": "rgba8" if rgba8 else "f32",
                       "frames_per_launch": (round(args.steps / max(k_launches, 1), 2) if batch[0] > 1 else 1),
                       "temporal_accumulation": bool(args.accumulate),
                       "options": args.opt or None,
                       "frame_contexts_calibration_ms": ({str(k): round(v, 3) for k, v in calib.items()}
                                                         if calib else None),
                       "rays_per_frame": int(rays_all / args.steps), "paths_per_frame": int(paths_all / args.steps),
                       "rays_total": int(rays_all),
                       "node_visits_per_ray": round(visits_all / max(rays_all, 1), 2),
                       "rect_tests_per_ray": round(rtests_all / max(rays_all, 1), 2)},
            "roofline": roofline(ops, alg_bytes, k_avg_s, k_launches, frames_per_launch, measured, traffic,
                                 active[0], kern_res),
            "distributed": dist_info,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, u, make_ext(spp, bl, ml, frame=0), W, H, args.cpu_seconds)
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    if comm is not None:
        torch.cuda.synchronize(dev)
        comm.close()
    for r in rens:
        r.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
