"""The multi-GPU frame path on the MI355X: a fresh torchrun job renders
frames through the library's RCCL communicator (mm_comm_init_rank +
mm_gather_rows, scripts/rccl_frames.py) and the assembled frames must equal
trace_tile's, bit for bit; bench.py's N-GPU path, started by the driver's
torchrun command and by `bench.py --gpus 1 --launcher torchrun`, delivers the
same frame.  The reference runs one Metal device (src/main.rs:616); the
gather is the build's replacement for that single-device plumbing."""
from __future__ import annotations

import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("config,frames", [("c1", 3), ("c3", 2)])
def test_rccl_gathered_frames_equal_trace_tile(gpu, tmp_path, config, frames):
    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    out = tmp_path / f"{config}.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(REPO / "scripts" / "rccl_frames.py"), "--config", config, "--frames", str(frames), "--out", str(out)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    got = np.load(out)
    maps = (tmp_path / f"{config}.npy.maps.txt").read_text()
    assert "librccl" in maps, maps
    maze_n, W, H, spp, bl, ml, _ = CONFIGS[config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    assert got.shape == (frames, H, W, 4)
    for f in range(frames):
        want, _ = r.trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, 0, W, H)
        assert torch.equal(torch.from_numpy(got[f]).view(torch.int32), want.cpu().view(torch.int32)), f
    r.close()


@pytest.mark.parametrize("config,launcher", [("c2", "driver"), ("c3", "driver"), ("c2", "bench")])
def test_bench_distributed_path_delivers_the_frame(gpu, tmp_path, config, launcher):
    """bench.py exactly as the driver launches it for N GPUs (torchrun, the
    "nccl" backend), at N = 1: batched launches, the RGBA8 conversion on the
    rank, the RCCL gather and the de-interleave on rank 0.  The frame rank 0
    holds after the timed steps must equal the texture-write conversion of
    trace_tile's last frame, byte for byte (C2: one launch without tail
    deferral; C3: three frames, 50 M paths, with it).  launcher "bench":
    `bench.py --gpus 1 --launcher torchrun` starts the same torchrun job as a
    child and relays its line."""
    import json

    import torch

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    out = tmp_path / "frame.npy"
    steps = 3
    args = ["--gpus", "1", "--config", config, "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline",
            "--save-frame", str(out)]
    if launcher == "driver":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py")] + args
    else:
        cmd = [sys.executable, str(REPO / "bench.py")] + args + ["--launcher", "torchrun"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["config"]["frame_format"] == "rgba8"
    assert "RCCL" in line["config"]["parallelism"]
    # the multi-GPU instrumentation, consistent at N = 1
    d = line["distributed"]
    assert d["rccl_world"] == 1 and d["torch_distributed_world"] == 1 and "mm_gather_rows" in d["backend"]
    assert d["rccl_version"] >= 22600
    k = d["kernel_ms_per_rank"]
    assert k["min"] == k["max"] == k["rank0"] > 0
    assert abs(k["rank0"] - line["roofline"]["kernel_avg_ms"] * line["roofline"]["launches"]) < 0.01
    g = d["exposed_gather_ms"]
    assert 0 <= g["rank0"] <= g["max"] <= line["ms_per_step"] * steps
    assert d["frames_per_gather"] == line["config"]["frames_per_launch"] and d["gathers_total"] >= 1
    got = np.load(out)
    maze_n, W, H, spp, bl, ml, _ = CONFIGS[config]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    want, _ = r.trace_tile(default_uniform(W, H, 0), make_ext(spp, bl, ml, frame=steps - 1), 0, 0, W, H)
    want8 = r.quantize(want).cpu().numpy()
    assert got.dtype == np.uint8 and got.shape == (H, W, 4)
    assert np.array_equal(got, want8)
    r.close()


@pytest.mark.parametrize("n_ranks", [2, 8])
def test_bench_n_ranks_on_one_gpu_run_the_n_gpu_path(gpu, tmp_path, n_ranks):
    """the product's N-rank path executed end to end on
    one GPU.  `bench.py --gpus N --shared-gpu` starts N ranks (torchrun, as for
    N GPUs) that all trace on GPU 0; their tiles reach rank 0 as host copies
    over gloo into mm_assemble_rows (mirror_maze.comm.HostComm: RCCL allows one
    rank per GPU) -- everything else is the N-GPU run: the interleaved row
    sets, NativeGatherer's slots and events, the rank >= 1 branches, the
    exposed-gather clock and the reductions.  Rank 0's saved frame must equal
    the texture-write conversion of trace_tile's last frame byte for byte, the
    ranks' rays must add up to the 1-GPU frames' rays, and n_gpus is N."""
    import json

    from bench import CONFIGS
    from mirror_maze import Renderer, Scene, default_uniform, make_ext

    out = tmp_path / "frame.npy"
    steps = 3
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", str(n_ranks), "--shared-gpu", "--config", "c2",
           "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline", "--save-frame", str(out)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == n_ranks and "diagnostics" in line["config"]["parallelism"]
    d = line["distributed"]
    assert d["shared_gpu"] is True and d["torch_distributed_world"] == n_ranks and d["rccl_world"] is None
    assert "HostComm" in d["backend"] and d["gathers_total"] >= 1
    k = d["kernel_ms_per_rank"]
    assert 0 < k["min"] <= k["max"]
    assert line["roofline"]["frac"] is None  # diagnostics: no roofline
    maze_n, W, H, spp, bl, ml, _ = CONFIGS["c2"]
    r = Renderer(0)
    r.upload_scene(Scene.build(maze_n, 0))
    u = default_uniform(W, H, 0)
    rays = 0
    for f in range(steps):
        img, st = r.trace_tile(u, make_ext(spp, bl, ml, frame=f), 0, 0, W, H, stats=True)
        rays += st.rays
    assert line["config"]["rays_total"] == rays
    got = np.load(out)
    assert got.dtype == np.uint8 and got.shape == (H, W, 4)
    assert np.array_equal(got, r.quantize(img).cpu().numpy())
    r.close()
