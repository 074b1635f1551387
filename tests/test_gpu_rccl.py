"""The multi-GPU frame path on the MI355X with the "nccl" backend (RCCL): a
fresh torchrun process group renders frames through FrameGatherer
(scripts/rccl_frames.py) and the assembled frames must equal trace_tile's,
bit for bit.  The reference runs one Metal device (src/main.rs:616); the
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
