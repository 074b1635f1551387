"""Test configuration: `-m gpu` tests need an MI355X; everything else runs on CPU."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "mirror-maze_amd"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the C ABI on the GPU)")
    config.addinivalue_line("markers", "slow: longer CPU-side checks")


def _ensure_built():
    lib = PKG / "lib" / "libmirror_maze.so"
    orc = REPO / "oracle" / "_build" / "libmm_oracle.so"
    if not orc.exists():
        subprocess.run(["make", "-s", "-C", str(REPO / "oracle")], check=True)
    if not lib.exists():
        subprocess.run(["make", "-s", "-j8", "-C", str(PKG)], check=True)


_ensure_built()


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU visible")
    import torch

    torch.cuda.init()
    return torch.device("cuda:0")


def host_threads() -> int:
    """Worker threads for CPU-side oracle runs: the usable CPUs of this
    process, capped at 16 (a GPU box's CPU share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def oracle_tile(o, uniform, ext, x0, y0, w, h, y_stride=1, threads=None, out=None):
    """oracle_trace_tile over a thread pool (the C call releases the GIL): the
    tile's rows in bands, bit-identical to one call (each pixel's value
    depends on its own (pixel, sample, frame) only).  `out` (h, w, 4) float32
    receives the tile (with MM_EXT_ACCUMULATE: adds into it).  Returns (out,
    rays)."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor

    threads = threads or host_threads()
    if out is None:
        out = np.zeros((h, w, 4), dtype=np.float32)
    band = max(1, -(-h // (4 * threads)))
    jobs = [(j0, min(band, h - j0)) for j0 in range(0, h, band)]

    def run(job):
        j0, n = job
        part, st = o.trace_tile(uniform, ext, x0, y0 + j0 * y_stride, w, n, y_stride=y_stride, out=out[j0:j0 + n])
        return st.rays

    with ThreadPoolExecutor(threads) as ex:
        rays = sum(ex.map(run, jobs))
    return out, rays
