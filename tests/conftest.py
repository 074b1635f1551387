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
