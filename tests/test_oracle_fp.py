"""The reference's denormal semantics.

The reference AIR is compiled with `air.compile.denorms_disable`
(src/shaders.ir metadata !47): denormals flush to zero on the Apple GPU.  The
HIP kernels and the oracle compute IEEE binary32 with denormals.  These CPU
tests run the oracle with the MXCSR sticky flags cleared and check that no
operation on the path sees a denormal operand or makes a tiny result, and
that the oracle under FTZ|DAZ (the reference's semantics) gives the same
bits -- a sample of scripts/denormal_census.py, whose full run over 504 M
queries is profiles/r03/denormal_census.json."""
from __future__ import annotations

import json

import numpy as np
import pytest

from conftest import REPO, oracle_tile


def _run_both(o, u, e, x0, y0, w, h):
    from oracle.oracle import fp_flags, set_fp_mode

    set_fp_mode(False)
    fp_flags(reset=True)
    ieee, rays = oracle_tile(o, u, e, x0, y0, w, h)
    flags = fp_flags(reset=True)
    set_fp_mode(True)
    try:
        ftz, _ = oracle_tile(o, u, e, x0, y0, w, h)
    finally:
        set_fp_mode(False)
    return ieee, ftz, flags, rays


@pytest.mark.parametrize("n,cfg,win", [
    (16, (1, 1, 15), (0, 0, 256, 256, 256, 256)),        # C1 whole frame
    (32, (8, 8, 8), (0, 500, 1920, 8, 1920, 1080)),      # C3 rows
    (64, (64, 16, 16), (1904, 1064, 32, 8, 3840, 2160)),  # a C5 window
])
def test_no_denormals_and_ftz_gives_the_same_bits(n, cfg, win):
    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import FP_DENORMAL_OPERAND, FP_UNDERFLOW, Oracle

    o = Oracle.from_scene(Scene.build(n, 0))
    x0, y0, w, h, W, H = win
    ieee, ftz, flags, rays = _run_both(o, default_uniform(W, H, 0), make_ext(*cfg, frame=3), x0, y0, w, h)
    assert rays > 0
    assert not flags & (FP_DENORMAL_OPERAND | FP_UNDERFLOW), hex(flags)
    assert np.array_equal(ieee.view(np.uint32), ftz.view(np.uint32))


def test_ftz_mode_flushes_denormals():
    """The FTZ|DAZ switch takes effect: a path whose direction has a denormal
    component traces differently in the two modes, and the IEEE run raises
    the denormal-operand flag."""
    from mirror_maze import Scene
    from oracle.oracle import FP_DENORMAL_OPERAND, Oracle, fp_flags, set_fp_mode

    o = Oracle.from_scene(Scene.build(10, 0))
    tiny = np.float32(1e-40)  # denormal
    fp_flags(reset=True)
    a = o.trace_path(np.float32([0.0, 0.0, -45.0]), np.float32([tiny, 0.0, 1.0]), 1234)
    assert fp_flags(reset=True) & FP_DENORMAL_OPERAND
    set_fp_mode(True)
    try:
        b = o.trace_path(np.float32([0.0, 0.0, -45.0]), np.float32([tiny, 0.0, 1.0]), 1234)
        assert not fp_flags(reset=True) & FP_DENORMAL_OPERAND  # DAZ: read as zero, no flag
    finally:
        set_fp_mode(False)
    assert a is not None and b is not None


def test_committed_census_is_clean():
    rec = json.loads((REPO / "profiles" / "r03" / "denormal_census.json").read_text())
    assert rec["rays"] > 5e8 and rec["workloads"] >= 20
    assert not rec["any_denormal_operand"] and not rec["any_underflow"] and rec["all_ftz_identical"]
