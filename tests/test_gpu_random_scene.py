"""Parity on scenes that are not mazes: random soups of axis-aligned rects
(with the reference's own SAH BVH over them, Scene.bvh).  They exercise what
the maze does not: thousands of distinct bound values (no dictionary nodes:
the BVH forms fall back to the top-of-tree cache), grid lists of
arbitrary rects, and -- in the lattice scene -- many coplanar overlapping
rects, whose equal hit distances are ties the certified grid search must
hand to the reference walk.  Bit-exact vs the oracle."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def random_scene(n, seed, lattice):
    """n axis-aligned rects around the default camera; coordinates on a grid of
    1/64 (lattice=False) or of 8 (lattice=True: coplanar overlaps everywhere)."""
    from mirror_maze import Scene

    rng = np.random.default_rng(seed)
    q = 8.0 if lattice else 1.0 / 64
    rects = np.zeros((n, 12), np.float32)
    for i in range(n):
        k = int(rng.integers(3))
        iv, iu = [a for a in range(3) if a != k][:: 1 if rng.random() < 0.5 else -1]
        rects[i, 0:3] = np.round(rng.uniform(-200, 200, 3) / q) * q
        rects[i, 3 + iv] = max(q, np.round(rng.uniform(2, 40) / q) * q) * rng.choice([-1, 1])
        rects[i, 6 + iu] = max(q, np.round(rng.uniform(2, 40) / q) * q) * rng.choice([-1, 1])
        if i % 97 == 0:
            rects[i, 3:6] = 0.0  # zero-length: never hit (shaders.metal:63)
        rects[i, 9:12] = rng.uniform(0.2, 0.9, 3)
    is_mirror = (rng.random(n) < 0.15).astype(np.uint8)
    emission = np.tile(np.float32([1, 0, 0, 0]), (n, 1))
    lights = rng.random(n) < 0.1
    emission[lights] = np.float32([1.0, 0.8, 0.3, 2.0])
    nodes, idx = Scene.bvh(rects)
    return Scene(0, rects, nodes, idx, is_mirror, emission, np.zeros((0, 0), np.uint8), 0)


# per scene: options -> (query method run, LDS modes it may use) or None when the
# method is unavailable (form 7 needs a compact record for every rect: the fine
# scene's rects have normals that are not exactly +-1, SLOW records).  The
# BVH's 192 KB of nodes exceed the LDS budget: the A/B build places them as
# dictionary nodes (mode 10) or the top-of-tree cache (6); the default build
# reads them through L1/L2 (mode 0, form 5; form 7 needs nodes + records in LDS).
CASES = {
    "auto-grid": ({}, {False: (11, (11, 12)), True: (11, (11, 12))}),
    "bvh-lean": ({7: 7}, {False: None, True: (7, (10,))}),
    "bvh-li": ({7: 5}, {False: (5, (6,)), True: (5, (10,))}),
    "bvh-li-nodict": ({7: 5, 20: 0, 9: 0}, {False: (5, (0,)), True: (5, (0,))}),
    "grid-global": ({7: 11, 1: 0}, {False: (11, (13,)), True: (11, (13,))}),
}
CASES_DEFAULT_BUILD = {
    "bvh-lean": {False: None, True: None},
    "bvh-li": {False: (5, (0,)), True: (5, (0,))},
}


@pytest.mark.parametrize("lattice", [False, True], ids=["fine", "lattice"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_random_scene_windows_bit_exact(gpu, lattice, case):
    from mirror_maze import (MM_INFO_DICT_OK, MM_INFO_GRID_OK, MM_INFO_LAST_FORM, MM_INFO_LAST_LDS_MODE,
                             MM_INFO_LEAN, MMError, Renderer, default_uniform, make_ext)
    from oracle.oracle import Oracle

    from mirror_maze import ab_variants

    opts, expect = CASES[case]
    if not ab_variants():
        expect = CASES_DEFAULT_BUILD.get(case, expect)
    expect = expect[lattice]
    s = random_scene(3000, 11 if lattice else 7, lattice)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 1.0
    # (MM_OPT_DICT_NODES 0 at upload: the dictionary is not built)
    assert r.scene_info(MM_INFO_DICT_OK) == (1.0 if lattice and opts.get(20, 1) != 0 else 0.0)
    assert r.scene_info(MM_INFO_LEAN) == (1.0 if lattice else 0.0)
    u = default_uniform(1920, 1080, 0)
    e = make_ext(8, 8, 8, frame=3)
    if expect is None:
        with pytest.raises(MMError):
            r.trace_tile(u, e, 0, 0, 32, 16)
        r.close()
        return
    for (x0, y0) in [(0, 0), (944, 532), (1888, 1064), (300, 800), (1500, 200)]:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, 32, 16)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        assert (st.rays, st.paths) == (rst.rays, rst.paths)
    assert r.scene_info(MM_INFO_LAST_FORM) == expect[0]
    assert r.scene_info(MM_INFO_LAST_LDS_MODE) in expect[1]
    r.close()


def test_scene_reaching_2_60_takes_the_bvh_bit_exact(gpu):
    """A rect corner at x = 2^60: the scene is inside the exact-division
    guards (every coordinate <= 2^60), but its grid box (widened by eps) would
    pass 2^60, which the per-query guard's integer form takes from the box
    (mm_trace.h ray_fast_ok_boxed) -- grid_build.cpp builds no grid, the
    queries walk the BVH, and the frames stay bit-exact."""
    from mirror_maze import MM_INFO_GRID_OK, Renderer, Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = random_scene(300, 5, False)
    rects = s.rects.copy()
    rects[0, 0:9] = np.float32([2.0**60 - 2.0**58, -8.0, 0.0, 2.0**58, 0.0, 0.0, 0.0, 16.0, 0.0])
    nodes, idx = Scene.bvh(rects)
    s = Scene(0, rects, nodes, idx, s.is_mirror, s.emission, np.zeros((0, 0), np.uint8), 0)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 0.0
    u = default_uniform(1920, 1080, 0)
    e = make_ext(8, 8, 8, frame=3)
    for (x0, y0) in [(0, 0), (944, 532), (1500, 200)]:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, 32, 16)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        assert (st.rays, st.paths) == (rst.rays, rst.paths)
    r.close()
