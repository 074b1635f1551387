"""Parity on scenes that are not mazes: random soups of axis-aligned rects
(with the reference's own SAH BVH over them, Scene.bvh).  They exercise what
the maze does not: thousands of distinct bound values (BVH nodes too large
for LDS: the BVH forms read them through L1/L2), grid lists of
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
# method is unavailable (form 7 needs a compact record for every rect -- the fine
# scene's rects have normals that are not exactly +-1, SLOW records -- and the
# nodes + records in LDS: the BVH's 192 KB of nodes exceed the LDS budget, so
# loop form 5 reads them through L1/L2, mode 0).
CASES = {
    "auto-grid": ({}, {False: (11, (11, 12)), True: (11, (11, 12))}),
    "bvh-lean": ({7: 7}, {False: None, True: None}),
    "bvh-li": ({7: 5}, {False: (5, (0,)), True: (5, (0,))}),
    "grid-global": ({7: 11, 1: 0}, {False: (11, (13,)), True: (11, (13,))}),
}


@pytest.mark.parametrize("lattice", [False, True], ids=["fine", "lattice"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_random_scene_windows_bit_exact(gpu, lattice, case):
    from mirror_maze import (MM_INFO_GRID_OK, MM_INFO_LAST_FORM, MM_INFO_LAST_LDS_MODE, MM_INFO_LEAN, MMError,
                             Renderer, default_uniform, make_ext)
    from oracle.oracle import Oracle

    opts, expect = CASES[case]
    expect = expect[lattice]
    s = random_scene(3000, 11 if lattice else 7, lattice)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 1.0
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


def test_grid_images_fit_the_static_lds_array(gpu):
    """LDS placements 11 / 14 stage the grid image into a static
    array (MM_INFO_GRID_LDS_CAP bytes, a little under 80 KB); the grid builder
    now takes that capacity as its budget, so no image between it and 80 KB
    can be built and then refused at launch.  Mazes and random soups over a
    sweep of cell sizes give many image sizes near the budget: every one is
    within the capacity wherever a whole-image placement runs, and every
    upload traces (whole-frame sample windows, bit-exact vs the oracle for a
    few)."""
    from mirror_maze import (MM_INFO_GRID_BYTES, MM_INFO_GRID_FACES, MM_INFO_GRID_LDS_CAP, MM_INFO_GRID_OK,
                             MM_INFO_LAST_LDS_MODE, Renderer, Scene, default_uniform, make_ext)
    from oracle.oracle import Oracle

    u = default_uniform(1920, 1080, 0)
    e = make_ext(4, 6, 6, frame=1)
    checked = 0
    sizes = []
    scenes = [("maze24", Scene.build(24, 0)), ("maze40", Scene.build(40, 0)),
              ("soup", random_scene(1500, 3, False))]
    for name, s in scenes:
        o = None
        for cell in range(40, 241, 25):
            r = Renderer(0)
            r.set_option(25, cell)
            r.upload_scene(s)
            if r.scene_info(MM_INFO_GRID_OK) != 1.0:
                r.close()
                continue
            cap = r.scene_info(MM_INFO_GRID_LDS_CAP)
            assert 79 * 1024 < cap < 80 * 1024
            nbytes = r.scene_info(MM_INFO_GRID_BYTES)
            if r.scene_info(MM_INFO_GRID_FACES):
                assert nbytes <= cap, (name, cell, nbytes, cap)
            got, _ = r.trace_tile(u, e, 944, 532, 32, 16)
            mode = r.scene_info(MM_INFO_LAST_LDS_MODE)
            if mode in (11, 14):
                assert nbytes <= cap or mode == 14, (name, cell, nbytes, mode)
            sizes.append((name, cell, int(nbytes), int(mode)))
            if checked < 4:
                o = o or Oracle.from_scene(s)
                ref, _ = o.trace_tile(u, e, 944, 532, 32, 16)
                assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (name, cell)
                checked += 1
            r.close()
    assert len(sizes) >= 12, sizes
