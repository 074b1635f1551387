"""The CPU oracle against reference-derived fixtures and independent numpy
restatements of its pieces (CPU only)."""
from __future__ import annotations

import ctypes as C
import json

import numpy as np
import pytest

from conftest import GOLDEN

f32 = np.float32


def _ol():
    from oracle.oracle import lib

    return lib()


def test_noise_texel_fixture_pins_seed_constant():
    """compute_shader samples texel (0,0) for every thread; the oracle's seed
    uses 128/255 for noise.x and noise.y (src/shaders.metal:291, 298)."""
    g = json.loads((GOLDEN / "noise_texel.json").read_text())
    r, gch, _, _ = g["texel_0_0_rgba8"]
    n_x, n_y = f32(r) / f32(255), f32(gch) / f32(255)
    L = _ol()
    for tx, ty, t in [(0, 0, 0), (31, 7, 0), (1023, 767, 5), (512, 100, 60), (77, 3, 1)]:
        s = n_y + f32(np.uint32(tx * 15823 & 0xFFFFFFFF))
        s = s + n_x
        s = s + f32(np.uint32(ty * 9737333 & 0xFFFFFFFF))
        s = s + f32(t)
        want = 0xFFFFFFFF if s >= f32(4294967296.0) else int(s)
        assert L.oracle_seed_reference(tx, ty, t) == want


def _pcg_pm1(state):
    s = (state * 747796405 + 291336453) & 0xFFFFFFFF
    r = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & 0xFFFFFFFF
    r = (r >> 22) ^ r
    return s, f32(r) * f32(2.0**-31) - f32(1.0)


def test_random_matches_numpy_restatement():
    L = _ol()
    st = C.c_uint32(12345)
    py = 12345
    for _ in range(1000):
        a = L.oracle_rand_pm1(C.byref(st))
        py, b = _pcg_pm1(py)
        assert st.value == py and np.float32(a) == b
        assert -1.0 <= a <= 1.0


def test_intersect_aabb_matches_numpy_slab():
    L = _ol()
    rng = np.random.default_rng(1)
    for _ in range(2000):
        o = rng.uniform(-60, 60, 3).astype(f32)
        d = rng.normal(size=3).astype(f32)
        if rng.random() < 0.1:
            d[rng.integers(3)] = 0.0
        mn = rng.uniform(-60, 60, 3).astype(f32)
        mx = (mn + rng.uniform(0, 30, 3)).astype(f32)
        t = f32(rng.choice([1e30, rng.uniform(0, 100)]))
        with np.errstate(divide="ignore", invalid="ignore"):
            t1 = (mn - o) / d
            t2 = (mx - o) / d
        tmin = np.fmin(t1[0], t2[0]); tmax = np.fmax(t1[0], t2[0])
        tmin = np.fmax(tmin, np.fmin(t1[1], t2[1])); tmax = np.fmin(tmax, np.fmax(t1[1], t2[1]))
        tmin = np.fmax(tmin, np.fmin(t1[2], t2[2])); tmax = np.fmin(tmax, np.fmax(t1[2], t2[2]))
        want = tmin if (tmax >= tmin and tmin < t and tmax > 0) else f32(1e30)
        got = L.oracle_intersect_aabb(o.ctypes.data, d.ctypes.data, t, mn.ctypes.data, mx.ctypes.data)
        assert np.float32(got) == want


def test_primary_ray_centre_pixel():
    """Centre pixel of the reference view points along the camera quaternion."""
    from mirror_maze import default_uniform

    L = _ol()
    u = default_uniform(1024, 768, 0)
    ub = C.create_string_buffer(bytes(u), 56)
    d = np.zeros(3, f32)
    L.oracle_primary_dir(ub, 512, 384, d.ctypes.data)
    # rotation of (0,0,1) by the (0.1,0,1)-direction quaternion, unit length
    assert abs(float(np.linalg.norm(d)) - 1.0) < 1e-6
    expect = np.array([0.1, 0.0, 1.0]) / np.linalg.norm([0.1, 0.0, 1.0])
    assert np.allclose(np.abs(d), np.abs(expect), atol=1e-6)


def test_oracle_p0_regression_fixture():
    """Oracle outputs frozen at fixture time (regression, not a pin)."""
    from mirror_maze import Scene, default_uniform
    from oracle.oracle import Oracle

    g = np.load(GOLDEN / "oracle_p0.npz")
    o = Oracle.from_scene(Scene.build(10, 0))
    for t in (0, 1):
        fb = np.zeros((768, 1024, 4), f32)
        for gx in range(0, 32, 5):
            o.trace_group(default_uniform(1024, 768, t), g["chunks"], gx, 0, fb)
        m = fb[g["ys"], g["xs"], 3] == 1.0
        got = fb[g["ys"], g["xs"], :3][m]
        assert m.sum() == 16 * 7
        assert np.array_equal(got.view(np.uint32), g[f"rgb_t{t}"][m].view(np.uint32))


def test_oracle_c1_regression_fixture():
    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    g = np.load(GOLDEN / "oracle_c1.npz")
    o = Oracle.from_scene(Scene.build(16, 0))
    img, st = o.trace_tile(default_uniform(256, 256, 0), make_ext(1, 1, 15), 0, 0, 256, 256)
    assert np.array_equal(img[..., :3].view(np.uint32), g["rgb"].view(np.uint32))
    assert st.rays == int(g["rays"]) == 256 * 256
    assert np.all(img[..., 3] == 1.0)


def test_reduction_order_is_reference_tree():
    """Throughput-mode spp=8 reduction equals ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7))
    computed from single-sample tiles of the same seeds."""
    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    o = Oracle.from_scene(Scene.build(10, 0))
    u = default_uniform(64, 48, 0)
    img8, _ = o.trace_tile(u, make_ext(8, 3, 15), 10, 10, 4, 2)
    # per-sample values through trace_path with the tile seeds
    L = _ol()
    for j in range(2):
        for i in range(4):
            px, py = 10 + i, 10 + j
            s = []
            for k in range(8):
                seed = C.c_uint32(L.oracle_tile_seed(py * 64 + px, k, 0))
                d = np.zeros(3, f32)
                L.oracle_primary_dir(C.create_string_buffer(bytes(u), 56), px, py, d.ctypes.data)
                j1 = L.oracle_rand_pm1(C.byref(seed)); j2 = L.oracle_rand_pm1(C.byref(seed))
                dj = np.array([d[0] + f32(j1) * f32(0.001), d[1] + f32(j2) * f32(0.001), d[2] + f32(0.0)], f32)
                rgb, _, rc = o.trace_path(np.array(u.cam.center, f32), dj, seed.value, 3, 15)
                assert rc == 0
                s.append(rgb.astype(f32))
            acc = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]))
            assert np.array_equal((acc / f32(8)).view(np.uint32), img8[j, i, :3].view(np.uint32))


def test_same_algorithm_cpu_baseline_equals_the_oracle():
    """oracle/grid_cpu.c (bench.py's same-algorithm CPU baseline: the oracle's
    path loop with the product's certified grid search as the query) returns
    the reference walk's answers: bit-identical rows and the same ray counts
    on the C2 / C3 / C5-scene mazes and the parity-mode dispatch of the
    reference scene."""
    import sys

    sys.path.insert(0, str(GOLDEN.parent.parent / "mirror-maze_amd"))
    from mirror_maze import ChunkScheduler, Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    for n, (spp, b, m) in [(16, (1, 4, 15)), (32, (8, 8, 8)), (64, (2, 16, 16))]:
        s = Scene.build(n, 0)
        u = default_uniform(1920, 1080, 0)
        e = make_ext(spp, b, m, frame=3)
        walk, sw = Oracle.from_scene(s).trace_tile(u, e, 0, 530, 1920, 1)
        grid, sg = Oracle.from_scene(s, method="grid").trace_tile(u, e, 0, 530, 1920, 1)
        assert np.array_equal(walk.view(np.uint32), grid.view(np.uint32)), n
        assert sw.rays == sg.rays
    s = Scene.build(10, 0)
    u = default_uniform(1024, 768, 1)
    chunks = ChunkScheduler(1024, 768, 4, seed=3).next(768)
    ow, og = Oracle.from_scene(s), Oracle.from_scene(s, method="grid")
    fw, fg = np.zeros((768, 1024, 4), np.float32), np.zeros((768, 1024, 4), np.float32)
    for gx, gy in [(0, 0), (5, 3), (31, 23), (17, 11)]:  # threadgroups of the reference dispatch
        ow.trace_group(u, chunks, gx, gy, fw)
        og.trace_group(u, chunks, gx, gy, fg)
    assert fw[..., 3].sum() == 4 * 16
    assert np.array_equal(fw.view(np.uint32), fg.view(np.uint32))


def test_grid_baseline_refuses_another_scenes_grid():
    """grid_cpu keeps one grid per process.  A second grid Oracle
    rebuilds it for its scene; the first then refuses to trace (its queries
    would otherwise walk the BVH under the same-algorithm label), and the
    query counts separate grid answers from walk fallbacks."""
    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    a = Oracle.from_scene(Scene.build(8, 0), method="grid")
    u, e = default_uniform(64, 48, 0), make_ext(1, 2, 2)
    a.trace_tile(u, e, 0, 0, 64, 48)
    st = Oracle.grid_stats()
    assert st["grid"] > 0 and st["other_scene"] == 0
    b = Oracle.from_scene(Scene.build(9, 0), method="grid")
    with pytest.raises(RuntimeError, match="another scene"):
        a.trace_tile(u, e, 0, 0, 64, 48)
    b.trace_tile(u, e, 0, 0, 64, 48)
    assert Oracle.grid_stats()["other_scene"] == 0


def test_grid_baseline_counts_every_query_across_threads():
    """The same-algorithm baseline's query counters are per thread (one shared
    atomic made the 16-thread baseline 12x slower in round 5): traced from
    four threads at once, the grid answers plus walk fallbacks still equal the
    rays the rows report, and a reset zeroes every thread's slot."""
    import threading

    from mirror_maze import Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    o = Oracle.from_scene(Scene.build(16, 0), method="grid")
    u, e = default_uniform(256, 64, 0), make_ext(2, 4, 4, frame=1)
    Oracle.grid_stats(reset=True)
    rays = [0] * 4

    def work(i):
        for y in range(i, 64, 4):
            _, st = o.trace_tile(u, e, 0, y, 256, 1)
            rays[i] += st.rays

    ths = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    st = Oracle.grid_stats(reset=True)
    assert st["other_scene"] == 0
    assert st["grid"] + st["fallback"] == sum(rays) > 0
    assert Oracle.grid_stats() == {"grid": 0, "fallback": 0, "other_scene": 0}
