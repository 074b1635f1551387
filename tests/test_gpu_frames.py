"""Whole-frame parity on the paths bench.py times: the HIP output of entire
C2 / C3 frames, of rank 0's row set of an 8-way C4 split, and of C5 windows at
64 spp (single frames and 3-frame temporal accumulation) against the CPU
oracle, bit for bit.  The oracle runs over a thread pool on the host's CPUs
(conftest.oracle_tile).  Reference: src/shaders.metal:245-368 (the kernel),
342-364 (the 64-sample reduction), src/main.rs:778-784 (temporal refresh)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import oracle_tile

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _scene(n):
    from mirror_maze import Scene

    return Scene.build(n, 0)


def _diff(got, ref):
    bad = (_bits(got) != _bits(ref)).any(axis=-1)
    return int(bad.sum())


@pytest.mark.parametrize("opts", [{21: 32, 22: 1 << 24}, {21: 0}], ids=["tail-deferral", "no-tail-deferral"])
def test_c3_bench_path_two_whole_frames(gpu, opts):
    """C3 as bench.py renders it: MM_PIPE_AUTO (the grid search), consecutive
    frames in ONE mm_trace_tile_frames launch, every pixel of both 1920x1080
    frames (2 x 137 M closest-hit queries) vs the oracle -- with mirror-tail
    deferral through the block-local tail rings (32 lanes, past
    MM_OPT_DEFER_MIN = 2^24 paths) and without it."""
    from mirror_maze import MM_PIPE_AUTO, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(32)
    r = Renderer(0)
    r.set_pipeline(MM_PIPE_AUTO)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    u = default_uniform(1920, 1080, 0)
    e = make_ext(8, 8, 8, frame=0)
    got, st = r.trace_tile_frames(u, e, 2, 0, 0, 1920, 1080, stats=True)
    got = got.cpu().numpy()
    o = Oracle.from_scene(s)
    rays = 0
    for f in range(2):
        ref, n = oracle_tile(o, u, make_ext(8, 8, 8, frame=f), 0, 0, 1920, 1080)
        rays += n
        assert _diff(got[f], ref) == 0, f"frame {f}: {_diff(got[f], ref)} pixels differ"
    assert st.rays == rays
    r.close()


def test_c2_whole_frame(gpu):
    """C2: 16x16 maze, 1920x1080, 1 spp, 4/15 bounces, the whole frame."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(16)
    r = Renderer(0)
    r.upload_scene(s)
    u = default_uniform(1920, 1080, 0)
    e = make_ext(1, 4, 15, frame=0)
    got, st = r.trace_tile(u, e, 0, 0, 1920, 1080, stats=True)
    ref, rays = oracle_tile(Oracle.from_scene(s), u, e, 0, 0, 1920, 1080)
    assert _diff(got.cpu().numpy(), ref) == 0
    assert st.rays == rays
    r.close()


def test_c4_rank0_of_eight_way_split(gpu):
    """C4 (32x32 maze, 3840x2160, 16 spp, 8/15 bounces): rank 0's rows of the
    8-way interleaved split (mirror_maze.dist.row_shard), as an 8-GPU run
    renders them, vs the oracle on the same rows."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from mirror_maze.dist import row_shard
    from oracle.oracle import Oracle

    s = _scene(32)
    r = Renderer(0)
    r.upload_scene(s)
    W, H = 3840, 2160
    y0, stride, rows = row_shard(H, 8, 0)
    u = default_uniform(W, H, 0)
    e = make_ext(16, 8, 15, frame=0)
    got, st = r.trace_tile(u, e, 0, y0, W, rows, y_stride=stride, stats=True)
    ref, rays = oracle_tile(Oracle.from_scene(s), u, e, 0, y0, W, rows, y_stride=stride)
    assert _diff(got.cpu().numpy(), ref) == 0
    assert st.rays == rays
    r.close()


C5_WINDOWS = [(0, 0), (1904, 1064), (3808, 2144), (700, 1500), (2900, 300), (1200, 40)]


@pytest.mark.parametrize("opts", [{}, {21: 32, 22: 0}, {7: 5}], ids=["auto", "tail-deferral", "bvh-walk"])
def test_c5_windows_64spp(gpu, opts):
    """C5: 64x64 maze, 3840x2160 frame coordinates, 64 spp, 16/16 bounces --
    the reference's 64-sample reduction (shaders.metal:342-364) as the fused
    resolve, one pixel per wave -- on six 32x16 windows.  "bvh-walk": loop
    form 5 over nodes read through L1/L2 (form 7 needs the N=64 tree in LDS)."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(64)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    u = default_uniform(3840, 2160, 0)
    e = make_ext(64, 16, 16, frame=7)
    for (x0, y0) in C5_WINDOWS:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rays = oracle_tile(o, u, e, x0, y0, 32, 16)
        assert _diff(got.cpu().numpy(), ref) == 0, (x0, y0)
        assert st.rays == rays
    r.close()


def test_c5_temporal_accumulation_three_frames(gpu):
    """C5's temporal accumulation (MM_EXT_ACCUMULATE: every frame adds its
    per-pixel 64-spp mean into one running sum, alpha counts frames) over
    frames 0, 1, 2 on two windows and a row band, vs the oracle's accumulate."""
    from mirror_maze import MM_EXT_ACCUMULATE, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(64)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    r.upload_scene(s)
    u = default_uniform(3840, 2160, 0)
    for (x0, y0, w, h) in [(1904, 1064, 32, 16), (100, 1800, 32, 16), (0, 1080, 1024, 2)]:
        import torch

        acc = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        ref = np.zeros((h, w, 4), dtype=np.float32)
        for f in range(3):
            e = make_ext(64, 16, 16, frame=f, flags=MM_EXT_ACCUMULATE)
            r.trace_tile(u, e, x0, y0, w, h, out=acc)
            o.trace_tile(u, e, x0, y0, w, h, out=ref)
        got = acc.cpu().numpy()
        assert np.all(got[..., 3] == 3.0)
        assert _diff(got, ref) == 0, (x0, y0)
    r.close()


def test_c5_temporal_accumulation_120_frames(gpu):
    """C5 exactly as BASELINE.json states it (configs[4]): the 64x64 maze at
    3840x2160 frame coordinates, 64 spp, 16/16 bounces, temporal accumulation
    (MM_EXT_ACCUMULATE) over 120 frames, on two 32x16 windows -- the running
    sum after frame 120 vs the oracle's accumulate, 0 ulp (reference temporal
    path: src/main.rs:778-784 with src/shaders.metal:342-366)."""
    import torch

    from mirror_maze import MM_EXT_ACCUMULATE, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(64)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    r.upload_scene(s)
    u = default_uniform(3840, 2160, 0)
    frames = 120
    for (x0, y0) in [(1904, 1064), (2900, 300)]:
        acc = torch.zeros((16, 32, 4), dtype=torch.float32, device="cuda")
        ref = np.zeros((16, 32, 4), dtype=np.float32)
        rays = 0
        for f in range(frames):
            e = make_ext(64, 16, 16, frame=f, flags=MM_EXT_ACCUMULATE)
            r.trace_tile(u, e, x0, y0, 32, 16, out=acc)
            rays += oracle_tile(o, u, e, x0, y0, 32, 16, out=ref)[1]
        r.sync()
        got = acc.cpu().numpy()
        assert np.all(got[..., 3] == float(frames))
        assert rays >= frames * 32 * 16 * 64  # at least one closest-hit query per path
        assert _diff(got, ref) == 0, (x0, y0)
    r.close()


@pytest.mark.parametrize("cell,direction", [((3, 4), (1.0, 0.05, 0.2)), ((16, 16), (-0.3, -0.1, 1.0)),
                                            ((30, 2), (0.7, 0.3, -0.6)), ((0, 31), (0.0, -0.2, -1.0))],
                         ids=["corridor", "centre", "corner-up", "edge-down"])
def test_cameras_inside_the_maze(gpu, cell, direction):
    """C3's scene and limits with the camera inside the maze (cell centres,
    assorted view directions, quaternion by calculate_quaternion,
    src/maths.rs:139-156): whole 320x180 frames at 8 spp vs the oracle.  The
    bench camera looks along the outer wall; these rays start in corridors,
    exercise every face range of the grid and the mirrors at close range."""
    from mirror_maze import MM_PIPE_AUTO, Renderer, calculate_quaternion, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(32)
    base = -10.0 * (32 / 2)
    u = default_uniform(320, 180, 0)
    u.cam.center[0] = base + 10.0 * cell[0] + 5.0
    u.cam.center[1] = 0.0
    u.cam.center[2] = base + 10.0 * cell[1] + 5.0
    q = calculate_quaternion(np.asarray(direction, dtype=np.float32))
    for i in range(4):
        u.cam.quat[i] = float(q[i])
    e = make_ext(8, 8, 8, frame=3)
    ref, n = oracle_tile(Oracle.from_scene(s), u, e, 0, 0, 320, 180)
    assert n > 4 * 320 * 180 * 8 and ref[..., :3].mean() > 0.01  # the paths bounce inside the maze
    for opts in ({}, {21: 32, 22: 0}):  # fused resolve; tail deferral with staged samples
        r = Renderer(0)
        r.set_pipeline(MM_PIPE_AUTO)
        for k, v in opts.items():
            r.set_option(k, v)
        r.upload_scene(s)
        got, st = r.trace_tile(u, e, 0, 0, 320, 180, stats=True)
        assert _diff(got.cpu().numpy(), ref) == 0, opts
        assert st.rays == n
        r.close()


@pytest.mark.parametrize("maze_n,bl,ml", [(32, 8, 8), (64, 16, 16), (16, 4, 15)], ids=["c3-scene", "c5-scene", "c2-scene"])
def test_camera_sweep(gpu, maze_n, bl, ml):
    """12 seeded random cameras inside each maze (random cell, random view
    direction, random frame index), 240x135 at 8 spp with the config's bounce
    limits, every pixel vs the oracle.  The N=64 maze runs the plain 32-bit
    grid cells with records in global memory, the others the per-face ranges
    with the whole image in LDS."""
    from mirror_maze import MM_PIPE_AUTO, Renderer, calculate_quaternion, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(maze_n)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    r.set_pipeline(MM_PIPE_AUTO)
    r.upload_scene(s)
    rng = np.random.default_rng(maze_n)
    base = -10.0 * (maze_n / 2)
    for _ in range(12):
        u = default_uniform(240, 135, 0)
        cx, cz = rng.integers(0, maze_n, size=2)
        u.cam.center[0] = base + 10.0 * cx + 5.0 + rng.uniform(-3, 3)
        u.cam.center[1] = rng.uniform(-6.0, 1.5)
        u.cam.center[2] = base + 10.0 * cz + 5.0 + rng.uniform(-3, 3)
        d = rng.normal(size=3).astype(np.float32)
        q = calculate_quaternion(d)
        for i in range(4):
            u.cam.quat[i] = float(q[i])
        e = make_ext(8, bl, ml, frame=int(rng.integers(0, 1000)))
        got, st = r.trace_tile(u, e, 0, 0, 240, 135, stats=True)
        ref, n = oracle_tile(o, u, e, 0, 0, 240, 135)
        assert _diff(got.cpu().numpy(), ref) == 0, (cx, cz, d)
        assert st.rays == n
    r.close()


@pytest.mark.parametrize("spp", [16, 24, 40])
def test_staged_resolve_spp_multiples_of_eight(gpu, spp):
    """k_resolve8 (one thread per pixel for spp % 8 == 0): 16 (a power of two:
    the mean as an exact multiply), 24 and 40 (the IEEE division; 64 % spp !=
    0, so no fused resolve either) through forced deferral, every pixel vs the
    oracle."""
    from mirror_maze import MM_PIPE_AUTO, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(16)
    u = default_uniform(96, 54, 0)
    e = make_ext(spp, 8, 8, frame=5)
    ref, n = oracle_tile(Oracle.from_scene(s), u, e, 0, 0, 96, 54)
    r = Renderer(0)
    r.set_pipeline(MM_PIPE_AUTO)
    r.set_option(21, 32)
    r.set_option(22, 0)
    r.upload_scene(s)
    got, st = r.trace_tile(u, e, 0, 0, 96, 54, stats=True)
    assert _diff(got.cpu().numpy(), ref) == 0
    assert st.rays == n
    r.close()


@pytest.mark.parametrize("bl,ml", [(40, 40), (3, 200)], ids=["long-paths", "mirror-chains"])
def test_long_paths_through_the_tail_rings(gpu, bl, ml):
    """Paths parked in the tail rings and resumed carry their state in a 64-B
    record: (n - mh) | mh << 15 | bank << 30 and the first banked trial's end
    s1 (trace_kernels.hip tail_store).  Long paths (40 / 40 bounces) and long
    mirror chains (mirror limit 200, so mh runs past what 8 bits hold) through
    forced deferral, every pixel vs the oracle; the same frame with deferral
    off too."""
    from mirror_maze import MM_PIPE_AUTO, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(16)
    u = default_uniform(160, 90, 0)
    e = make_ext(8, bl, ml, frame=11)
    ref, n = oracle_tile(Oracle.from_scene(s), u, e, 0, 0, 160, 90)
    for opts in ({21: 32, 22: 0}, {21: 0}):
        r = Renderer(0)
        r.set_pipeline(MM_PIPE_AUTO)
        for k, v in opts.items():
            r.set_option(k, v)
        r.upload_scene(s)
        got, st = r.trace_tile(u, e, 0, 0, 160, 90, stats=True)
        assert _diff(got.cpu().numpy(), ref) == 0, opts
        assert st.rays == n
        r.close()


@pytest.mark.parametrize("case", ["c3-two-frames-rings", "c3-two-frames-fused", "c2-frame", "spp3-strided"])
def test_rgba8_frames_equal_the_quantized_float_frames(gpu, case):
    """MM_EXT_RGBA8: the trace writes each pixel's texture-write conversion
    itself (the fused resolve in the wave, the staged resolve after the tail
    rings, and the per-pixel resolve for spp that does not divide 64); every
    byte equals mm_quantize_rgba8 of the float frame the same call writes
    without the flag (whose floats the other tests hold to the oracle)."""
    import torch

    from mirror_maze import MM_EXT_ACCUMULATE, MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    n_maze, W, H, spp, bl, ml = {"c3-two-frames-rings": (32, 1920, 1080, 8, 8, 8),
                                 "c3-two-frames-fused": (32, 1920, 1080, 8, 8, 8),
                                 "c2-frame": (16, 1920, 1080, 1, 4, 15),
                                 "spp3-strided": (16, 640, 480, 3, 4, 15)}[case]
    r.upload_scene(_scene(n_maze))
    if case == "c3-two-frames-rings":
        r.set_option(21, 32)
        r.set_option(22, 1 << 24)
    elif case == "c3-two-frames-fused":
        r.set_option(21, 0)
    u, e = default_uniform(W, H, 0), make_ext(spp, bl, ml, frame=7)
    if case.startswith("c3"):
        f32, _ = r.trace_tile_frames(u, e, 2, 0, 0, W, H)
        u8, _ = r.trace_tile_frames(u, e, 2, 0, 0, W, H, rgba8=True)
    elif case == "c2-frame":
        f32, _ = r.trace_tile(u, e, 0, 0, W, H)
        u8, _ = r.trace_tile(u, e, 0, 0, W, H, rgba8=True)
    else:  # every 7th row from row 3, a ragged 61-row tile
        f32, _ = r.trace_tile(u, e, 5, 3, 600, 61, y_stride=7)
        u8 = torch.zeros((61, 600, 4), dtype=torch.uint8, device="cuda")
        r.trace_tile(u, e, 5, 3, 600, 61, y_stride=7, out=u8)
    want = r.quantize(f32)
    torch.cuda.synchronize()
    assert u8.dtype == torch.uint8 and torch.equal(u8, want), case
    with pytest.raises(MMError):
        r.trace_tile(u, make_ext(spp, bl, ml, flags=MM_EXT_ACCUMULATE), 0, 0, 64, 8, rgba8=True)
    r.close()
