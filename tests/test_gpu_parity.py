"""GPU parity: the HIP path (through the C ABI) against the CPU oracle,
bit-exact (tolerance 0 ulp on every float; the north star allows 1e-4)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def ren(gpu):
    from mirror_maze import Renderer

    r = Renderer(0)
    yield r
    r.close()


def _scene(n):
    from mirror_maze import Scene

    return Scene.build(n, 0)


def _quantize(x):
    """RGBA8Unorm store conversion: round-half-even of clamp(x,0,1)*255."""
    return np.rint(np.clip(x, 0, 1).astype(np.float32) * np.float32(255)).astype(np.uint8)


def test_parity_mode_matches_committed_fixture(ren):
    """P0 subset: reference scene, 1024x768, first 32 threadgroups, time 0 and 1."""
    from mirror_maze import default_uniform

    g = np.load(GOLDEN / "oracle_p0.npz")
    s = _scene(10)
    ren.upload_scene(s)
    for t in (0, 1):
        ren.compute_shader(default_uniform(1024, 768, t), g["chunks"])
        f, _ = ren.read_texture()
        assert np.array_equal(_bits(f[g["ys"], g["xs"], :3]), _bits(g[f"rgb_t{t}"]))


@pytest.mark.parametrize("t,seed", [(0, 7), (1, 11), (60, 3)])
def test_parity_mode_full_dispatch_bit_exact(ren, t, seed):
    """One full reference dispatch (768 chunks x 16 px x 64 samples)."""
    from mirror_maze import ChunkScheduler, default_uniform
    from oracle.oracle import Oracle

    s = _scene(10)
    ren.upload_scene(s)
    chunks = ChunkScheduler(1024, 768, 4, seed=seed).next(768)
    u = default_uniform(1024, 768, t)
    ren.compute_shader(u, chunks)
    f, b = ren.read_texture()
    ref, st = Oracle.from_scene(s).trace_chunks(u, chunks)
    w = ref[..., 3] == 1.0
    assert w.sum() == 768 * 16
    diff = _bits(f[w]) != _bits(ref[w])
    assert not diff.any(), f"{diff.any(axis=1).sum()} texels differ"
    assert np.array_equal(b[w][:, :3], _quantize(ref[w][:, :3]))
    assert np.all(b[w][:, 3] == 255)


def test_parity_mode_accumulates_over_frames(ren):
    """The texture is never cleared: 64 dispatches cover every chunk once."""
    from mirror_maze import ChunkScheduler, default_uniform

    s = _scene(10)
    ren.upload_scene(s)
    cs = ChunkScheduler(1024, 768, 4, seed=5)
    for frame in range(64):
        ren.compute_shader(default_uniform(1024, 768, frame), cs.next(768))
    f, _ = ren.read_texture()
    assert np.all(f[..., 3] == 1.0)
    assert np.isfinite(f).all() and f[..., :3].max() > 0.5


def test_c1_full_frame_matches_fixture_and_oracle(ren, gpu):
    """C1: 16x16 maze, 256x256, 1 spp, 1 bounce."""
    from mirror_maze import default_uniform, make_ext

    g = np.load(GOLDEN / "oracle_c1.npz")
    ren.upload_scene(_scene(16))
    img, st = ren.trace_tile(default_uniform(256, 256, 0), make_ext(1, 1, 15), 0, 0, 256, 256, stats=True)
    img = img.cpu().numpy()
    assert np.array_equal(_bits(img[..., :3]), _bits(g["rgb"]))
    assert st.rays == int(g["rays"]) and st.node_visits == int(g["visits"]) and st.rect_tests == int(g["rtests"])


WINDOWS = [(0, 0), (960, 540), (1888, 1064), (300, 700), (1500, 100)]


PIPES = {  # (pipeline, {option: value}); options: 1 lds, 2 block, 3 persist, 4 threshold
    "reference": (3, {}),
    "mega-global": (1, {1: 0, 3: 0}),
    "mega-lds": (1, {1: 1, 3: 0}),
    "mega-lds-b1024": (1, {1: 1, 2: 1024, 3: 0}),
    "persist-lds": (1, {1: 1, 3: 1, 8: 0}),
    "persist-ldsrects": (1, {1: 1, 3: 1, 8: 1}),
    "persist-global-t0": (1, {1: 0, 3: 1, 4: 0}),
    "persist-ldsrects-t63-b512-w6": (1, {1: 1, 3: 1, 4: 63, 2: 512, 5: 6}),
    "persist-lds-t16-b1024-w1": (1, {1: 1, 3: 1, 4: 16, 2: 1024, 5: 1, 8: 0}),
    "wavepersist-lds": (1, {1: 1, 3: 2, 6: 0, 8: 0, 11: 0}),
    "wavepersist-ldsrects": (1, {1: 1, 3: 2, 8: 1}),
    "wavepersist-ldsrects-b512-w6": (1, {1: 1, 3: 2, 8: 1, 2: 512, 5: 6}),
    "wavepersist-ldsstack": (1, {1: 1, 3: 2, 6: 1, 8: 0}),
    "wavepersist-ldsstack-b512-w6": (1, {1: 1, 3: 2, 6: 1, 2: 512, 5: 6}),
    "whilewhile-lds": (1, {1: 1, 3: 2, 7: 1}),
    "leafbatch16-ldsrects": (1, {1: 1, 3: 2, 7: 16, 8: 1}),
    "leafbatch8-global": (1, {1: 0, 3: 2, 7: 8}),
    "whilewhile-global-ldsstack": (1, {1: 0, 3: 2, 7: 1, 6: 1}),
    "wavepersist-lds-b512-w8": (1, {1: 1, 3: 2, 2: 512, 5: 8}),
    "wavepersist-split2kb": (1, {1: 1, 3: 2, 9: 2}),
    "lean-ldsrects": (1, {1: 1, 3: 2, 7: 2, 8: 1}),
    "lean-ldsstack": (1, {1: 1, 3: 2, 7: 2, 6: 1, 8: 0}),
    "lean-global-b512-w6": (1, {1: 0, 3: 2, 7: 2, 2: 512, 5: 6}),
    "lean-split2kb": (1, {1: 1, 3: 2, 7: 2, 9: 2}),
    "regtop-ldsrects": (1, {1: 1, 3: 2, 7: 3, 8: 1}),
    "coldlds": (1, {1: 1, 3: 2, 10: 1}),
    "lds-globalrects": (1, {1: 1, 3: 2, 8: 0, 11: 1}),
    "split2kb-globalrects": (1, {1: 1, 3: 2, 9: 2, 11: 1}),
    "split2kb-generalrects": (1, {1: 1, 3: 2, 9: 2, 11: 0}),
    "bouncerefill-ldsrects": (1, {1: 1, 3: 2, 7: 4, 8: 1}),
    "bouncerefill-global-b512-w6": (1, {1: 0, 3: 2, 7: 4, 2: 512, 5: 6}),
    "bouncerefill-split2kb": (1, {1: 1, 3: 2, 7: 4, 9: 2}),
    "coldlds-b512-w6": (1, {1: 1, 3: 2, 10: 1, 2: 512, 5: 6}),
    "regtop-split2kb-b512-w6": (1, {1: 1, 3: 2, 7: 3, 9: 2, 2: 512, 5: 6}),
    "wavepersist-split20kb-b512-w6": (1, {1: 1, 3: 2, 9: 20, 2: 512, 5: 6}),
    "wavepersist-global-b256": (1, {1: 0, 3: 2, 2: 256}),
    "leafinterior-ldsrects": (1, {1: 1, 3: 2, 7: 5, 8: 1}),
    "ifif-ldsrects": (1, {1: 1, 3: 2, 7: 0, 8: 1}),
    "leafinterior-grab3-fair": (1, {1: 1, 3: 2, 7: 5, 15: 3, 14: 1}),
    "blocksync": (1, {3: 2, 16: 1}),
    "leanli": (1, {3: 2, 7: 7}),
    "leanli-order": (1, {3: 2, 7: 7, 17: 1}),
    "leanli-dict": (1, {3: 2, 7: 7, 20: 2}),
    "leafinterior-dict": (1, {3: 2, 7: 5, 20: 2}),
    "leafinterior-order-grab2": (1, {3: 2, 7: 5, 17: 1, 15: 2}),
    "cons": (1, {3: 2, 7: 9}),
    "cons-split2kb": (1, {3: 2, 7: 9, 9: 2}),
    "cons-globalrects": (1, {3: 2, 7: 9, 8: 0, 11: 1}),
    "leanli-split2kb": (1, {3: 2, 7: 7, 9: 2}),
    "blocksync-nofuse": (1, {3: 2, 16: 1, 12: 0}),
    "leafinterior-lds": (1, {1: 1, 3: 2, 7: 5, 8: 0, 11: 0}),
    "leafinterior-split2kb": (1, {1: 1, 3: 2, 7: 5, 9: 2}),
    "leafinterior-global": (1, {1: 0, 3: 2, 7: 5}),
    "wavepersist-ldsrects-nofuse": (1, {1: 1, 3: 2, 8: 1, 12: 0}),
    "wavefront": (2, {}),
    "wavefront-global": (2, {1: 0}),
}


@pytest.mark.parametrize("pipe", sorted(PIPES))
@pytest.mark.parametrize("cfg", [
    dict(n=16, spp=1, b=4, m=15),   # C2 settings
    dict(n=32, spp=8, b=8, m=8),    # C3 settings (the benchmark)
    dict(n=10, spp=3, b=5, m=15),   # non-multiple-of-8 spp
    dict(n=32, spp=16, b=8, m=15),  # C4 settings
])
def test_tile_windows_bit_exact(gpu, cfg, pipe):
    from mirror_maze import Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(cfg["n"])
    ren = Renderer(0)
    p, opts = PIPES[pipe]
    ren.set_pipeline(p)
    for k, v in opts.items():
        ren.set_option(k, v)
    ren.upload_scene(s)
    o = Oracle.from_scene(s)
    u = default_uniform(1920, 1080, 0)
    e = make_ext(cfg["spp"], cfg["b"], cfg["m"], frame=2)
    for (x0, y0) in WINDOWS:
        w, h = 32, 16
        got, st = ren.trace_tile(u, e, x0, y0, w, h, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, w, h)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        if pipe.startswith("cons"):  # the verified search does its own (larger) amount of work
            assert (st.rays, st.paths) == (rst.rays, rst.paths)
        else:
            assert (st.rays, st.node_visits, st.rect_tests, st.paths) == \
                   (rst.rays, rst.node_visits, rst.rect_tests, rst.paths)
    ren.close()


@pytest.mark.parametrize("pipe", ["wavepersist-ldsrects", "wavepersist-lds", "mega-global", "leafbatch16-ldsrects",
                                  "lean-ldsrects", "bouncerefill-ldsrects", "leafinterior-ldsrects",
                                  "wavepersist-ldsrects-nofuse", "ifif-ldsrects",
                                  "leafinterior-grab3-fair", "blocksync", "leanli", "cons", "leanli-order",
                                  "leafinterior-order-grab2", "leanli-dict", "leafinterior-dict"])
def test_small_full_frames_bit_exact(gpu, pipe):
    """Whole 256x144 frames (8 spp, 8/8 bounces, 3 frames, N=32 maze): ~7 M
    closest-hit queries per pipeline against the oracle, so rare boundary
    cases of the exact-division and threshold tests get exercised."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(32)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    p, opts = PIPES[pipe]
    r.set_pipeline(p)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    u = default_uniform(256, 144, 0)
    for frame in range(3):
        e = make_ext(8, 8, 8, frame=frame)
        got, _ = r.trace_tile(u, e, 0, 0, 256, 144)
        ref, _ = o.trace_tile(u, e, 0, 0, 256, 144)
        bad = (_bits(got.cpu().numpy()) != _bits(ref)).any(axis=-1)
        assert not bad.any(), f"frame {frame}: {int(bad.sum())} pixels differ"
    r.close()


def test_tiling_and_device_count_invariance_full_frame(ren, gpu):
    """C3 at full size: the frame rendered whole equals the frame assembled
    from 4 interleaved row sets (how 4 GPUs would split it), bit for bit,
    and a second render is identical (determinism)."""
    import torch

    from mirror_maze import default_uniform, make_ext

    ren.upload_scene(_scene(32))
    u = default_uniform(1920, 1080, 0)
    e = make_ext(8, 8, 8, frame=0)
    full, st = ren.trace_tile(u, e, 0, 0, 1920, 1080, stats=True)
    again, _ = ren.trace_tile(u, e, 0, 0, 1920, 1080)
    assert torch.equal(full, again)
    parts = [ren.trace_tile(u, e, 0, r, 1920, 270, y_stride=4)[0] for r in range(4)]
    asm = torch.stack(parts, dim=1).reshape(1080, 1920, 4)
    assert torch.equal(full.view(torch.int32), asm.view(torch.int32))
    assert st.paths == 1920 * 1080 * 8
    assert st.rays >= st.paths  # at least one query per path
    img = full.cpu().numpy()
    assert np.isfinite(img).all() and (img[..., :3] >= 0).all() and np.all(img[..., 3] == 1.0)


def test_chunk_order_bit_identical(gpu):
    """MM_OPT_CHUNK_ORDER: chunks handed out longest first (by the previous
    launch's durations) give the same frames and the same work counts as pixel
    order -- C3 over several frames, a row-split tile of another geometry in
    between (the order is keyed on the tile), and an accumulated frame."""
    import torch

    from mirror_maze import MM_EXT_ACCUMULATE, Renderer, default_uniform, make_ext

    s = _scene(32)
    base, lpt = Renderer(0), Renderer(0)
    lpt.set_option(17, 1)
    for r in (base, lpt):
        r.upload_scene(s)
    u = default_uniform(1920, 1080, 0)
    plan = [(0, 0, 1080, 1), (1, 0, 1080, 1), (2, 0, 1080, 1), (3, 1, 540, 2), (4, 1, 540, 2), (5, 0, 1080, 1),
            (6, 0, 1080, 1)]
    for frame, y0, h, stride in plan:
        e = make_ext(8, 8, 8, frame=frame)
        a, sa = base.trace_tile(u, e, 0, y0, 1920, h, y_stride=stride, stats=True)
        b, sb = lpt.trace_tile(u, e, 0, y0, 1920, h, y_stride=stride, stats=True)
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), frame
        assert (sa.rays, sa.node_visits, sa.rect_tests, sa.paths) == (sb.rays, sb.node_visits, sb.rect_tests, sb.paths)
    e = make_ext(8, 8, 8, frame=7, flags=MM_EXT_ACCUMULATE)
    base.trace_tile(u, e, 0, 0, 1920, 1080, out=a)
    lpt.trace_tile(u, e, 0, 0, 1920, 1080, out=b)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    base.close()
    lpt.close()


@pytest.mark.parametrize("opts", [{}, {9: 2}, {7: 5, 15: 2, 17: 1}, {19: 8}])
def test_multi_frame_launch_bit_identical(gpu, opts):
    """mm_trace_tile_frames: F frames in one launch (one work queue) equal the
    F single-frame launches bit for bit, with summed work counts -- C3 whole
    frames and a row-split tile; the split node cache; loop form 5 with
    grab 2 and longest-first order; a grid 8 CUs short (MM_OPT_RESERVE_CUS)."""
    import torch

    from mirror_maze import Renderer, default_uniform, make_ext

    s = _scene(32)
    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    u = default_uniform(1920, 1080, 0)
    # whole frames, a row-split tile, and a ragged 37x13 tile (each frame's last chunk partial)
    for (x0, y0, w, h, stride, F, f0) in [(0, 0, 1920, 1080, 1, 3, 5), (0, 3, 1920, 135, 8, 5, 0),
                                          (101, 200, 37, 13, 3, 4, 9)]:
        many, sm = r.trace_tile_frames(u, make_ext(8, 8, 8, frame=f0), F, x0, y0, w, h, y_stride=stride,
                                       stats=True)
        rays = visits = paths = 0
        for f in range(F):
            one, so = r.trace_tile(u, make_ext(8, 8, 8, frame=f0 + f), x0, y0, w, h, y_stride=stride, stats=True)
            assert torch.equal(one.view(torch.int32), many[f].view(torch.int32)), (y0, f)
            rays += so.rays; visits += so.node_visits; paths += so.paths
        assert (sm.rays, sm.node_visits, sm.paths) == (rays, visits, paths)
    r.close()


def test_multi_frame_launch_errors(gpu):
    from mirror_maze import MM_EXT_ACCUMULATE, MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(10))
    u = default_uniform(64, 64, 0)
    with pytest.raises(MMError):  # frames of one launch cannot accumulate
        r.trace_tile_frames(u, make_ext(8, 3, 15, flags=MM_EXT_ACCUMULATE), 2, 0, 0, 64, 64)
    with pytest.raises(MMError):  # 3 spp: no fused resolve
        r.trace_tile_frames(u, make_ext(3, 3, 15), 2, 0, 0, 64, 64)
    with pytest.raises(MMError):
        r.trace_tile_frames(u, make_ext(8, 3, 15), 0, 0, 0, 64, 64)
    one, _ = r.trace_tile_frames(u, make_ext(8, 3, 15, frame=4), 1, 0, 0, 64, 64)
    ref, _ = r.trace_tile(u, make_ext(8, 3, 15, frame=4), 0, 0, 64, 64)
    assert np.array_equal(_bits(one[0].cpu().numpy()), _bits(ref.cpu().numpy()))
    r.close()


def test_c4_eight_way_row_split_invariance(ren, gpu):
    """C4 (32x32 maze, 3840x2160, 16 spp, 8/15 bounces) — the multi-GPU
    config: the whole frame equals the frame assembled from the 8 interleaved
    row sets the 8 ranks render (mirror_maze.dist), bit for bit, and the
    8-way stats add up to the whole frame's."""
    import torch

    from mirror_maze import default_uniform, make_ext
    from mirror_maze.dist import assemble, row_shard, rows_max

    ren.upload_scene(_scene(32))
    W, H, N = 3840, 2160, 8
    u = default_uniform(W, H, 0)
    e = make_ext(16, 8, 15, frame=3)
    full, st = ren.trace_tile(u, e, 0, 0, W, H, stats=True)
    tiles, rays = [], 0
    for r in range(N):
        y0, stride, rows = row_shard(H, N, r)
        t = torch.zeros((rows_max(H, N), W, 4), dtype=torch.float32, device="cuda")
        _, sr = ren.trace_tile(u, e, 0, y0, W, rows, y_stride=stride, out=t[:rows], stats=True)
        tiles.append(t)
        rays += sr.rays
    asm = assemble(tiles, H)
    assert torch.equal(full.view(torch.int32), asm.view(torch.int32))
    assert rays == st.rays and st.paths == W * H * 16


@pytest.mark.parametrize("fuse", [1, 0])
def test_accumulate_flag(ren, gpu, fuse):
    from mirror_maze import MM_EXT_ACCUMULATE, default_uniform, make_ext

    ren.upload_scene(_scene(10))
    ren.set_option(12, fuse)
    u = default_uniform(128, 96, 0)
    a, _ = ren.trace_tile(u, make_ext(4, 3, 15, frame=0), 0, 0, 128, 96)
    b, _ = ren.trace_tile(u, make_ext(4, 3, 15, frame=1), 0, 0, 128, 96)
    acc, _ = ren.trace_tile(u, make_ext(4, 3, 15, frame=0), 0, 0, 128, 96)
    ren.trace_tile(u, make_ext(4, 3, 15, frame=1, flags=MM_EXT_ACCUMULATE), 0, 0, 128, 96, out=acc)
    assert np.array_equal(_bits((a + b).cpu().numpy()), _bits(acc.cpu().numpy()))


def test_argument_errors(ren, gpu):
    from mirror_maze import MMError, Scene, default_uniform, make_ext
    from mirror_maze.scene import NODE_DTYPE

    ren.upload_scene(_scene(10))
    u = default_uniform(64, 64, 0)
    with pytest.raises(MMError):
        ren.trace_tile(u, make_ext(4, 3, 15), 60, 0, 8, 8)          # outside the frame
    with pytest.raises(MMError):
        ren.compute_shader(default_uniform(1024, 768, 0), np.zeros((10, 2), np.uint32))  # short chunk list
    # a degenerate 60-deep chain BVH exceeds the reference's 50-entry stack
    # chain: interior node 2d -> (leaf 2d+1, next interior 2d+2), depth n-1
    s = _scene(10)
    n = 61
    arr = np.zeros(2 * (n - 1) + 1, dtype=NODE_DTYPE)
    for d in range(n - 1):
        arr[2 * d] = ((-1e3, -1e3, -1e3), (1e3, 1e3, 1e3), 2 * d + 1, 0)
        arr[2 * d + 1] = ((-1e3, -1e3, -1e3), (1e3, 1e3, 1e3), d % s.n_rects, 1)
    arr[2 * (n - 1)] = ((-1e3, -1e3, -1e3), (1e3, 1e3, 1e3), 0, 1)
    bad = Scene(10, s.rects, arr, s.idx, s.is_mirror, s.emission, s.grid, 0)
    with pytest.raises(MMError) as ei:
        ren.upload_scene(bad)
    assert ei.value.code == -5  # MM_ERR_STACK


@pytest.mark.parametrize("opts", [{}, {9: 0}, {9: 8}, {9: 0, 1: 0}, {3: 0}, {11: 0}, {7: 5}, {7: 0}, {7: 7}, {7: 9},
                                  {20: 1}, {20: 1, 7: 5}],
                         ids=["auto-split", "split-off", "split-8kb", "global", "mega", "split-generalrects",
                              "leafinterior", "ifif", "leanli", "cons", "dict", "dict-leafinterior"])
def test_large_scene_top_of_tree_cache(gpu, opts):
    """C5's N=64 maze: 5.5 k nodes (177 KB) exceed the LDS budget, so the
    default kernel caches the top of the breadth-first node array in LDS and
    reads the rest through L1/L2.  Bit-exact vs the oracle at C5 limits."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(64)
    assert s.n_nodes * 32 > 160 * 1024
    o = Oracle.from_scene(s)
    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    u = default_uniform(3840, 2160, 0)
    e = make_ext(4, 16, 16, frame=5)
    for (x0, y0) in [(0, 0), (1900, 1000), (3000, 1800), (640, 1500)]:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, 32, 16)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        if opts.get(7) == 9:  # the verified search does its own (larger) amount of work
            assert st.rays == rst.rays
        else:
            assert (st.rays, st.node_visits, st.rect_tests) == (rst.rays, rst.node_visits, rst.rect_tests)
    r.close()


def test_bench_prints_one_json_line(gpu):
    """bench.py's driver contract: exactly one JSON line on stdout with the
    metric, the roofline and the issue mode (short C2 run)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--config", "c2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["unit"] == "Mrays/s" and d["value"] > 0 and d["n_gpus"] == 1 and d["steps"] == 2
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert d["config"]["frame_contexts"] in (1, 2)
    assert d["config"]["frames_per_launch"] == 2  # default batching: the 2 timed frames in one launch
    assert d["roofline"]["launches"] == 1


def test_bench_issue_mode_calibration(gpu):
    """bench.py --batch 0 times one context, two contexts and batches of 8
    after warmup and reports all three; --batch 1 --contexts 2 alternates
    single-frame launches over two contexts."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    for extra, check in ((["--batch", "0"], lambda d: set(d["config"]["frame_contexts_calibration_ms"]) ==
                          {"1", "2", "batch8"}),
                         (["--batch", "1", "--contexts", "2"], lambda d: d["config"]["frame_contexts"] == 2 and
                          d["config"]["frames_per_launch"] == 1 and d["roofline"]["launches"] == 3)):
        r = subprocess.run([sys.executable, str(repo / "bench.py"), "--config", "c1", "--steps", "3", "--warmup", "1",
                            "--no-cpu-baseline"] + extra, capture_output=True, text=True, timeout=240, cwd=repo)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
        assert len(lines) == 1, r.stdout
        assert check(json.loads(lines[0])), lines[0]
