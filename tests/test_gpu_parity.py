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
    """C1: 16x16 maze, 256x256, 1 spp, 1 bounce -- the default query method
    (grid search) and the lean BVH form, whose work counts are the oracle's."""
    from mirror_maze import MM_TRAV_AUTO, MM_TRAV_LEAN, default_uniform, make_ext

    g = np.load(GOLDEN / "oracle_c1.npz")
    ren.upload_scene(_scene(16))
    for form in (MM_TRAV_AUTO, MM_TRAV_LEAN):
        ren.set_option(7, form)
        img, st = ren.trace_tile(default_uniform(256, 256, 0), make_ext(1, 1, 15), 0, 0, 256, 256, stats=True)
        img = img.cpu().numpy()
        assert np.array_equal(_bits(img[..., :3]), _bits(g["rgb"]))
        assert st.rays == int(g["rays"])
        if form == MM_TRAV_LEAN:
            assert st.node_visits == int(g["visits"]) and st.rect_tests == int(g["rtests"])
    ren.set_option(7, MM_TRAV_AUTO)


WINDOWS = [(0, 0), (960, 540), (1888, 1064), (300, 700), (1500, 100)]


# (pipeline, {option: value}, exact_counts); options (include/mm_api.h): 1 LDS,
# 7 traversal (-1 auto, 5, 7 BVH loop forms, 11 grid search), 8 LDS rect
# records, 12 fused resolve, 21 / 22 tail deferral.  (The A/B-only variants --
# one thread per path, loop form 0, split node cache, dictionary nodes, form 7
# with global records -- were removed in round 6; the
# options that chose them fail: test_removed_variants_refused.)
# exact_counts: node visits and rect tests equal the oracle's (BVH walks); the
# grid search counts its own work (cells, rect tests), only rays and paths match.
PIPES = {
    "reference": (3, {}, True),
    "auto": (0, {}, False),                                  # grid search (C3 default)
    "grid": (1, {7: 11}, False),
    "grid-nofuse": (1, {7: 11, 12: 0}, False),
    "grid-nodefer": (1, {21: 0}, False),
    "grid-defer": (1, {21: 32, 22: 0}, False),               # tail deferral (32 lanes) on any launch size
    "grid-defer16": (1, {21: 16, 22: 0}, False),
    "grid-defer63": (1, {21: 63, 22: 0}, False),
    "grid-defer64": (1, {21: 64, 22: 0}, False),             # every path at bounce 1: tail rings run full
    "bvh-lean-defer32": (1, {7: 7, 21: 32, 22: 0}, True),
    "bvh-lean-ldsrects": (1, {7: 7}, True),
    "bvh-li-ldsrects": (1, {7: 5}, True),
    "bvh-li-globalrecs": (1, {7: 5, 8: 0}, True),
    "bvh-li-global": (1, {7: 5, 1: 0}, True),
    "wavefront": (2, {}, False),                             # mirror-tail deferral always on
    "wavefront-global": (2, {1: 0}, False),
}


def _renderer(pipe, scene):
    from mirror_maze import Renderer

    r = Renderer(0)
    p, opts, _ = PIPES[pipe]
    r.set_pipeline(p)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(scene)
    return r


@pytest.mark.parametrize("pipe", sorted(PIPES))
@pytest.mark.parametrize("cfg", [
    dict(n=16, spp=1, b=4, m=15),   # C2 settings
    dict(n=32, spp=8, b=8, m=8),    # C3 settings (the benchmark)
    dict(n=10, spp=3, b=5, m=15),   # non-multiple-of-8 spp
    dict(n=32, spp=16, b=8, m=15),  # C4 settings
])
def test_tile_windows_bit_exact(gpu, cfg, pipe):
    from mirror_maze import default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(cfg["n"])
    ren = _renderer(pipe, s)
    o = Oracle.from_scene(s)
    u = default_uniform(1920, 1080, 0)
    e = make_ext(cfg["spp"], cfg["b"], cfg["m"], frame=2)
    for (x0, y0) in WINDOWS:
        w, h = 32, 16
        got, st = ren.trace_tile(u, e, x0, y0, w, h, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, w, h)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        assert (st.rays, st.paths) == (rst.rays, rst.paths)
        if PIPES[pipe][2]:
            assert (st.node_visits, st.rect_tests) == (rst.node_visits, rst.rect_tests)
    ren.close()


@pytest.mark.parametrize("pipe", ["auto", "grid-nofuse", "grid-nodefer", "grid-defer", "grid-defer64",
                                  "bvh-lean-ldsrects", "bvh-li-global", "reference", "wavefront"])
def test_small_full_frames_bit_exact(gpu, pipe):
    """Whole 256x144 frames (8 spp, 8/8 bounces, 3 frames, N=32 maze): ~7 M
    closest-hit queries per pipeline against the oracle, so rare boundary
    cases of the exact-division and threshold tests get exercised."""
    from mirror_maze import default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(32)
    o = Oracle.from_scene(s)
    r = _renderer(pipe, s)
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


@pytest.mark.parametrize("opts", [{}, {7: 5}, {7: 5, 1: 0}, {7: 7}, {19: 8}, {21: 0}, {21: 32, 22: 0}])
def test_multi_frame_launch_bit_identical(gpu, opts):
    """mm_trace_tile_frames: F frames in one launch (one work queue) equal the
    F single-frame launches bit for bit, with summed work counts -- C3 whole
    frames and a row-split tile; the grid search (default), loop form 5 with
    the nodes in LDS and through L1/L2, the lean BVH form; a grid 8 CUs short
    (MM_OPT_RESERVE_CUS)."""
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
    with pytest.raises(MMError):
        r.trace_tile_frames(u, make_ext(8, 3, 15), 0, 0, 0, 64, 64)
    # 3 spp: no fused resolve; with tail deferral the frames are staged and resolved per frame
    r.set_option(22, 0)
    three, _ = r.trace_tile_frames(u, make_ext(3, 3, 15, frame=1), 2, 0, 0, 64, 64)
    for f in range(2):
        ref, _ = r.trace_tile(u, make_ext(3, 3, 15, frame=1 + f), 0, 0, 64, 64)
        assert np.array_equal(_bits(three[f].cpu().numpy()), _bits(ref.cpu().numpy()))
    r.set_option(21, 0)  # without deferral: needs the fused resolve
    with pytest.raises(MMError):
        r.trace_tile_frames(u, make_ext(3, 3, 15), 2, 0, 0, 64, 64)
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


@pytest.mark.parametrize("fuse,defer_min", [(1, 1 << 30), (0, 1 << 30), (1, 0), (1, 1 << 21)])
def test_accumulate_flag(ren, gpu, fuse, defer_min):
    from mirror_maze import MM_EXT_ACCUMULATE, default_uniform, make_ext

    ren.upload_scene(_scene(10))
    ren.set_option(12, fuse)
    ren.set_option(22, defer_min)
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


@pytest.mark.parametrize("opts", [{}, {7: 5}, {7: 5, 1: 0}, {7: 11, 1: 0}],
                         ids=["auto", "li-global-nodes", "li-nothing-in-lds", "grid-not-in-lds"])
def test_large_scene_bit_exact(gpu, opts):
    """C5's N=64 maze: the grid image (cells, lists, records, leaf boxes) and
    the BVH (5.5 k nodes, 177 KB) exceed the LDS budget.  Auto runs the grid
    search with its index in LDS and records / leaf boxes through L1/L2; loop
    form 5 reads the nodes through L1/L2.
    Bit-exact vs the oracle at C5 limits (16/16 bounces) on 4 windows."""
    from mirror_maze import MM_INFO_GRID_BYTES, MM_INFO_GRID_INDEX_BYTES, MM_INFO_GRID_OK, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(64)
    assert s.n_nodes * 32 > 160 * 1024
    o = Oracle.from_scene(s)
    from mirror_maze import Renderer

    r = Renderer(0)
    for k, v in opts.items():
        r.set_option(k, v)
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 1.0
    assert r.scene_info(MM_INFO_GRID_BYTES) > 80 * 1024 >= r.scene_info(MM_INFO_GRID_INDEX_BYTES)
    u = default_uniform(3840, 2160, 0)
    e = make_ext(4, 16, 16, frame=5)
    for (x0, y0) in [(0, 0), (1900, 1000), (3000, 1800), (640, 1500)]:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, 32, 16)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        assert st.rays == rst.rays
        if opts.get(7) in (5, 7):
            assert (st.node_visits, st.rect_tests) == (rst.node_visits, rst.rect_tests)
    r.close()


def test_grid_cell_formats(gpu):
    """The grid build picks 64-bit cell words with per-face list ranges where
    the index fits the LDS budget (C3's N=32 maze) and plain 32-bit words at
    the same cell size otherwise (N=64), before coarser cells; both are
    covered bit-exact by the whole-frame / window tests (test_gpu_frames.py)."""
    from mirror_maze import MM_INFO_GRID_CELLS_X, MM_INFO_GRID_FACES, MM_INFO_GRID_OK, Renderer

    for n, faces, cells_x in [(32, 1.0, 33), (64, 0.0, 65)]:
        r = Renderer(0)
        r.upload_scene(_scene(n))
        assert r.scene_info(MM_INFO_GRID_OK) == 1.0
        assert r.scene_info(MM_INFO_GRID_FACES) == faces, n
        assert r.scene_info(MM_INFO_GRID_CELLS_X) == cells_x, n
        r.close()


def test_plain_cell_words_option_bit_exact(gpu):
    """MM_OPT_GRID_WIDE 0: C3's maze indexed with plain 32-bit cell words (the
    whole list per cell) instead of per-face list ranges -- the format the
    N=64 scene uses -- is 0 ulp against the oracle on C3 windows, with the
    same ray count."""
    from oracle.oracle import Oracle

    from mirror_maze import MM_INFO_GRID_FACES, MM_INFO_GRID_OK, MM_OPT_GRID_WIDE, Renderer, default_uniform, make_ext

    s = _scene(32)
    o = Oracle.from_scene(s)
    r = Renderer(0)
    r.set_option(MM_OPT_GRID_WIDE, 0)
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 1.0 and r.scene_info(MM_INFO_GRID_FACES) == 0.0
    u = default_uniform(1920, 1080, 0)
    e = make_ext(8, 8, 8, frame=2)
    for (x0, y0) in [(0, 0), (944, 520), (1888, 1064), (300, 800)]:
        got, st = r.trace_tile(u, e, x0, y0, 32, 16, stats=True)
        ref, rst = o.trace_tile(u, e, x0, y0, 32, 16)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref)), (x0, y0)
        assert st.rays == rst.rays
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
    # (a C2 line: executed lane-ops from profiles/pmc_c2.json when it holds these sources, else null)
    rf = d["roofline"]
    assert rf["bound"] == "valu" and (rf["frac"] is None or 0 < rf["frac"] < 1) and rf["basis"]
    assert rf["model_hbm"]["bytes_per_ray"] == 136 and "measured" in rf
    assert rf["reference_equivalent"]["model_ratio"] > 0
    kr = d["roofline"]["kernel_resources"]
    assert 0 < kr["vgprs_per_lane"] <= 64 and kr["scratch_bytes_per_lane"] >= 0
    assert d["distributed"] is None  # one process, no torchrun
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


@pytest.mark.gpu
def test_trace_tile_rejects_limits_beyond_the_packed_state(gpu):
    """Bounce / mirror limits above 32767 would overflow the tail records'
    (n - mh) | mh << 15 | bank << 30 word: an error code, not a wrong image."""
    from mirror_maze import Renderer, default_uniform, make_ext
    from mirror_maze._lib import MMError

    u = default_uniform(64, 32, 0)
    with Renderer(0) as r:
        r.upload_scene(_scene(10))
        for bl, ml in ((40000, 8), (8, 40000)):
            with pytest.raises(MMError):
                r.trace_tile(u, make_ext(1, bl, ml), 0, 0, 4, 4)
        img, _ = r.trace_tile(u, make_ext(1, 32767, 8), 0, 0, 4, 4)  # the bound itself is accepted
        assert img.shape == (4, 4, 4)


def test_removed_variants_refused(gpu):
    """the A/B-only kernel variants were deleted; the
    option values that chose them fail with MM_ERR_UNSUPPORTED (-6) by name,
    the values that select nothing are still accepted, and the version string
    carries no A/B marker."""
    from mirror_maze import MM_INFO_DICT_OK, MMError, Renderer, lib

    assert "+ab" not in lib().mm_version().decode()
    r = Renderer(0)
    for key, val in [(3, 0), (7, 0), (9, 2), (20, 2)]:
        with pytest.raises(MMError) as ei:
            r.set_option(key, val)
        assert ei.value.code == -6 and "removed" in str(ei.value), (key, val)
    for key, val in [(3, 2), (7, 5), (9, 0), (9, 1), (20, 0), (20, 1)]:
        r.set_option(key, val)
    r.upload_scene(_scene(10))
    assert r.scene_info(MM_INFO_DICT_OK) == 0.0
    r.close()
