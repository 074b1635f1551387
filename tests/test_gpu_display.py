"""Display stage on the GPU, bit-exact against the oracle: the reference's
per-frame sequence (chunk scheduler -> compute_shader -> fragment_shader blur,
src/main.rs:778-894) on the RGBA8 texture, the shaders.air packet format and
the device RGBA8 quantisation."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_display_loop_frames_bit_exact(gpu):
    """Three frames of the reference loop at P0 (N=10, 1024x768, 768 chunks
    per frame from the seeded scheduler, time = frame): the RGBA8 texture after
    each present equals the oracle's, texel for texel."""
    from mirror_maze import ChunkScheduler, Renderer, Scene, default_uniform
    from oracle.oracle import DisplayLoop, Oracle

    s = Scene.build(10, 0)
    r = Renderer(0)
    r.upload_scene(s)
    loop = DisplayLoop(Oracle.from_scene(s), 1024, 768)
    sched = ChunkScheduler(1024, 768, 4, seed=7)
    for frame in range(3):
        chunks = sched.next(768)
        u = default_uniform(1024, 768, frame)
        r.compute_shader(u, chunks)
        r.present()
        _, got = r.read_texture()
        ref = loop.frame(u, chunks)
        bad = (got != ref).any(axis=-1)
        assert not bad.any(), f"frame {frame}: {int(bad.sum())} texels differ"
    assert (got[..., 3] == 255).all() and got[..., :3].any()
    r.close()


def test_packets_match_framebuffer_and_coordinates(gpu):
    from mirror_maze import ChunkScheduler, Renderer, Scene, default_uniform
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    r = Renderer(0)
    r.upload_scene(s)
    chunks = ChunkScheduler(1024, 768, 4, seed=1).next(768)
    u = default_uniform(1024, 768, 0)
    r.compute_shader(u, chunks)
    pk = r.read_packets(768)
    ref, _ = Oracle.from_scene(s).trace_chunks(u, chunks)
    pn = np.arange(16)
    xs = chunks[:, 0:1] + pn[None, :] // 4
    ys = chunks[:, 1:2] + pn[None, :] % 4
    assert np.array_equal(pk[..., 3].view(np.uint32), (xs << 16 | ys).astype(np.uint32))
    assert np.array_equal(pk[..., :3].view(np.uint32), ref[ys, xs, :3].view(np.uint32))
    with pytest.raises(Exception):
        r.read_packets(769)
    r.close()


def test_device_quantize_matches_host_twin(gpu):
    import torch

    from mirror_maze import Renderer, io

    rng = np.random.default_rng(5)
    x = rng.uniform(-0.5, 1.5, size=(37, 53, 4)).astype(np.float32)
    x[0, :, 0] = (np.arange(53, dtype=np.float32) + np.float32(0.5)) / np.float32(255)  # exact ties
    x[1, :4, 1] = [np.nan, np.inf, -np.inf, -0.0]
    r = Renderer(0)
    got = r.quantize(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(got, io.quantize(x))
    r.close()


def test_offline_frame_to_png(gpu, tmp_path):
    """trace_tile -> device quantise -> PNG, and the file decodes to the
    oracle's quantised frame."""
    from mirror_maze import Renderer, Scene, default_uniform, io, make_ext
    from oracle.oracle import Oracle
    from test_display import _read_png

    s = Scene.build(16, 0)
    r = Renderer(0)
    r.upload_scene(s)
    u = default_uniform(128, 72, 0)
    e = make_ext(2, 4, 15, frame=0)
    img, _ = r.trace_tile(u, e, 0, 0, 128, 72)
    rgba8 = r.quantize(img).cpu().numpy()
    io.write_png(tmp_path / "f.png", rgba8)
    ref, _ = Oracle.from_scene(s).trace_tile(u, e, 0, 0, 128, 72)
    assert np.array_equal(_read_png(tmp_path / "f.png"), io.quantize(ref))
    r.close()
