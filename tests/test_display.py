"""Display stage and frame files on the CPU: the oracle's fragment_shader blur
against an independent numpy statement, the RGBA8 store conversion (product
host twin vs oracle vs numpy) and the PPM / PNG writers (decoded back)."""
from __future__ import annotations

import struct
import zlib

import numpy as np
import pytest


def _blur_numpy(tex: np.ndarray) -> np.ndarray:
    """fragment_shader (src/shaders.metal:214-225) in the IR's operation order
    (src/shaders.ir: ((L+R)+D)+U, *0.5, +C, *RN(1/3)), Jacobi, OOB = 0."""
    f = tex[..., :3].astype(np.float32) / np.float32(255)
    p = np.pad(f, ((1, 1), (1, 1), (0, 0)))
    C, R, L = p[1:-1, 1:-1], p[1:-1, 2:], p[1:-1, :-2]
    D, U = p[2:, 1:-1], p[:-2, 1:-1]
    s = ((L + R) + D) + U
    s = s * np.float32(0.5)
    s = s + C
    s = s * np.float32(1.0 / 3.0)  # RN(1/3) = 0x1.555556p-2
    out = np.empty_like(tex)
    out[..., :3] = np.rint(np.clip(s, 0, 1) * np.float32(255)).astype(np.uint8)
    out[..., 3] = 255
    return out


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (9, 1), (5, 6), (48, 64)])
@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_blur_matches_numpy(shape, seed):
    from oracle.oracle import present_blur

    assert np.float32(1.0 / 3.0).view(np.uint32) == 0x3EAAAAAB  # the IR constant 0x3FD5555560000000
    rng = np.random.default_rng(seed)
    tex = rng.integers(0, 256, size=shape + (4,), dtype=np.uint8)
    assert np.array_equal(present_blur(tex), _blur_numpy(tex))


def test_blur_jacobi_properties():
    from oracle.oracle import present_blur

    # a black texture stays black; one white texel spreads to its 4 neighbours
    tex = np.zeros((5, 5, 4), np.uint8)
    assert np.array_equal(present_blur(tex)[..., :3], tex[..., :3])
    tex[2, 2, :3] = 255
    out = present_blur(tex)
    assert out[2, 2, 0] == 85            # 255/3
    # neighbours: RN(RN(0.5 * RN(1/3)) * 255) is exactly 42.5, a tie -> even 42
    assert out[1, 2, 0] == out[3, 2, 0] == out[2, 1, 0] == out[2, 3, 0] == 42
    assert out[0, 0, 0] == 0 and (out[..., 3] == 255).all()


def _special_floats(rng, n):
    x = rng.uniform(-0.5, 1.5, size=(n, 4)).astype(np.float32)
    ties = (np.arange(256, dtype=np.float32) + np.float32(0.5)) / np.float32(255)
    x[: len(ties), 0] = ties
    x[:4, 1] = [np.nan, np.inf, -np.inf, -0.0]
    return x


def test_quantize_host_twin_matches_oracle_and_numpy():
    from mirror_maze import io
    from oracle.oracle import quantize as oq

    x = _special_floats(np.random.default_rng(3), 4096)
    got = io.quantize(x)
    assert np.array_equal(got, oq(x))
    ref = np.rint(np.clip(np.nan_to_num(x, nan=0.0), 0, 1) * np.float32(255)).astype(np.uint8)
    assert np.array_equal(got, ref)


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(typ + body) == crc, typ
        chunks.append((typ, body))
        pos += 12 + n
    assert [c[0] for c in chunks] == [b"IHDR", b"IDAT", b"IEND"]
    w, h, depth, ctype, comp, filt, lace = struct.unpack(">IIBBBBB", chunks[0][1])
    assert (depth, ctype, comp, filt, lace) == (8, 6, 0, 0, 0)
    raw = zlib.decompress(chunks[1][1])  # checks the Adler-32 too
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 4 * w)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 4)


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (97, 211), (300, 400)])
def test_png_and_ppm_round_trip(tmp_path, shape):
    from mirror_maze import io

    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, size=shape + (4,), dtype=np.uint8)
    io.write_png(tmp_path / "a.png", img)
    assert np.array_equal(_read_png(tmp_path / "a.png"), img)
    io.write_ppm(tmp_path / "a.ppm", img)
    data = open(tmp_path / "a.ppm", "rb").read()
    hdr = f"P6\n{shape[1]} {shape[0]}\n255\n".encode()
    assert data.startswith(hdr)
    assert np.array_equal(np.frombuffer(data[len(hdr):], np.uint8).reshape(shape + (3,)), img[..., :3])


def test_writer_errors(tmp_path):
    from mirror_maze import MMError, io

    with pytest.raises(ValueError):
        io.write_png(tmp_path / "x.png", np.zeros((4, 4, 3), np.uint8))
    with pytest.raises(MMError):
        io.write_png(tmp_path / "no_such_dir" / "x.png", np.zeros((4, 4, 4), np.uint8))
