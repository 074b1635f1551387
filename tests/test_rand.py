"""rand 0.8.5 StdRng restatement (ChaCha12 + seed_from_u64 + gen + shuffle).

Pinned by the RFC 8439 ChaCha20 known answers; the 12-round StdRng stream and
the rand crate's sampling algorithms are cross-checked between the product's
C++ (mirror-maze_amd/csrc/scene.cpp) and the independent Python restatement
(oracle/scene_oracle.py).  Stream parity with the real crate: UNPINNED
(crate not vendored, no Rust toolchain).
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np
import pytest

from conftest import GOLDEN


def _c():
    from mirror_maze import _lib

    return _lib, _lib.lib()


def _words_le(b: bytes):
    return [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]


def test_chacha20_rfc8439_block():
    from oracle import scene_oracle as so

    g = json.loads((GOLDEN / "chacha_rfc8439.json").read_text())["block_2_3_2"]
    key = _words_le(bytes(g["key"]))
    nonce = _words_le(bytes.fromhex(g["nonce_hex"]))
    # IETF layout: word12 = counter, words 13..15 = nonce -> djb 64-bit fields
    counter = g["counter"] | (nonce[0] << 32)
    stream = nonce[1] | (nonce[2] << 32)
    _, L = _c()
    k = (C.c_uint32 * 8)(*key)
    out = (C.c_uint32 * 16)()
    L.mm_chacha_block(k, counter, stream, 20, out)
    assert list(out) == g["out_words"]
    assert so.chacha_block(key, counter, stream, 20) == g["out_words"]


def test_chacha20_zero_key_keystream():
    from oracle import scene_oracle as so

    g = json.loads((GOLDEN / "chacha_rfc8439.json").read_text())["a1_tv1"]
    want = _words_le(bytes.fromhex(g["keystream_hex"]))
    _, L = _c()
    out = (C.c_uint32 * 16)()
    L.mm_chacha_block((C.c_uint32 * 8)(), 0, 0, 20, out)
    assert list(out) == want
    assert so.chacha_block([0] * 8, 0, 0, 20) == want


@pytest.mark.parametrize("seed", [0, 1, 42, 2**63 + 5])
def test_stdrng_stream_cpp_vs_python(seed):
    from oracle import scene_oracle as so

    _lib, L = _c()
    r = _lib.mm_rng()
    L.mm_rng_seed_from_u64(C.byref(r), seed)
    py = so.StdRng.seed_from_u64(seed)
    assert list(r.key) == py.key
    # 300 words crosses several 64-word refills
    assert [L.mm_rng_next_u32(C.byref(r)) for _ in range(300)] == [py.next_u32() for _ in range(300)]


def test_gen_f32_and_gen_range():
    from oracle import scene_oracle as so

    _lib, L = _c()
    r = _lib.mm_rng()
    L.mm_rng_seed_from_u64(C.byref(r), 0)
    py = so.StdRng.seed_from_u64(0)
    for i in range(200):
        a = L.mm_rng_gen_f32(C.byref(r))
        b = float(py.gen_f32())
        assert a == b and 0.0 <= a < 1.0
        hi = 1 + (i * 7919) % 1000
        assert L.mm_rng_gen_range_u32(C.byref(r), 0, hi) == py.gen_range_u32(0, hi)


def test_gen_range_rejects_in_zone():
    """Lemire zone: results are in range and roughly uniform."""
    _lib, L = _c()
    r = _lib.mm_rng()
    L.mm_rng_seed_from_u64(C.byref(r), 3)
    v = np.array([L.mm_rng_gen_range_u32(C.byref(r), 5, 12) for _ in range(7000)])
    assert v.min() == 5 and v.max() == 11
    counts = np.bincount(v - 5)
    assert counts.min() > 850 and counts.max() < 1150


def test_next_u64_straddles_buffer():
    _lib, L = _c()
    a, b = _lib.mm_rng(), _lib.mm_rng()
    L.mm_rng_seed_from_u64(C.byref(a), 9)
    L.mm_rng_seed_from_u64(C.byref(b), 9)
    for _ in range(63):
        L.mm_rng_next_u32(C.byref(a))
        L.mm_rng_next_u32(C.byref(b))
    lo = L.mm_rng_next_u32(C.byref(b))
    hi = L.mm_rng_next_u32(C.byref(b))
    assert L.mm_rng_next_u64(C.byref(a)) == (hi << 32) | lo
