"""Generates the committed fixtures in tests/golden/.  Run from the repo root:

    python tests/golden/make_golden.py            # reference-derived fixtures
    python tests/golden/make_golden.py --oracle   # + oracle regression fixtures

Reference-derived (pin the oracle):
  * noise_texel.json — texel (0,0) of the reference's textures/noiseTexture-2.png
    (the only texel compute_shader ever samples, src/shaders.metal:288-291).
    Needs /root/reference (this container only).
Published-spec (pin the RNG restatement):
  * chacha_rfc8439.json — RFC 8439 §2.3.2 block-function test vector and the
    all-zero-key ChaCha20 keystream block (RFC 8439 §A.1 test vector #1).
Oracle regression (NOT a pin: frozen outputs of oracle/ so later rounds notice
an unintended change; the GPU tests also read them on the box):
  * oracle_p0.npz — N=10 reference scene, 1024x768, 32 chunks, time 0/1.
  * oracle_c1.npz — C1: N=16, 256x256, 1 spp, 1 bounce, full frame.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent


def noise_texel() -> None:
    from PIL import Image

    png = Path("/root/reference/textures/noiseTexture-2.png")
    im = Image.open(png).convert("RGBA")
    rec = {
        "source": "reference textures/noiseTexture-2.png (src/main.rs:354, 667-695)",
        "size": list(im.size),
        "texel_0_0_rgba8": list(im.getpixel((0, 0))),
        "note": "sampler(repeat, nearest), normalized coords at float2(gid) -> texel (0,0) for every thread",
    }
    (HERE / "noise_texel.json").write_text(json.dumps(rec, indent=1) + "\n")


def chacha() -> None:
    rec = {
        "source": "RFC 8439 (ChaCha20 and Poly1305), IETF, published test vectors",
        "block_2_3_2": {
            "key": list(range(32)),
            "counter": 1,
            "nonce_hex": "000000090000004a00000000",
            "out_words": [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204,
                          0x4E6CD4C3, 0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE,
                          0xE883D0CB, 0x4E3C50A2],
        },
        "a1_tv1": {
            "key": [0] * 32,
            "counter": 0,
            "nonce_hex": "000000000000000000000000",
            "keystream_hex": ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                              "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586"),
        },
    }
    (HERE / "chacha_rfc8439.json").write_text(json.dumps(rec, indent=1) + "\n")


def oracle_fixtures() -> None:
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "mirror-maze_amd"))
    from mirror_maze import ChunkScheduler, Scene, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = Scene.build(10, 0)
    o = Oracle.from_scene(s)
    cs = ChunkScheduler(1024, 768, 4, seed=7)
    chunks = cs.next(768)
    out = {}
    for t in (0, 1):
        u = default_uniform(1024, 768, t)
        fb = np.zeros((768, 1024, 4), np.float32)
        # only the first 32 groups (gy = 0) to keep the fixture small
        for gx in range(32):
            o.trace_group(u, chunks, gx, 0, fb)
        out[f"fb_t{t}"] = fb
    ys, xs = np.nonzero(out["fb_t0"][..., 3] == 1.0)
    np.savez_compressed(HERE / "oracle_p0.npz", chunks=chunks, ys=ys.astype(np.uint16), xs=xs.astype(np.uint16),
                        rgb_t0=out["fb_t0"][ys, xs, :3], rgb_t1=out["fb_t1"][ys, xs, :3])
    s16 = Scene.build(16, 0)
    o16 = Oracle.from_scene(s16)
    u = default_uniform(256, 256, 0)
    img, st = o16.trace_tile(u, make_ext(spp=1, bounce_limit=1, mirror_limit=15), 0, 0, 256, 256)
    np.savez_compressed(HERE / "oracle_c1.npz", rgb=img[..., :3], rays=st.rays, visits=st.node_visits,
                        rtests=st.rect_tests)


if __name__ == "__main__":
    if Path("/root/reference").exists():
        noise_texel()
    chacha()
    if "--oracle" in sys.argv:
        oracle_fixtures()
