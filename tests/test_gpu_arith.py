"""Exact rewrites of IEEE operations, checked exhaustively on the MI355X.

mm::rsq (mm_device.h) computes the reference's fast_rsqrt with its IEEE
meaning -- RN(1 / RN(sqrt(x))), the AIR intrinsic as the oracle states it --
from the hardware v_sqrt_f32 / v_rcp_f32 with exact corrections on
[2^-40, 2^40].  lib/verify_fast_rsq (scripts/verify_fast_rsq.hip, built by the
library's Makefile with its flags) compares it with the IEEE expansion
1.0f / sqrtf(x) for every float x in [2^-44, 2^44], and mm::rcp_guarded (the
per-ray RN(1/d) the Markstein quotients read: one Newton step on v_rcp_f32)
with 1.0f / d for every d of either sign with |d| in [2^-40, 2^40]; and
mm::ray_fast_ok_boxed (the per-query guard as integer compares on the
magnitudes' bits) with mm::ray_fast_ok on every 32-bit pattern."""
from __future__ import annotations

import subprocess

import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu


def test_fast_rsq_is_bit_identical_to_the_ieee_expansion(gpu):
    exe = PKG / "lib" / "verify_fast_rsq"
    assert exe.exists(), "build the library first (make -C mirror-maze_amd)"
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    print(p.stdout)
    assert p.returncode == 0, p.stdout + p.stderr
    rows = {ln.split()[0]: ln.split() for ln in p.stdout.splitlines() if ln.strip()}
    for name, binades in (("rsq", 88), ("rcp_guarded", 80)):  # (rcp_guarded: each value with both signs)
        w = rows[name]
        checked, bad = int(w[2]), int(w[4])
        assert checked > binades * (1 << 23) and bad == 0, w
    # the per-query guard in integer form (mm::ray_fast_ok_boxed) equals the
    # float compares on every 32-bit pattern (origin: where the box can pass)
    w = rows["ray_guard"]
    assert int(w[2]) == 1 << 32 and int(w[4]) == 0, w
