"""CPU model of the rejection sampling's two-trial bank (mm_trace.h
shade_step) against the reference's plain loop (shaders.metal:315-318).

The reference draws trials from a path's RNG stream until one is accepted,
once per diffuse bounce.  The kernel lets the lanes of a wave that do not need
a trial draw ahead while the wave loops for the lanes that do, banking up to
two accepted trials (the first's end state in s1, the second's in seed) and
re-deriving a banked trial later by rewinding the LCG three steps.  This model
runs the kernel's statement, lane-parallel in numpy uint32 / float32 with the
device's operations, over many bounces with random diffuse / mirror masks and
random parking of paths through the tail record ((n - mh) | mh << 15 |
bank << 30, s1), and checks that every lane's k-th diffuse direction sample is
the k-th accepted trial of its stream -- what the reference computes.
"""
from __future__ import annotations

import numpy as np

A, C = np.uint32(747796405), np.uint32(291336453)
HASH = np.uint32(277803737)
ONE_PLUS = np.float32(1.0) + np.float32(2.0 ** -23)      # length(r) > 1 <=> len2 > 1 + 2^-23
ACC_EDGE = np.float32(1.0) + np.float32(2.0 ** -22)      # accepted <=> q2 < 1 + 2^-22 (the kernel's sign test)


def lcg_inv(a: int) -> int:
    x = a
    for _ in range(5):
        x = (x * (2 - a * x)) % 2**32
    return x


A3 = (int(A) ** 3) % 2**32
BACK3_A = np.uint32(lcg_inv(A3))
BACK3_C = np.uint32((-int(BACK3_A) * (int(C) * (1 + int(A) + int(A) ** 2))) % 2**32)


def rand_pm1(s):
    """mm_device.h rand_pm1 on uint32 arrays: the new state and RN(RN(float(r)) * 2^-31 - 1)."""
    with np.errstate(over="ignore"):
        s = s * A + C
        r = ((s >> ((s >> np.uint32(28)) + np.uint32(4))) ^ s) * HASH
    r = (r >> np.uint32(22)) ^ r
    # float(r) * 2^-31 is exact, so the fma's single rounding is the float32 subtraction's
    return s, (r.astype(np.float32) * np.float32(2.0 ** -31)) - np.float32(1.0)


def trial(s):
    s, x = rand_pm1(s)
    s, y = rand_pm1(s)
    s, z = rand_pm1(s)
    q2 = (x * x + y * y) + z * z  # dot3 in the IR's order, float32 throughout
    return s, np.stack([x, y, z], axis=-1), q2


def reference_samples(seed0, count):
    """Per lane, its first `count` accepted trials in stream order (the reference's loop)."""
    out = []
    for s0 in seed0:
        s = np.array([s0], dtype=np.uint32)
        got = []
        while len(got) < count:
            s, d, q2 = trial(s)
            if not q2[0] > ONE_PLUS:
                got.append(d[0])
        out.append(got)
    return out


def pack(n, mh, bank):
    return (n - mh) | (mh << 15) | (bank << 30)


def unpack(w):
    mh = (w >> 15) & 0x7FFF
    return (w & 0x7FFF) + mh, mh, w >> 30


def test_rewind_constants():
    s = np.arange(1, 1000, dtype=np.uint32) * np.uint32(2654435761)
    t, _, _ = trial(s)
    with np.errstate(over="ignore"):
        assert np.array_equal(t * BACK3_A + BACK3_C, s)


def test_tail_word_round_trip():
    rng = np.random.default_rng(3)
    for _ in range(2000):
        mh = int(rng.integers(0, 32767))
        n = mh + int(rng.integers(0, 32767))
        bank = int(rng.integers(0, 3))
        assert unpack(pack(n, mh, bank)) == (n, mh, bank)


def test_two_trial_bank_yields_the_reference_samples():
    rng = np.random.default_rng(7)
    lanes, bounces = 64, 60
    seed0 = rng.integers(0, 2**32, size=lanes, dtype=np.uint64).astype(np.uint32)
    ref = reference_samples(seed0, bounces)
    seed = seed0.copy()
    s1 = np.zeros(lanes, np.uint32)
    bank = np.zeros(lanes, np.uint32)
    n = np.zeros(lanes, np.int64)
    mh = np.zeros(lanes, np.int64)
    used = np.zeros(lanes, np.int64)  # diffuse samples taken per lane
    loops = 0
    for b in range(bounces):
        diffuse = rng.random(lanes) < 0.9
        # the in-line trial: the first banked one (rewound from s1) or a fresh one
        banked = bank > 0
        with np.errstate(over="ignore"):
            s = np.where(banked, s1 * BACK3_A + BACK3_C, seed)
        s_end, rd, len2 = trial(s)
        seed = np.where(diffuse & ~banked, s_end, seed)
        s1 = np.where(diffuse, seed, s1)
        bank = np.where(diffuse & banked, bank - 1, bank).astype(np.uint32)
        need = (diffuse & (len2 > ONE_PLUS)).astype(np.uint32)
        while need.any():
            loops += 1
            t_end, d, q2 = trial(seed)
            acc = (q2 < ACC_EDGE).astype(np.uint32)
            act = ((bank >> 1) ^ 1) & diffuse  # (the loop runs in the diffuse branch only)
            seed = np.where(act == 1, t_end, seed)
            take = need & acc
            rd = np.where(take[:, None] == 1, d, rd)
            gain = ((acc & act) - take).astype(np.uint32)
            s1 = np.where(gain > bank, t_end, s1)
            bank = bank + gain
            need = need - take
        for i in np.nonzero(diffuse)[0]:
            assert np.array_equal(rd[i], ref[i][used[i]]), (b, i)
            used[i] += 1
        mh += ~diffuse
        n += 1
        # park a random subset through the tail record and resume them in other lanes
        park = rng.random(lanes) < 0.3
        idx = np.nonzero(park)[0]
        if len(idx) > 1:
            perm = rng.permutation(idx)
            words = [(int(seed[i]), pack(int(n[i]), int(mh[i]), int(bank[i])), int(s1[i])) for i in idx]
            for j, i in zip(perm, idx):
                w_seed, w_nmb, w_s1 = words[list(idx).index(i)]
                seed[j], s1[j] = w_seed, w_s1
                n[j], mh[j], bank[j] = unpack(w_nmb)
            # the lanes' bookkeeping follows the paths
            for arr in (used,):
                arr[perm] = arr[idx].copy()
            ref_moved = {int(j): ref[int(i)] for j, i in zip(perm, idx)}
            for j, r in ref_moved.items():
                ref[j] = r
            seed0[perm] = seed0[idx].copy()
    assert used.min() > bounces // 2 and loops > 0
    # the bank saves loop iterations against a wave that draws only for the lanes in need
    assert loops < 3.2 * bounces
