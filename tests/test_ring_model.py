"""CPU model check of the tail ring's protocol (trace_kernels.hip ring_reserve /
ring_claim / ring_wait / wavepersist_ring_body, mm_path.h bounce_loop_r):
tests/ring_model/ring_model.cpp runs one block's waves under a seeded random
scheduler, one atomic LDS step at a time, with the SIMT rule that a wave's
waiting lanes release nothing before all of them are satisfied.

What it found (the round-3 timeout in
profiles/r03/gpu_tests_r3d_failure.log):
* round-3 kernel (policy 0), 64-lane deferral: a wave in its main phase that
  claims 64 parked tails re-parks all 64 at the top of their first bounce (64
  <= defer_lanes) and claims them again -- no bounce is ever run.  Once its
  block-mates have drained and exited, nothing breaks the cycle: the 32-bit
  entry counters run on until lap = seq / 512 wraps from 2^23 - 1 to 0, where
  the writer waits for turn 0 while the slot holds 2^24 -- the "tail ring wait
  timed out" the GPU run reported.
* round-4 kernel (policy 3): a claimed tail chunk of <= defer_lanes lanes runs
  with deferral off (every claim then runs >= 1 bounce), and turn values are
  taken modulo 2^24 (the wrap is seamless).  No deadlock, livelock, lost or
  duplicated path over the sweep below.
"""
from __future__ import annotations

import json
import subprocess
from pathlib import Path

import pytest

SRC = Path(__file__).resolve().parent / "ring_model" / "ring_model.cpp"
WRAP = 2**32 - 200  # counters just below the 32-bit wrap


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    exe = tmp_path_factory.mktemp("ring_model") / "ring_model"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-o", str(exe), str(SRC)], check=True)

    def run(waves, lanes, ring, chunks, max_b, defer_lanes, seed, policy, burst=4, cost=10, steps=3_000_000,
            seq0=None):
        args = [str(exe), *map(str, (waves, lanes, ring, chunks, max_b, defer_lanes, 1, steps, seed, policy, burst,
                                     cost))]
        if seq0 is not None:
            args.append(str(seq0))
        r = subprocess.run(args, capture_output=True, text=True, timeout=60)
        return json.loads(r.stdout)

    return run


def test_round3_protocol_livelocks_with_64_lane_deferral(model):
    """The counter-example: a lone wave cycling 64 tails through the ring."""
    verdicts = [model(2, 64, 512, 2, 20, 64, s, policy=0, burst=1, cost=1)["verdict"] for s in range(1, 61)]
    assert "livelock" in verdicts
    assert set(verdicts) <= {"ok", "livelock"}


def test_round3_turn_values_stall_at_the_sequence_wrap(model):
    r = model(4, 64, 512, 24, 20, 32, 1, policy=1, seq0=WRAP)
    assert r["verdict"] == "deadlock" and r["states"].split() == ["W_WAIT"] * 4  # writers wait for turn 0
    assert model(4, 64, 512, 24, 20, 32, 1, policy=3, seq0=WRAP)["verdict"] == "ok"


@pytest.mark.parametrize("defer_lanes", [16, 32, 63, 64])
def test_round4_protocol_terminates_and_conserves_paths(model, defer_lanes):
    """Kernel geometry (16 waves of 64 lanes, 512 entries) and small blocks,
    queues of 1..24 chunks, several scheduler quanta and bounce costs."""
    n = 0
    for waves in (2, 4, 16):
        for chunks in (1, 2, 12, 24):
            for seed in range(1, 9):
                r = model(waves, 64, 512, chunks, 20, defer_lanes, seed, policy=3, burst=1 + seed % 8,
                          cost=1 + 7 * (seed % 4))
                assert r["verdict"] == "ok", (waves, chunks, seed, r)
                assert r["lost"] == 0 and r["dup"] == 0 and r["reserved"] == r["claimed"]
                n += 1
    assert n == 96


def test_round4_protocol_small_rings(model):
    """Rings of 4..16 entries and 4-lane waves: many laps per run."""
    for ring in (4, 6, 8, 16):
        for seed in range(1, 41):
            r = model(2 + seed % 5, 4, ring, 1 + seed % 7, 12, 1 + seed % 4, seed, policy=3, burst=1 + seed % 9,
                      cost=1 + seed % 20)
            assert r["verdict"] == "ok", (ring, seed, r)
            assert r["lost"] == 0 and r["dup"] == 0


@pytest.mark.parametrize("defer_lanes", [16, 32, 64])
def test_end_split_terminates_and_conserves_paths(model, defer_lanes):
    """The end-of-queue split (MM_END_SPLIT, A/B; policy bit 2): new chunks of
    the queue's last 4 x waves chunks park all their live lanes once a wave has
    seen the queue out, and claims made then take an even share of the ring.
    Each new chunk parks this way at most once and every claim still runs >= 1
    bounce: no deadlock, livelock, lost or duplicated path."""
    end_parks = 0
    for waves in (2, 4, 16):
        for chunks in (1, 12, 24, 80):
            for seed in range(1, 7):
                r = model(waves, 64, 512, chunks, 20, defer_lanes, seed, policy=7, burst=1 + seed % 8,
                          cost=1 + 7 * (seed % 4))
                assert r["verdict"] == "ok", (waves, chunks, seed, r)
                assert r["lost"] == 0 and r["dup"] == 0 and r["reserved"] == r["claimed"]
                end_parks += r["end_parks"]
    for ring in (4, 8, 16):
        for seed in range(1, 21):
            r = model(2 + seed % 5, 4, ring, 1 + seed % 9, 12, 1 + seed % 4, seed, policy=7, burst=1 + seed % 9,
                      cost=1 + seed % 20)
            assert r["verdict"] == "ok", (ring, seed, r)
            assert r["lost"] == 0 and r["dup"] == 0
            end_parks += r["end_parks"]
    assert end_parks > 0  # the split path ran
