"""Errors raised on the GPU reach the caller, attributed to the call that
caused them, and valid long paths raise none.

* Long chunks with the tail rings: a bounce limit of 32767 (the largest the
  API takes) with deferral forced makes every chunk run far longer than the
  round-2 drain bound (2^21 polls of s_sleep(2), ~0.13 s); the launch must end
  clean and bit-exact against the oracle.  The loop whose length nothing may
  cap is src/shaders.metal:306 (`n < bounce_limit + mirror_hits`).
* An injected fault (MM_OPT_FAULT_INJECT 1) is reported naming its own call
  -- by mm_sync, by the next trace call (which is then not enqueued) and by
  mm_call_status -- never blamed on a later call.
* Ring protocol timeouts (MM_OPT_FAULT_INJECT 2: waits give up at once) are
  reported with a record of the first stuck wait.
* The round-3 tail-ring livelock (a lone wave cycling 64 tails, 64-lane
  deferral) is gone; a failed enqueue releases its status slot; the status of
  a call older than the kept failures is not reported clean."""
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


def closed_room(n_tiles, mirror_frac, seed):
    """A closed cube [-10, 10]^3 (faces overlapping at the edges: no ray from
    inside escapes) holding n_tiles horizontal 18x18 tiles stacked along y.
    The grid has one cell listing every tile, so every closed-hit query
    tests them all; a fraction of the tiles are mirrors (paths run
    bounce_limit + their mirror hits, so lanes finish at different bounces
    and the tail rings take their last bounces)."""
    from mirror_maze import Scene

    rng = np.random.default_rng(seed)
    rects = []
    for sgn in (-1.0, 1.0):
        rects.append([10 * sgn, -11, -11, 0, 22, 0, 0, 0, 22])   # x faces
        rects.append([-11, 10 * sgn, -11, 22, 0, 0, 0, 0, 22])   # y faces
        rects.append([-11, -11, 10 * sgn, 22, 0, 0, 0, 22, 0])   # z faces
    for i in range(n_tiles):
        y = -9.5 + 19.0 * (i + 0.5) / n_tiles
        rects.append([-9, y, -9, 18, 0, 0, 0, 0, 18])
    r = np.zeros((len(rects), 12), np.float32)
    r[:, :9] = np.asarray(rects, np.float32)
    r[:, 9:12] = rng.uniform(0.3, 0.9, (len(rects), 3))
    is_mirror = np.zeros(len(rects), np.uint8)
    is_mirror[6:] = rng.random(n_tiles) < mirror_frac
    emission = np.tile(np.float32([1, 1, 1, 0.05]), (len(rects), 1))
    nodes, idx = Scene.bvh(r)
    return Scene(0, r, nodes, idx, is_mirror, emission, np.zeros((0, 0), np.uint8), 0)


def test_long_chunks_with_tail_rings_end_clean_and_bit_exact(gpu):
    """Round 2's drain gave up after 2^21 polls of s_sleep(2) (>= 2^21 x 128
    clocks = 0.11 s at 2.4 GHz) although a block-mate's valid chunk may run
    bounce_limit + mirror_limit iterations of arbitrarily long queries.  Here
    one chunk (8 px x 8 spp) runs 32767 + its mirror-hit bounces in a closed
    room where every query tests ~300 tiles, with the tail rings on; the other
    15 waves of its block are past the global queue at once.  The chunk must
    outlast the old bound several times over, and the launch must end clean
    and bit-exact (the loop nothing may cap: src/shaders.metal:306)."""
    import torch

    from mirror_maze import MM_INFO_GRID_OK, MM_INFO_LAST_DEFER, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = closed_room(300, 0.1, 5)
    r = Renderer(0)
    r.set_option(21, 32)  # MM_OPT_DEFER: 32 lanes
    r.set_option(22, 0)   # MM_OPT_DEFER_MIN: any launch size
    r.upload_scene(s)
    assert r.scene_info(MM_INFO_GRID_OK) == 1.0
    u = default_uniform(64, 64, 0)
    for i in range(3):
        u.cam.center[i] = 0.0
    e = make_ext(8, 32767, 32767, frame=1)
    ts = torch.zeros((256 * 2 * 16, 4), dtype=torch.int64, device="cuda")
    r.set_wave_timeline(ts)
    got, st = r.trace_tile(u, e, 30, 30, 8, 1, stats=True)  # 64 paths: one chunk
    r.sync()  # raises if the launch reported an error
    r.set_wave_timeline(None)
    assert r.scene_info(MM_INFO_LAST_DEFER) == 1.0
    t = ts.cpu().numpy()
    busy = t[t[:, 3] > 0]                              # waves that traced at least one chunk
    span_s = (busy[:, 2] - busy[:, 0]).max() / 100e6   # wall_clock64: 100 MHz
    print(f"longest wave: {span_s:.3f} s; {len(busy)} busy waves, {int(busy[:, 3].sum())} chunks; "
          f"{st.rays} queries ({st.rays / 64:.0f} per path), {st.rect_tests / max(st.rays, 1):.0f} tests each")
    # (a path started within 0.1 of a face it then heads for passes through it -- the reference's a > 0.1,
    # src/shaders.metal:63 -- so a few paths leave the room early; most run all 32767 + mirror bounces)
    assert st.rays >= 64 * 10000
    assert span_s > 0.3, span_s
    ref, rays = oracle_tile(Oracle.from_scene(s), u, e, 30, 30, 8, 1)
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref))
    assert st.rays == rays
    r.close()


def test_injected_fault_is_reported_by_the_call_that_caused_it(gpu):
    from mirror_maze import MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(10))
    u = default_uniform(256, 128, 0)
    e = make_ext(8, 8, 8)
    # 1. a clean call, then a faulting one, then mm_sync names the faulting call
    r.trace_tile(u, e, 0, 0, 256, 128)
    ok = r.last_call()
    r.set_option(23, 1)
    r.trace_tile(u, e, 0, 0, 256, 128)  # returns at once: the fault happens on the GPU
    bad = r.last_call()
    r.set_option(23, 0)
    assert bad == ok + 1
    with pytest.raises(MMError) as ei:
        r.sync()
    assert f"call #{bad} " in str(ei.value) and "injected fault" in str(ei.value)
    assert r.call_status(ok) is True
    r.sync()  # reported once: the context is clean again
    # 2. the next trace call reports a failed earlier call and is not enqueued
    r.set_option(23, 1)
    r.trace_tile(u, e, 0, 0, 256, 128)
    bad2 = r.last_call()
    r.set_option(23, 0)
    import torch

    torch.cuda.synchronize()  # let it finish (the status words need no mm_sync)
    with pytest.raises(MMError) as ei:
        r.trace_tile(u, e, 0, 0, 256, 128)
    assert f"call #{bad2} " in str(ei.value) and "not enqueued" in str(ei.value)
    assert r.last_call() == bad2  # the refused call got no number
    with pytest.raises(MMError):  # mm_call_status keeps naming it
        r.call_status(bad2)
    img, _ = r.trace_tile(u, e, 0, 0, 256, 128)
    r.sync()
    assert r.call_status(r.last_call()) is True and np.isfinite(img.cpu().numpy()).all()
    # 3. with stats the call syncs and reports its own fault directly
    r.set_option(23, 1)
    with pytest.raises(MMError) as ei:
        r.trace_tile(u, e, 0, 0, 256, 128, stats=True)
    assert f"call #{r.last_call()} " in str(ei.value)
    r.set_option(23, 0)
    r.close()


def test_pending_status_is_visible_without_waiting(gpu):
    """mm_call_status does not block: a long call reads as pending, then clean."""
    import time

    from mirror_maze import Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(32))
    u = default_uniform(1920, 1080, 0)
    r.trace_tile_frames(u, make_ext(8, 8, 8), 8, 0, 0, 1920, 1080)  # ~25 ms of GPU work
    c = r.last_call()
    first = r.call_status(c)
    t0 = time.time()
    while not r.call_status(c):
        assert time.time() - t0 < 30
        time.sleep(0.001)
    assert first is False  # seen running before it ended
    r.sync()
    r.close()


def test_ring_timeouts_are_reported_with_the_stuck_entry(gpu):
    """MM_OPT_FAULT_INJECT 2: every protocol wait gives up at its first failed
    poll.  The call fails by name, mm_last_error carries the launch's first
    timed-out wait (trace_kernels.hip ring_timeout: role, entry, wanted and
    seen turn values, the ring's counters), and a writer that gave up leaves
    NaN in its sample."""
    import re

    from mirror_maze import MMError, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = _scene(32)
    r = Renderer(0)
    r.set_option(21, 64)  # every path defers at bounce 1: the rings run full
    r.set_option(22, 0)
    r.upload_scene(s)
    u = default_uniform(256, 144, 0)
    e = make_ext(8, 8, 8, frame=0)
    r.set_option(23, 2)   # protocol waits give up at once
    got, _ = r.trace_tile(u, e, 0, 0, 256, 144)
    call = r.last_call()
    r.set_option(23, 0)
    try:
        r.sync()
        failed = False
    except MMError as ex:
        failed = True
        msg = str(ex)
        assert f"call #{call} " in msg and "tail ring wait timed out" in msg
        m = re.search(r"first timed-out wait \(launch \d+\): (reader|writer) of entry (\d+) \(slot (\d+), lap (\d+)\) "
                      r"in block \d+ wave (\d+) lane (\d+) wanted turn (\d+), saw (\d+); reserved (\d+), claimed (\d+)",
                      msg)
        assert m, msg
        role, seq, slot, lap, wave, lane, want, seen, res, cl = m.groups()
        seq, want, seen, res, cl = map(int, (seq, want, seen, res, cl))
        assert int(slot) == seq % 512 and int(lap) == seq // 512 and int(wave) < 16 and int(lane) < 64
        assert want == (2 * (seq // 512) + (1 if role == "reader" else 0)) and seen != want
        assert cl <= res and seq < res
    img = got.cpu().numpy()
    if not failed:  # no wait was ever needed: the image is exact
        ref, _ = oracle_tile(Oracle.from_scene(s), u, e, 0, 0, 256, 144)
        assert np.array_equal(_bits(img), _bits(ref))
    # the context works normally afterwards
    again, _ = r.trace_tile(u, e, 0, 0, 256, 144)
    r.sync()
    assert np.isfinite(again.cpu().numpy()).all()
    r.close()


def test_lone_wave_with_64_lane_deferral_terminates(gpu):
    """The round-3 livelock (tests/test_ring_model.py): one 64-path chunk in a
    closed room (every path survives its first bounce), deferral at 64 lanes.
    The wave parks its 64 paths at bounce 1; its 15 block-mates found the
    queue empty and have left; in round 3 it then claimed the 64 tails and
    re-parked them at the top of their first bounce, forever (the launch ended
    ~2^26 cycles later at the 32-bit counter wrap with a ring timeout).  Now a
    claimed chunk of <= defer_lanes tails runs with deferral off: the call
    ends in milliseconds, clean and bit-exact."""
    import time

    from mirror_maze import MM_INFO_LAST_DEFER, Renderer, default_uniform, make_ext
    from oracle.oracle import Oracle

    s = closed_room(40, 0.2, 3)
    r = Renderer(0)
    r.set_option(21, 64)
    r.set_option(22, 0)
    r.upload_scene(s)
    u = default_uniform(64, 64, 0)
    for i in range(3):
        u.cam.center[i] = 0.0
    e = make_ext(8, 8, 8, frame=0)
    for rep in range(3):
        t0 = time.time()
        got, st = r.trace_tile(u, e, 20 + rep, 30, 8, 1, stats=True)  # 64 paths: one chunk, one block
        r.sync()
        dt = time.time() - t0
        assert r.scene_info(MM_INFO_LAST_DEFER) == 1.0
        assert dt < 2.0, dt
        ref, rays = oracle_tile(Oracle.from_scene(s), u, e, 20 + rep, 30, 8, 1)
        assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref))
        assert st.rays == rays
    r.close()


def test_failed_enqueue_releases_its_status_slot(gpu):
    """a call that took a status slot and then failed to enqueue
    its launch (MM_OPT_FAULT_INJECT 3) must not leave the slot owned: the next
    1100 calls (more than the 1024 slots) run clean."""
    from mirror_maze import MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(10))
    u = default_uniform(64, 64, 0)
    e = make_ext(1, 1, 1)
    r.trace_tile(u, e, 0, 0, 8, 8)
    r.set_option(23, 3)
    with pytest.raises(MMError) as ei:
        r.trace_tile(u, e, 0, 0, 8, 8)
    assert "injected enqueue failure" in str(ei.value)
    r.set_option(23, 0)
    for i in range(1100):
        r.trace_tile(u, e, 0, 0, 8, 8)
    r.sync()
    assert r.call_status(r.last_call()) is True
    r.close()


def test_status_of_calls_older_than_the_failed_list_is_not_reported_clean(gpu):
    """mm_call_status keeps the last 64 failed calls; for an older
    call it no longer knows the outcome of, it says so instead of MM_OK."""
    from mirror_maze import MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(10))
    u = default_uniform(64, 64, 0)
    e = make_ext(8, 8, 8)
    r.trace_tile(u, e, 0, 0, 8, 8)
    clean = r.last_call()
    ids = []
    for i in range(70):  # a failed call is reported once (here by mm_sync), then the context runs on
        r.set_option(23, 1)
        r.trace_tile(u, e, 0, 0, 8, 8)
        ids.append(r.last_call())
        r.set_option(23, 0)
        with pytest.raises(MMError):
            r.sync()
    with pytest.raises(MMError) as ei:
        r.call_status(ids[0])  # dropped from the list of 64
    assert "no longer kept" in str(ei.value)
    with pytest.raises(MMError) as ei:
        r.call_status(ids[-1])  # still kept: its own failure
    assert "injected fault" in str(ei.value)
    with pytest.raises(MMError):
        r.call_status(clean)  # older than a dropped failure: unknown, not clean
    r.close()


def test_staging_bound_for_multi_frame_launches(gpu):
    """staged samples are bounded at 2^29 paths (6 GiB of 12-B records) per launch.
    A multi-frame launch over it runs with the fused resolve when it can
    (MM_INFO_LAST_DEFER 0, frames bit-identical to single-frame launches) and
    is refused otherwise; a single frame over it is split into row batches."""
    import torch

    from mirror_maze import MM_INFO_LAST_DEFER, MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.upload_scene(_scene(16))
    u = default_uniform(1920, 1080, 0)
    # 1920 x 1080 x 8 spp x 33 frames = 547 M staged paths > 2^29: fused resolve instead of the rings
    n = 33
    many, _ = r.trace_tile_frames(u, make_ext(8, 8, 8, frame=0), n, 0, 0, 1920, 1080)
    assert r.scene_info(MM_INFO_LAST_DEFER) == 0.0
    for f in (0, n - 1):
        one, _ = r.trace_tile(u, make_ext(8, 8, 8, frame=f), 0, 0, 1920, 1080)
        assert torch.equal(one.view(torch.int32), many[f].view(torch.int32)), f
    del many
    # 3 spp cannot fuse: 1920 x 1080 x 3 x 87 frames > 2^29 is refused before any launch
    with pytest.raises(MMError):
        r.trace_tile_frames(u, make_ext(3, 8, 8), 87, 0, 0, 1920, 1080)
    r.sync()
    r.close()


def test_auto_tail_deferral_policy(gpu):
    """MM_OPT_DEFER auto (mm_runtime.hip): the tail rings run for paths of >= 8
    bounces on launches of >= 2^24 paths where the maze grid sits whole in LDS
    -- C3's 20-frame launches and rank 0's rows of an 8-way split (41 M paths)
    -- and not on a single C3 frame (16.6 M paths), for 4-bounce paths (C2) or
    on the N=64 scene (leaf boxes via L1/L2); MM_OPT_DEFER 0 turns it off."""
    from mirror_maze import MM_INFO_LAST_DEFER, MM_INFO_LAST_LDS_MODE, Renderer, default_uniform, make_ext
    from mirror_maze.dist import row_shard

    u = default_uniform(1920, 1080, 0)
    r = Renderer(0)
    r.upload_scene(_scene(32))
    r.trace_tile(u, make_ext(8, 8, 8, frame=0), 0, 0, 1920, 1080)  # one frame: 16.6 M paths
    assert r.scene_info(MM_INFO_LAST_DEFER) == 0.0 and r.scene_info(MM_INFO_LAST_LDS_MODE) == 11.0
    y0, stride, rows = row_shard(1080, 8, 0)
    r.trace_tile_frames(u, make_ext(8, 8, 8, frame=0), 20, 0, y0, 1920, rows, y_stride=stride)  # 41 M paths
    assert r.scene_info(MM_INFO_LAST_DEFER) == 1.0
    r.trace_tile_frames(u, make_ext(8, 4, 4, frame=0), 2, 0, 0, 1920, 1080)  # 4-bounce paths
    assert r.scene_info(MM_INFO_LAST_DEFER) == 0.0
    r.set_option(21, 0)
    r.trace_tile_frames(u, make_ext(8, 8, 8, frame=0), 2, 0, 0, 1920, 1080)
    assert r.scene_info(MM_INFO_LAST_DEFER) == 0.0
    r.sync()
    r.close()
    r = Renderer(0)
    r.upload_scene(_scene(64))
    r.trace_tile_frames(u, make_ext(8, 16, 16, frame=0), 2, 0, 0, 1920, 1080)
    assert r.scene_info(MM_INFO_LAST_DEFER) == 0.0 and r.scene_info(MM_INFO_LAST_LDS_MODE) == 14.0
    r.sync()
    r.close()


def test_lost_ring_entry_ends_the_launch_quickly(gpu):
    """after one protocol wait times out, the slot's turn word
    never catches up, so every later wait of that slot would spin the whole
    bound (2^20 polls, ~50 ms) and time out in turn -- a launch of minutes.
    MM_OPT_FAULT_INJECT 4 loses the launch's first deferred path (its entry
    is reserved and never written) with the NORMAL spin bound: its reader
    times out once, every later wait sees the launch's error bit and gives
    up within 256 polls, and the call fails by name, with the lost entry's
    record, in well under a second of GPU time."""
    import re
    import time

    import torch

    from mirror_maze import MMError, Renderer, default_uniform, make_ext

    r = Renderer(0)
    r.set_option(21, 64)  # every path defers at bounce 1: the rings cycle many laps
    r.set_option(22, 0)
    r.upload_scene(_scene(32))
    u = default_uniform(512, 288, 0)
    e = make_ext(8, 8, 8, frame=0)
    r.set_option(23, 4)
    t0 = time.time()
    r.trace_tile(u, e, 0, 0, 512, 288)
    call = r.last_call()
    r.set_option(23, 0)
    with pytest.raises(MMError) as ei:
        r.sync()
    dt = time.time() - t0
    msg = str(ei.value)
    assert f"call #{call} " in msg and "lost tail-ring entry" in msg, msg
    assert "tail ring wait timed out" in msg and re.search(r"first timed-out wait \(launch \d+\): (reader|writer)", msg), msg
    assert dt < 5.0, dt
    # the record was consumed with its call; the context runs clean afterwards
    again, _ = r.trace_tile(u, e, 0, 0, 512, 288)
    r.sync()
    assert torch.isfinite(again).all()
    r.close()
