"""Interactive camera and player collision: the product's
C++ restatement (mm_player_*, mm_check_collision, mm_quat_mult) against the
independent Python restatement in oracle/scene_oracle.py, bit for bit, plus
properties of the reference's behaviour.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest


@pytest.fixture(scope="module")
def scene():
    from mirror_maze import Scene

    return Scene.build(10, 0)


def _node_tuples(nodes):
    return [(tuple(n["mn"]), tuple(n["mx"]), int(n["left_first"]), int(n["count"])) for n in nodes]


def test_quat_mult_matches_oracle_and_rotates_view_axis():
    from mirror_maze import calculate_quaternion
    from mirror_maze.scene import quat_mult
    from oracle import scene_oracle as so

    q = calculate_quaternion((0.1, 0.0, 1.0))
    rng = np.random.default_rng(3)
    for v in rng.normal(size=(200, 3)).astype(np.float32):
        assert np.array_equal(quat_mult(v, q).view(np.uint32), so.quat_mult(v, q).view(np.uint32))
    # the rotation takes the default view axis (0,0,1) ~ to the camera direction (0.1,0,1)
    d = quat_mult((0, 0, 1), q)
    want = np.array([0.1, 0.0, 1.0]) / np.linalg.norm([0.1, 0.0, 1.0])
    assert np.allclose(np.abs(d), np.abs(want), atol=1e-5)


def test_check_collision_matches_oracle(scene):
    from mirror_maze import check_collision
    from oracle import scene_oracle as so

    nodes = _node_tuples(scene.nodes)
    rng = np.random.default_rng(7)
    hits = 0
    for c in rng.uniform(-50, 50, size=(400, 3)).astype(np.float32):
        c[1] = np.float32(rng.uniform(-8, 2))
        d = np.array([0.5, 0.2, 0.5], dtype=np.float32)
        got = check_collision(scene.nodes, c - d, c + d)
        want = so.check_collision(nodes, c - d, c + d)
        assert got == (-1 if want is None else want)
        hits += got >= 0
    assert 0 < hits < 400


def test_spawn_is_free_and_walls_stop_the_player(scene):
    from mirror_maze import Player
    from mirror_maze import check_collision
    from mirror_maze._lib import MM_PLAYER_COLLIDED

    p = Player(scene)
    c0 = p.center
    d = np.array([0.5, 0.2, 0.5], dtype=np.float32)
    assert check_collision(scene.nodes, c0 - d, c0 + d) == -1   # the reference starts here
    # walk forward until a wall stops the player; every blocked step leaves the centre unchanged
    blocked = 0
    for _ in range(600):
        before = p.center
        f = p.step(keys=[Player.KEY_W])
        if f & MM_PLAYER_COLLIDED:
            blocked += 1
            assert np.array_equal(before, p.center)
        else:
            assert check_collision(scene.nodes, p.center - d, p.center + d) == -1
    assert blocked > 0


def test_player_frames_match_oracle(scene):
    from mirror_maze import Player
    from oracle import scene_oracle as so

    nodes = _node_tuples(scene.nodes)
    p = Player(scene)
    c, q, h = p.center, p.quat, np.float32(np.arccos(np.float64(p.quat[3])))
    rng = np.random.default_rng(11)
    for f in range(300):
        keys = [k for k in (0, 1, 2, 13) if rng.random() < 0.4]
        rng.shuffle(keys)
        mouse = list(rng.normal(0, 40, size=rng.integers(0, 3)).astype(np.float32))
        flags = p.step(keys, mouse)
        c, q, h, collided, rotated = so.player_step(c, q, h, keys, mouse, nodes)
        assert np.array_equal(p.center.view(np.uint32), c.view(np.uint32)), f
        assert np.array_equal(p.quat.view(np.uint32), q.view(np.uint32)), f
        assert bool(flags & 1) == collided and bool(flags & 2) == rotated


def test_player_uniform_carries_camera(scene):
    from mirror_maze import Player, default_uniform

    p = Player(scene, 256, 192)
    p.step([Player.KEY_D], [25.0])
    u = p.uniform(time=3)
    ref = default_uniform(256, 192, 3)
    assert list(u.cam.center) == list(p.center) and list(u.cam.quat) == list(p.quat)
    assert u.view_w == ref.view_w and u.time == 3 and u.cam.focal == ref.cam.focal
