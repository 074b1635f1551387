"""Host scene builder (C++) vs the independent Python restatement, plus the
structural invariants of the maze and the SAH BVH."""
from __future__ import annotations

import numpy as np
import pytest


def _build(n, seed=0):
    from mirror_maze import Scene

    return Scene.build(n, seed)


@pytest.mark.parametrize("n,seed", [(10, 0), (4, 0), (16, 0), (10, 3)])
def test_planes_match_python_restatement(n, seed):
    from oracle import scene_oracle as so

    s = _build(n, seed)
    rects, mats, emis, grid = so.build_planes(n, seed)
    assert np.array_equal(s.grid, grid)
    assert s.rects.shape == rects.shape
    assert np.array_equal(s.rects.view(np.uint32), rects.view(np.uint32))  # bit-exact
    assert np.array_equal(s.is_mirror, mats)
    assert np.array_equal(s.emission.view(np.uint32), emis.view(np.uint32))


@pytest.mark.parametrize("n", [4, 10, 16])
def test_bvh_matches_python_restatement(n):
    from oracle import scene_oracle as so

    s = _build(n)
    nodes, idx = so.build_bvh(s.rects)
    assert list(s.idx) == idx
    assert s.n_nodes == len(nodes)
    for k, (mn, mx, lf, cnt) in enumerate(nodes):
        got = s.nodes[k]
        assert np.array_equal(got["mn"].view(np.uint32), np.array(mn, np.float32).view(np.uint32)), k
        assert np.array_equal(got["mx"].view(np.uint32), np.array(mx, np.float32).view(np.uint32)), k
        assert (int(got["left_first"]), int(got["count"])) == (lf, cnt), k


@pytest.mark.parametrize("n", [10, 32])
def test_maze_is_spanning_tree(n):
    s = _build(n)
    g = s.grid.astype(int)
    # passages counted once: 'up' (1) and 'left' (4) bits
    passages = int(((g & 1) != 0).sum() + ((g & 4) != 0).sum())
    assert passages == n * n - 1
    # symmetric bits
    assert np.all(((g[1:] & 1) != 0) == ((g[:-1] & 2) != 0))
    assert np.all(((g[:, 1:] & 4) != 0) == ((g[:, :-1] & 8) != 0))
    # connected: flood fill from (0,0)
    seen = np.zeros_like(g, bool)
    stack = [(0, 0)]
    while stack:
        y, x = stack.pop()
        if seen[y, x]:
            continue
        seen[y, x] = True
        if g[y, x] & 1: stack.append((y - 1, x))
        if g[y, x] & 2: stack.append((y + 1, x))
        if g[y, x] & 4: stack.append((y, x - 1))
        if g[y, x] & 8: stack.append((y, x + 1))
    assert seen.all()


@pytest.mark.parametrize("n", [10, 32])
def test_bvh_invariants(n):
    s = _build(n)
    nodes, idx, rects = s.nodes, s.idx, s.rects
    assert sorted(idx.tolist()) == list(range(s.n_rects))
    covered = np.zeros(s.n_rects, int)
    depth = 0
    stack = [(0, 0)]
    while stack:
        k, d = stack.pop()
        depth = max(depth, d)
        nd = nodes[k]
        lf, cnt = int(nd["left_first"]), int(nd["count"])
        if cnt > 0:
            for i in range(lf, lf + cnt):
                covered[idx[i]] += 1
                r = rects[idx[i]]
                o, u, v = r[0:3], r[6:9], r[3:6]
                for p in (o, o + u, o + v):
                    assert np.all(p >= nd["mn"]) and np.all(p <= nd["mx"])
        else:
            for c in (lf, lf + 1):
                assert np.all(nodes[c]["mn"] >= nd["mn"]) and np.all(nodes[c]["mx"] <= nd["mx"])
                stack.append((c, d + 1))
    assert np.all(covered == 1)
    assert depth == s.bvh_depth <= 50


def test_reference_scene_shape():
    """N=10, seed 0: the 7 fixed planes close the box; walls are axis aligned."""
    s = _build(10)
    r = s.rects
    # last 7 planes: 4 boundary walls, floor, spawn light, roof (src/main.rs:517-585)
    assert np.allclose(r[-7, 0:3], [-50, 2, -50]) and np.allclose(r[-3, 9:12], [0.4, 0.45, 0.3])
    assert np.allclose(r[-2, 0:3], [-5, 2, -49.9]) and np.allclose(s.emission[-1], [1, 0.8, 0.3, 0.02])
    v, u = r[:, 3:6], r[:, 6:9]
    for vec in (v, u):
        nz = (vec != 0).sum(axis=1)
        assert np.all(nz <= 1)  # axis aligned or zero-length (main.rs:416, 437)
    # light panels are matte emitters of strength 2 (main.rs:479, 513)
    lights = s.emission[:, 3] == 2.0
    assert np.all(s.is_mirror[lights] == 0)


def test_boundary_scales_with_maze_size():
    s = _build(32)
    r = s.rects
    assert np.allclose(r[-7, 0:3], [-160, 2, -160]) and np.allclose(r[-7, 6:9], [320, 0, 0])
    assert np.allclose(r[-1, 0:3], [-160, -8, 160])


def test_quaternion_cpp_vs_python():
    from mirror_maze import calculate_quaternion, default_uniform
    from oracle import scene_oracle as so

    for d in [(0.1, 0.0, 1.0), (0.3, 0.0, 1.0), (-0.7, 0.0, 0.2)]:
        assert np.array_equal(calculate_quaternion(d).view(np.uint32), so.calculate_quaternion(d).view(np.uint32))
    u = default_uniform(1024, 768, 3)
    assert list(u.cam.center) == [-5.0, 0.0, -45.0] and u.cam.focal == 1.0
    assert np.float32(u.cam.viewport[0]) == np.float32(2.0) * (np.float32(1024) / np.float32(768))
    assert u.chunk_w == 4 and u.time == 3
    q = np.array(u.cam.quat, np.float32)
    assert abs(float(np.dot(q, q)) - 1.0) < 1e-6 and q[0] == 0 and q[2] == 0


def test_chunk_scheduler_pops_and_refills():
    from mirror_maze import ChunkScheduler

    cs = ChunkScheduler(1024, 768, 4, seed=1)
    assert cs.total == 256 * 192
    seen = np.concatenate([cs.next(768) for _ in range(64)])  # exactly one full cycle
    assert len({(int(a), int(b)) for a, b in seen}) == 256 * 192
    assert seen[:, 0].max() == 1020 and seen[:, 1].max() == 764 and np.all(seen % 4 == 0)
    again = cs.next(768)  # refill from the original shuffled list: same order as cycle 1
    assert np.array_equal(again, seen[:768])


def _same_tree(a, b):
    (na, ia), (nb, ib) = a, b
    assert len(na) == len(nb)
    assert np.array_equal(ia, ib)
    assert np.array_equal(na.view(np.uint8), nb.view(np.uint8))  # every bit of every node


@pytest.mark.parametrize("n", [4, 10, 32, 64])
def test_bvh_sweep_equals_exhaustive_maze(n):
    """The O(n log n) sweep split search builds the reference's tree bit for bit
    (the exhaustive form is the reference's loop, src/main.rs:110-125, 180-211)."""
    from mirror_maze import Scene
    from mirror_maze._lib import MM_BVH_EXHAUSTIVE, MM_BVH_SWEEP

    s = _build(n)
    sweep = Scene.bvh(s.rects, MM_BVH_SWEEP)
    _same_tree(sweep, (s.nodes, s.idx))
    _same_tree(sweep, Scene.bvh(s.rects, MM_BVH_EXHAUSTIVE))


@pytest.mark.parametrize("seed", range(6))
def test_bvh_sweep_equals_exhaustive_adversarial(seed):
    """Ties everywhere: coordinates on a coarse grid (equal centers and equal
    costs), zero-length rects, signed zeros, huge and tiny extents."""
    from mirror_maze import Scene
    from mirror_maze._lib import MM_BVH_EXHAUSTIVE, MM_BVH_SWEEP

    rng = np.random.default_rng(seed)
    P = int(rng.integers(2, 300))
    r = rng.integers(-4, 5, size=(P, 12)).astype(np.float32) * np.float32(2.5)
    r[rng.random(P) < 0.2, 3:6] = 0.0                       # zero-length v
    r[rng.random((P, 12)) < 0.05] = -0.0                    # signed zeros
    if seed % 2:
        r[rng.random(P) < 0.1, 0] = np.float32(3e20)        # far outliers
        r[rng.random(P) < 0.1, 6:9] *= np.float32(1e-6)     # tiny extents
    _same_tree(Scene.bvh(r, MM_BVH_SWEEP), Scene.bvh(r, MM_BVH_EXHAUSTIVE))
