"""bench.py host logic that needs no GPU: how timed frames are grouped into
multi-frame launches (mm_trace_tile_frames), and which PMC record a bench line
may quote (the one of its own sources and launch shape)."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


@pytest.mark.parametrize("count,per,expect", [
    (10, 8, [5, 5]), (16, 8, [8, 8]), (17, 8, [5, 6, 6]), (3, 8, [3]), (1, 8, [1]), (0, 8, []), (9, 1, [1] * 9),
])
def test_launch_sizes(count, per, expect):
    from bench import launch_sizes

    sizes = launch_sizes(count, per)
    assert sizes == expect
    assert sum(sizes) == count and all(0 < s <= per for s in sizes)
    assert max(sizes, default=0) - min(sizes, default=0) <= 1


def _args(config="c3", emulate_ranks=0):
    from types import SimpleNamespace

    return SimpleNamespace(config=config, emulate_ranks=emulate_ranks, pipeline="auto", opt=[])


def test_pmc_record_of_the_same_sources_is_used(monkeypatch):
    """profiles/pmc_<config>.json counts only for the sources it was taken on;
    its lane-ops and HBM bytes scale to the run's frames per launch."""
    import json

    import bench

    rec = json.loads((bench.REPO / "profiles" / "pmc_c3.json").read_text())
    monkeypatch.setattr(bench, "src_hash", lambda: rec["src_hash"])
    m, traffic = bench.pmc_profile(_args(), rec["frames_per_launch"] * 2, 0.1, 1)
    assert m["source"] == "profiles/pmc_c3.json" and not m.get("stale")
    assert traffic == round(rec["hbm_bytes_per_launch"] * 2)
    assert m["valu_lane_ops_tops"] == round(rec["valu_lane_ops_per_launch"] * 2 / 0.1 / 1e12, 3)


def test_pmc_record_of_other_sources_is_marked_stale(monkeypatch):
    import bench

    monkeypatch.setattr(bench, "src_hash", lambda: "0" * 16)
    m, traffic = bench.pmc_profile(_args(), 20, 0.05, 1)
    assert m["stale"] is True and traffic is None and "stale_valu_lane_ops_tops" in m


def test_pmc_record_per_emulated_rank_share(monkeypatch):
    """--emulate-ranks N reads pmc_<config>_r<N>.json (rank 0's own launch
    shape), not the whole frame's record; without one there is no record."""
    import json

    import bench

    rec = json.loads((bench.REPO / "profiles" / "pmc_c3_r8.json").read_text())
    monkeypatch.setattr(bench, "src_hash", lambda: rec["src_hash"])
    m, _ = bench.pmc_profile(_args(emulate_ranks=8), 20, 0.0065, 1)
    assert m["source"] == "profiles/pmc_c3_r8.json"
    m, traffic = bench.pmc_profile(_args(emulate_ranks=4), 20, 0.013, 1)
    assert m["source"] is None and traffic is None
    m, _ = bench.pmc_profile(_args(), 20, 0.05, 8)  # N > 1 ranks: no single-GPU record applies
    assert m["source"] is None
