"""bench.py host logic that needs no GPU: how timed frames are grouped into
multi-frame launches (mm_trace_tile_frames)."""
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
