"""Write a scene in scripts/grid_sim.c's input format (n_rects, n_nodes as u32;
rects 48 B, nodes 32 B, idx u32, is_mirror u8, emission 16 B each).

    python scripts/dump_scene.py <maze_n> <out.bin>
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "mirror-maze_amd"))
from mirror_maze import Scene  # noqa: E402

s = Scene.build(int(sys.argv[1]), 0)
with open(sys.argv[2], "wb") as f:
    f.write(np.array([s.n_rects, s.n_nodes], np.uint32).tobytes())
    for a, dt in ((s.rects, None), (s.nodes, None), (s.idx, np.uint32), (s.is_mirror, np.uint8), (s.emission, np.float32)):
        arr = np.ascontiguousarray(a if dt is None else np.asarray(a).astype(dt))
        f.write(arr.tobytes())
print("wrote", sys.argv[2], s.n_rects, "rects", s.n_nodes, "nodes")
