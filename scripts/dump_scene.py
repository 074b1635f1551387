"""Write a scene in scripts/grid_sim.c's input format (n_rects, n_nodes as u32;
rects 48 B, nodes 32 B, idx u32, is_mirror u8, emission 16 B each).  With a
view size, also the default uniform (mm_uniform_default, 56 B) as <out.bin>.uni
(scripts/stage_model.c reads it).

    python scripts/dump_scene.py <maze_n> <out.bin> [W H]
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
if len(sys.argv) > 4:
    import ctypes

    from mirror_maze import default_uniform

    u = default_uniform(float(sys.argv[3]), float(sys.argv[4]), 0)
    Path(sys.argv[2] + ".uni").write_bytes(ctypes.string_at(ctypes.addressof(u), ctypes.sizeof(u)))
print("wrote", sys.argv[2], s.n_rects, "rects", s.n_nodes, "nodes")
