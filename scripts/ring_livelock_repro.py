"""One 64-path launch with 64-lane tail deferral in a closed room (every path
survives its first bounce), timed: the lone-wave case of the tail-ring model
(tests/test_ring_model.py, test_gpu_errors.py
test_lone_wave_with_64_lane_deferral_terminates).  Run it against a library
built from the round-3 sources (MIRROR_MAZE_LIB=...) to see the livelock end
at the 32-bit entry counters' wrap, and against the current library to see it
finish in milliseconds.  Prints a heartbeat while the call runs and one JSON
line at the end (also written to the path given as argv[1])."""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "mirror-maze_amd", REPO / "tests"):
    sys.path.insert(0, str(p))


def main() -> int:
    from mirror_maze import MMError, Renderer, default_uniform, make_ext
    from mirror_maze._lib import LIB_PATH
    from test_gpu_errors import closed_room

    out = Path(sys.argv[1]) if len(sys.argv) > 1 else None
    s = closed_room(40, 0.2, 3)
    r = Renderer(0)
    r.set_option(21, 64)
    r.set_option(22, 0)
    r.upload_scene(s)
    u = default_uniform(64, 64, 0)
    for i in range(3):
        u.cam.center[i] = 0.0
    e = make_ext(8, 8, 8, frame=0)
    done = threading.Event()
    t0 = time.time()

    def beat():
        while not done.wait(15.0):
            print(f"  ... call running for {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    rec = {"lib": str(LIB_PATH), "paths": 64}
    try:
        r.trace_tile(u, e, 20, 30, 8, 1)
        r.sync()
        rec["result"] = "ok"
    except MMError as ex:
        rec["result"] = str(ex)
    rec["seconds"] = round(time.time() - t0, 3)
    done.set()
    r.close()
    line = json.dumps(rec)
    print(line, flush=True)
    if out:
        out.parent.mkdir(parents=True, exist_ok=True)
        out.write_text(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
