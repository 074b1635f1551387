"""One A/B runner for the GPU box (replaces the round-3 one-off ab_run*.sh,
ab_libs.sh, ab_multi*.sh, ab_defer_sweep.sh and prof_libs.sh drivers).

Times builds of the library (MIRROR_MAZE_LIB, built by scripts/build_variant.sh)
and/or runtime variants (scripts/ab_bench.py VARIANTS) on one or more
configurations, interleaved over repetitions so that clock drift hits every
arm alike.  Each arm is one scripts/ab_bench.py process under its own time
limit; every line carries the frames' checksum, and the runner fails if two
arms of one configuration disagree (the variants must be bit-identical).

    python scripts/ab.py --tag T --config c3:20:3 --config c4:2:2 \\
        --lib exp/base/lib.so --lib exp/new/lib.so [--variants default defer40] [--ranks 8]
    python scripts/ab.py --tag T --config c3:5:1 --lib exp/a/lib.so --rocprof
      (--rocprof: one rocprofv3 --kernel-trace --stats run per arm instead of timing reps)

Output: gpurun_out/<tag>/ab.txt (one line per arm and repetition) and a
summary of the median trace ms/frame per arm on stdout.
"""
from __future__ import annotations

import argparse
import os
import re
import statistics
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
LINE = re.compile(r"^(\S+)\s+rep \d+ trace\s+([\d.]+) ms/frame\s+wall\s+([\d.]+) ms/frame.*ck ([0-9a-f]+)")


def run_arm(lib, cfg, frames, ranks, variants, timeout, rocprof_dir=None):
    env = dict(os.environ)
    if lib:
        env["MIRROR_MAZE_LIB"] = str((REPO / lib).resolve())
    cmd = [sys.executable, str(REPO / "scripts" / "ab_bench.py"), "--config", cfg, "--frames", str(frames),
           "--reps", "1", "--ranks", str(ranks), *variants]
    if rocprof_dir:
        env["TMPDIR"] = "/tmp"
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-f", "csv", "-d", str(rocprof_dir), "-o", "run", "--"] + \
              ["python3"] + cmd[1:]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd="/tmp")
    if p.returncode != 0:
        raise SystemExit(f"arm failed ({lib or 'in-tree'} {cfg}): rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}")
    return [l for l in p.stdout.splitlines() if LINE.match(l)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", action="append", required=True, help="name:frames:reps, e.g. c3:20:3")
    ap.add_argument("--lib", action="append", default=[], help="library build (repeatable); none = in-tree")
    ap.add_argument("--variants", nargs="+", default=["default"])
    ap.add_argument("--ranks", type=int, default=1, help="trace rank 0's rows of an N-way split")
    ap.add_argument("--timeout", type=int, default=300, help="seconds per arm")
    ap.add_argument("--rocprof", action="store_true")
    a = ap.parse_args()
    out = REPO / "gpurun_out" / a.tag
    out.mkdir(parents=True, exist_ok=True)
    libs = a.lib or [None]
    times: dict[tuple, list] = {}
    checks: dict[tuple, set] = {}
    with open(out / "ab.txt", "a") as log:
        for spec in a.config:
            cfg, frames, reps = (spec.split(":") + ["5", "1"])[:3]
            for rep in range(int(reps)):
                for lib in libs:
                    name = Path(lib).parent.name if lib else "in-tree"
                    rp = out / f"{cfg}_{name}_rocprof" if a.rocprof else None
                    for line in run_arm(lib, cfg, int(frames), a.ranks, a.variants, a.timeout, rp):
                        m = LINE.match(line)
                        var, trace, wall, ck = m.group(1), float(m.group(2)), float(m.group(3)), m.group(4)
                        times.setdefault((cfg, name, var), []).append((trace, wall))
                        checks.setdefault((cfg, frames), set()).add(ck)
                        text = f"{cfg} r{a.ranks} {name:12s} {line}"
                        print(text, flush=True)
                        log.write(text + "\n")
                if a.rocprof:
                    break
    print("# median trace / wall ms per frame")
    for (cfg, name, var), v in sorted(times.items()):
        print(f"{cfg:5s} {name:12s} {var:14s} {statistics.median(t for t, _ in v):8.3f} "
              f"{statistics.median(w for _, w in v):8.3f}  (n={len(v)})")
    bad = {k: s for k, s in checks.items() if len(s) > 1}
    if bad:
        print(f"CHECKSUM MISMATCH: {bad}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
