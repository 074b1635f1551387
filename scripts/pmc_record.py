"""Record the PMC passes of scripts/pmc_bench.sh as profiles/pmc_<config>.json,
the file bench.py reads its measured roofline fields from.  Run HERE (in the
build container) right after the gpurun call, on the same tree: the record
carries the product source hash (bench.src_hash) and the git HEAD, and
bench.py ignores a record whose hash is not its own tree's.

    python scripts/pmc_record.py gpurun_out/<tag> <config> [frames_per_launch]
Per-dispatch means of the dominant kernel (k_trace_wavepersist, non-stats
instantiation) and the derived metrics:
  HBM bytes           = 2 x FETCH_SIZE (gfx950 half-count correction, MI355X_MICROARCH.md) + WRITE_SIZE
  lane utilisation    = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)
  VALU issue share    = SQ_INSTS_VALU / (1024 SIMDs x kernel cycles / 2)   (a wave64 VALU op takes 2 cycles)
  VALU lane-ops       = SQ_INSTS_VALU x 64 x lane utilisation
"""
from __future__ import annotations

import collections
import csv
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

PAT = "k_trace_wavepersist<false"


def main():
    root, cfg = Path(sys.argv[1]), sys.argv[2]
    frames = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
    agg = collections.defaultdict(list)
    for f in sorted(root.glob("pmc*/pmc_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if PAT in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), v in per.items():
            agg[name].append(v)
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    durs = []
    for f in sorted(root.glob("stats/run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if PAT in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    from bench import src_hash

    head = subprocess.run(["git", "-C", str(REPO), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    dirty = subprocess.run(["git", "-C", str(REPO), "status", "--porcelain", "--", "mirror-maze_amd/csrc",
                            "mirror-maze_amd/Makefile", "include"], capture_output=True, text=True).stdout.strip()
    cyc = m["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
    lane = m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])
    rec = {
        "config": cfg, "kernel_pattern": PAT, "source": root.name, "src_hash": src_hash(),
        "git_head": head + ("+uncommitted" if dirty else ""), "frames_per_launch": frames,
        "kernel_avg_ms": round(sum(durs) / len(durs), 4) if durs else None,
        "kernel_ms_each": [round(d, 4) for d in durs],
        "fetch_bytes_corrected": 2 * m["FETCH_SIZE"] * 1024, "write_bytes": m["WRITE_SIZE"] * 1024,
        "hbm_bytes_per_launch": 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024,
        "lane_utilisation": round(lane, 4),
        "valu_issue_share": round(m["SQ_INSTS_VALU"] / (1024 * cyc / 2), 4),
        "valu_lane_ops_per_launch": m["SQ_INSTS_VALU"] * 64 * lane,
        "wait_share": round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 4),
        "kernel_cycles_per_xcd": cyc,
        "counters": {k: m[k] for k in sorted(m)},
    }
    out = REPO / "profiles" / f"pmc_{cfg}.json"
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: v for k, v in rec.items() if k != "counters"}, indent=1))


if __name__ == "__main__":
    main()
