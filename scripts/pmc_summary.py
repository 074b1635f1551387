"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh output) for one kernel.

    python scripts/pmc_summary.py gpurun_out/<tag> [kernel-substring [traffic.json [frames-per-launch]]] > profiles/<name>.txt
Per-dispatch means of every counter, plus derived metrics:
  lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  VALU issue share = SQ_INSTS_VALU / (SIMDs * cycles / 2)   (wave64 VALU = 2 cycles on SIMD32)
  HBM bytes = 2 * FETCH_SIZE (gfx950 half-count correction, MI355X_MICROARCH.md) + WRITE_SIZE
"""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "k_trace"
agg = collections.defaultdict(list)
for f in sorted(root.glob("pmc*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, name), v in per.items():
        agg[name].append(v)
m = {k: sum(v) / len(v) for k, v in agg.items()}
print(f"# {root.name}: kernel ~ '{pat}', per-dispatch means over {max(len(v) for v in agg.values())} dispatches")
for k in sorted(m):
    print(f"{k:28s} {m[k]:.6g}")
if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
    print(f"lane utilisation (VALU)      {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
if "GRBM_GUI_ACTIVE" in m and "SQ_INSTS_VALU" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
    print(f"kernel cycles (per XCD)      {cyc:.6g}")
    print(f"VALU issue share             {m['SQ_INSTS_VALU'] / (1024 * cyc / 2):.3f}")
if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
    print(f"wave time waiting (s_waitcnt) {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
if "FETCH_SIZE" in m:
    print(f"HBM fetch bytes (x2 corr.)   {2 * m['FETCH_SIZE'] * 1024:.6g}")
if "WRITE_SIZE" in m:
    print(f"HBM write bytes              {m['WRITE_SIZE'] * 1024:.6g}")
if len(sys.argv) > 3 and "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    # bench.py reads this as roofline.traffic (HBM bytes per launch of the dominant kernel)
    import json
    frames = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0  # frames per profiled launch
    per_launch = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
    rec = {"kernel_pattern": pat, "source": root.name,
           "fetch_bytes_corrected": 2 * m["FETCH_SIZE"] * 1024, "write_bytes": m["WRITE_SIZE"] * 1024,
           "hbm_bytes_per_launch": per_launch, "frames_per_launch": frames,
           "hbm_bytes_per_frame": per_launch / frames,
           "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, per-dispatch mean"}
    Path(sys.argv[3]).write_text(json.dumps(rec, indent=1) + "\n")
