"""Per-kernel summary of rocprofv3 --pmc passes (scripts/pmc_wavefront.sh):
for every kernel name matching a pattern, the summed counters over its
dispatches, the summed duration (kernel trace of the same passes) and derived
metrics (HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE per the gfx950 correction,
achieved GB/s, lane utilisation, VALU issue share).

    python scripts/pmc_kernels.py gpurun_out/<tag> [pattern]
"""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "k_wf_"


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mm::", "")


cnt = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(list)
for f in sorted(root.glob("pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
for f in sorted(root.glob("stats/run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
passes = len(list(root.glob("pmc*/pmc_counter_collection.csv")))
print(f"# {root.name}: kernels ~ '{pat}'; counters summed over the dispatches of one PMC pass "
      f"(each pass replays the same 2 timed frames + 1 warm frame); durations from the --stats run")
for k in sorted(cnt):
    m = cnt[k]
    t = sum(dur.get(k, [])) / 1e3
    hbm = 2 * m.get("FETCH_SIZE", 0) * 1024 + m.get("WRITE_SIZE", 0) * 1024
    line = [f"{k:34s}", f"dispatches {len(dur.get(k, []))}", f"time {t * 1e3:9.3f} ms"]
    if hbm:
        line.append(f"HBM {hbm / 1e9:7.3f} GB -> {hbm / t / 1e9 if t else 0:7.1f} GB/s")
    if m.get("SQ_ACTIVE_INST_VALU"):
        line.append(f"lane util {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
    if m.get("GRBM_GUI_ACTIVE") and m.get("SQ_INSTS_VALU"):
        line.append(f"VALU issue {m['SQ_INSTS_VALU'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8 / 2):.3f}")
    if m.get("SQ_WAIT_ANY") and m.get("SQ_WAVE_CYCLES"):
        line.append(f"wait {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    print("  ".join(line))
    for c in sorted(m):
        print(f"    {c:26s} {m[c]:.6g}")
