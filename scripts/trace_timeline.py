"""Timeline of the last N kernel dispatches of a rocprofv3 kernel trace (ms from the first shown).
    python scripts/trace_timeline.py <run_kernel_trace.csv> [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} dur {(e - s) / 1e6:8.3f} gap {(s - prev) / 1e6:7.3f}  "
          f"{r['Kernel_Name'][:60]}")
    prev = e
