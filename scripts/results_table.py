#!/usr/bin/env python
"""Compose the BASELINE.md results table (GPU rate, CPU 1-core / all-core
rates, HBM and VALU roofline fractions per config) from bench.py JSON lines.

    python scripts/results_table.py gpurun_out/<tag>/*.json > profiles/r01_results_table.md
"""
import json
import sys

rows = []
for f in sys.argv[1:]:
    for line in open(f):
        line = line.strip()
        if line.startswith("{"):
            rows.append(json.loads(line))
order = {"C1": 1, "C2": 2, "C3": 3, "C4": 4, "C5": 5}
rows.sort(key=lambda d: (order.get(d["config"]["workload"][:2], 9), d["config"]["workload"]))
print("| config | GPU (1 x MI355X) | ms/frame | CPU 1 core | CPU all cores | HBM % (136 B/ray model) | VALU % (25/AABB + 71/rect) |")
print("|---|---|---|---|---|---|---|")
for d in rows:
    c, r, cb = d["config"], d["roofline"], d.get("cpu_baseline") or {}
    sc = cb.get("single_core") or {}
    acc = " (120-frame accumulation)" if c.get("temporal_accumulation") and d["steps"] >= 120 else (
        " (accumulated)" if c.get("temporal_accumulation") else "")
    print(f"| {c['workload']}{acc} | {d['value']:.0f} Mrays/s | {d['ms_per_step']:.3f} | "
          f"{sc.get('value', '—')} Mrays/s | {cb.get('value', '—')} Mrays/s ({cb.get('cores', '—')} threads of "
          f"{cb.get('host_cpus', '—')}) | {100 * r['frac']:.1f} | {100 * r['valu']['frac']:.1f} |")
