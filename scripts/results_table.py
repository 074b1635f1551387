#!/usr/bin/env python
"""Compose the per-configuration results table (GPU rate, CPU 1-core / all-core
rates, the executed VALU lane-ops fraction from the PMC record, and -- as
ratios, not fractions: they can pass 1 -- the reference-walk VALU model and
the SURVEY 8(d) HBM model) from bench.py JSON lines.

    python scripts/results_table.py gpurun_out/<tag>/*.json > profiles/r02/results_table.md
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
rows.sort(key=lambda d: (order.get(d["config"]["workload"][:2], 9), d["config"]["workload"],
                         d["config"]["parallelism"]))
print("| config | GPU (1 x MI355X) | ms/frame | CPU 1 core | CPU (usable cores), reference walk | CPU (usable cores), "
      "same algorithm | executed VALU lane-ops (PMC), fraction of peak |"
      " reference-walk VALU model / peak (ratio, not a measurement) | 136 B/ray HBM model / peak (ratio) |")
print("|---|---|---|---|---|---|---|---|---|")


def ratio(sub):
    """a model's count over the peak: model_ratio (round 6 on), frac in older lines"""
    v = sub.get("model_ratio", sub.get("frac"))
    return "—" if v is None else f"{v:.3f}"


for d in rows:
    c, r, cb = d["config"], d["roofline"], d.get("cpu_baseline") or {}
    sc = cb.get("single_core") or {}
    acc = f" (accumulated, {d['steps']} frames)" if c.get("temporal_accumulation") else ""
    par = "" if c["parallelism"] == "1 GPU" else f" [{c['parallelism']}]"
    cpu = f"{cb['value']} Mrays/s ({cb['cores']} cores)" if cb else "—"
    sa = cb.get("same_algorithm") or {}
    same = f"{sa['value']} Mrays/s ({sa['cores']} cores)" if sa else "—"
    ref = r.get("reference_equivalent", r)  # (round-2 lines: the headline was the model)
    hw = (f"{100 * r['frac']:.1f} % of {r['peak']} T" if r.get("frac") is not None and
          r.get("basis", "").startswith("executed") else
          "— (PMC record of other sources)" if r.get("stale") else "—")
    print(f"| {c['workload']}{acc}{par} | {d['value']:.0f} Mrays/s | {d['ms_per_step']:.3f} | "
          f"{sc.get('value', '—')} Mrays/s | {cpu} | {same} | {hw} | {ratio(ref)} | {ratio(r['model_hbm'])} |")
