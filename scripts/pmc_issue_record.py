"""Issue attribution of the dominant kernel: record the
rocprofv3 --pmc passes of `SETS=... scripts/pmc_bench.sh <tag>` (the issue
counter sets below) as profiles/pmc_<config>_issue.json with the product
source hash, and print where the SIMDs' VALU issue cycles go.

    python scripts/pmc_issue_record.py gpurun_out/<tag> c3 20

Counter units (rocprofiler-sdk counter_defs.yaml for gfx950): SQ_WAVE_CYCLES,
SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_* and SQ_ACTIVE_INST_VALU2 are
in quad-cycles (4 clocks); SQ_INSTS_* are instruction counts summed over the
SEs; GRBM_GUI_ACTIVE is clocks summed over the 8 XCDs.  A wave64 VALU
instruction occupies a SIMD-32 for 2 clocks, so one SIMD can issue at most 2
VALU instructions per quad-cycle -- SQ_ACTIVE_INST_VALU2 counts the quad-cycles
in which it issued two.
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
SIMDS = 256 * 4

# the passes (pass them to scripts/pmc_bench.sh as SETS, ';'-separated)
ISSUE_SETS = [
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES "
    "SQ_INSTS GRBM_GUI_ACTIVE",
    "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT "
    "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU",
    "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU "
    "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT",
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_WAVES "
    "SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE",
]


def counters(root: Path):
    """Per-dispatch mean of every counter over the dominant kernel's dispatches."""
    agg = collections.defaultdict(list)
    for f in sorted(root.glob("pmc*/pmc_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if PAT in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), v in per.items():
            agg[name].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def derive(m):
    cyc = m["GRBM_GUI_ACTIVE"] / 8            # kernel clocks (per XCD)
    quads = SIMDS * cyc / 4                   # SIMD quad-cycles in the kernel
    valu, valu2 = m["SQ_INSTS_VALU"], m.get("SQ_ACTIVE_INST_VALU2")
    d = {"kernel_clocks": cyc, "simd_quad_cycles": quads,
         "valu_issue_share": valu / (2 * quads)}
    if valu2 is not None:
        one = valu - 2 * valu2                # quad-cycles with exactly one VALU issued
        d.update({"quads_two_valu": valu2 / quads, "quads_one_valu": one / quads,
                  "quads_no_valu": 1 - (valu2 + one) / quads,
                  "dual_issue_fraction_of_valu": 2 * valu2 / valu})
    for k in ("SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM", "SQ_INSTS_LDS"):
        if k in m:
            d[k.lower().replace("sq_insts_", "") + "_per_valu"] = m[k] / valu
    if "SQ_INSTS" in m:
        d["all_insts_per_simd_quad"] = m["SQ_INSTS"] / quads
    mix = {k: m[k] for k in m if k.startswith("SQ_INSTS_VALU_")}
    if mix:
        d["valu_mix_fraction"] = {k.replace("SQ_INSTS_VALU_", ""): v / valu for k, v in mix.items()}
        d["valu_mix_unclassified"] = 1 - sum(mix.values()) / valu
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        d["wave_time"] = {k: m[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC") if k in m}
    if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
        d["lane_utilisation"] = m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])
    return d


def main():
    root, cfg = Path(sys.argv[1]), sys.argv[2]
    frames = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    m = counters(root)
    from bench import src_hash

    head = subprocess.run(["git", "-C", str(REPO), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    rec = {"config": cfg, "kernel_pattern": PAT, "source": root.name, "src_hash": src_hash(), "git_head": head,
           "frames_per_launch": frames, "sets": ISSUE_SETS, "derived": derive(m), "counters": m}
    out = REPO / "profiles" / f"pmc_{cfg}_issue.json"
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec["derived"], indent=1))


if __name__ == "__main__":
    main()
