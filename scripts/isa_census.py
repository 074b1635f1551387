#!/usr/bin/env python3
"""ISA census of one kernel in a gfx950 assembly file (hipcc --save-temps).

    python scripts/isa_census.py trace_kernels-hip-amdgcn-amd-amdhsa-gfx950.s \
        [--kernel 'k_trace_wavepersistILb0ELi11ELi17ELi2E'] [--loops] [--diff other.s]

Prints the kernel's resource metadata (VGPRs, SGPRs, scratch bytes, spill
counts) and its instructions by class.  With --loops, every natural loop
(a backward branch to a label) with its body's instruction classes, nested
loops indented, so the hot loop bodies (the grid search's rect test and cell
step, the rejection-sampling trials) can be read off: VALU, SALU, exec-mask
and branch instructions, s_waitcnt, readfirstlane, LDS, VMEM, scratch.
"""
from __future__ import annotations

import argparse
import collections
import re
import sys

CLASSES = [
    ("scratch", re.compile(r"^(scratch_|buffer_(load|store)_\w+.*\boffen\b.*\bs\[0:3\])")),
    ("waitcnt", re.compile(r"^s_waitcnt")),
    ("branch", re.compile(r"^s_(cbranch|branch|setpc|swappc|getpc)")),
    ("exec", re.compile(r"^s_\w+.*\bexec\b|^s_(and|or|andn2|xor)_saveexec")),
    ("smem", re.compile(r"^s_(load|buffer_load|memtime|memrealtime)")),
    ("sleep/nop", re.compile(r"^s_(sleep|nop|setprio|barrier|endpgm|trap)")),
    ("salu", re.compile(r"^s_")),
    ("readlane", re.compile(r"^v_(readfirstlane|readlane|writelane)")),
    ("v_cmp", re.compile(r"^v_cmpx?_")),
    ("v_cndmask", re.compile(r"^v_cndmask")),
    ("valu", re.compile(r"^v_")),
    ("lds", re.compile(r"^ds_")),
    ("vmem", re.compile(r"^(global_|buffer_|flat_)")),
]


def classify(ins: str) -> str:
    for name, rx in CLASSES:
        if rx.search(ins):
            return name
    return "other"


# Dual issue (scripts/isa_dual.hip, profiles/r05/isa_dual_r5c.txt): a SIMD-32 issues two wave64 VALU ops in a
# quad-cycle only if at most one is "single-slot".  Pairable ("D") forms measured: v_add/sub/mul/fma/fmac_f32
# (VGPR operands, literal or neg modifier allowed), v_add_u32 (VGPR, inline constant or literal; x + x),
# v_and/v_or/v_xor (literal allowed), v_lshrrev_b32 (by a VGPR or a constant), v_mov_b32.  Single-slot
# ("S"): every form with an SGPR or VCC operand (v_cmp*, v_cndmask*, readlane, carry-out adds), v_cvt*,
# three-source VOP3 (v_lshl_add, v_bfe, v_min3, v_max3_u32, v_or3), v_min/v_max, v_mul_lo, v_mul_u32_u24,
# v_lshlrev_b32 (by a constant or a VGPR), 64-bit ops; transcendentals take two quads
# (profiles/r05/isa_dual_r5c.txt, isa_dual_r5g.txt).
D_FORMS = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac)_f32|^v_(add|sub|subrev)_u32|^v_(and|or|xor)_b32|"
                     r"^v_mov_b32|^v_lshrrev_b32|^v_ashrrev_i32")
TRANS = re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_")


def slot(ins: str):
    """'D', 'S' or 'T' (transcendental) for a VALU op, None otherwise."""
    if not ins.startswith("v_"):
        return None
    if TRANS.search(ins):
        return "T"
    op, _, args = ins.partition(" ")
    sgpr = re.search(r"\b(s\d+|s\[|vcc|exec|ttmp)", args)
    if D_FORMS.search(op) and not sgpr and not op.endswith("_e64") or \
            (D_FORMS.search(op) and op.endswith("_e64") and not sgpr and "v_add_co" not in op):
        if op.startswith("v_ashrrev_i32") and re.match(r"\s*v\d+,\s*(-?\d+|0x)", args):
            return "S"  # (not measured; v_lshlrev_b32 by a constant is single-slot, v_lshrrev_b32 by one pairs)
        return "D"
    return "S"


def slots(items):
    c = collections.Counter()
    for kind, s in items:
        if kind == "ins":
            k = slot(s)
            if k:
                c[k] += 1
    return c


def quads(c):
    """Idealised quad-cycles for a body's VALU ops: at most one single-slot op per quad, two ops per quad."""
    return max(c["S"] + 2 * c["T"], (c["S"] + c["D"] + 2 * c["T"]) / 2)


def kernel_lines(lines, key):
    """The kernel's body lines (label to .Lfunc_end) and its metadata .set lines."""
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^(_Z\S*" + re.escape(key) + r"\S*):", ln):
            start, name = i, ln.split(":")[0]
            continue
        if start is not None and ln.startswith(".Lfunc_end"):
            body = lines[start + 1:i]
            meta = {}
            for m in lines[i:i + 40]:
                mm = re.match(r"\s*\.set\s+" + re.escape(name) + r"\.(\w+),\s*(\S+)", m)
                if mm:
                    meta[mm.group(1)] = mm.group(2)
            return name, body, meta
    raise SystemExit(f"kernel matching {key!r} not found")


def parse(body):
    """[(kind, text)]: kind 'label' or 'ins'."""
    out = []
    for ln in body:
        s = ln.split(";")[0].strip()
        if not s or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                out.append(("label", s[:-1]))
            continue
        out.append(("ins", s))
    return out


def census(items):
    c = collections.Counter()
    for kind, s in items:
        if kind == "ins":
            c[classify(s)] += 1
    return c


def fmt(c, keys=None):
    keys = keys or [k for k, _ in CLASSES] + ["other"]
    tot = sum(c.values())
    return f"{tot:5d} | " + " ".join(f"{k}={c[k]}" for k in keys if c[k])


def loops(items):
    """Natural loops from backward branches: (start index, end index, target label)."""
    pos = {s: i for i, (k, s) in enumerate(items) if k == "label"}
    res = []
    for i, (k, s) in enumerate(items):
        if k == "ins" and s.startswith("s_cbranch") or (k == "ins" and s.startswith("s_branch")):
            tgt = s.split()[-1]
            if tgt in pos and pos[tgt] < i:
                res.append((pos[tgt], i, tgt))
    # merge loops sharing a header: the outermost back edge
    by_head = {}
    for a, b, t in res:
        if a not in by_head or b > by_head[a][1]:
            by_head[a] = (a, b, t)
    return sorted(by_head.values(), key=lambda x: (x[0], -x[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="k_trace_wavepersistILb0ELi11ELi17ELi2E")
    ap.add_argument("--loops", action="store_true")
    ap.add_argument("--min-body", type=int, default=8, help="smallest loop body printed")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    name, body, meta = kernel_lines(lines, a.kernel)
    items = parse(body)
    print(f"kernel {name}")
    print("metadata: " + ", ".join(f"{k}={v}" for k, v in meta.items()
                                    if k in ("num_vgpr", "num_agpr", "numbered_sgpr", "private_seg_size")))
    spills = [ln.strip() for ln in body if re.search(r"(sgpr|vgpr)_spill_count|ScratchSize|NumVgprs|Occupancy", ln)]
    for s in spills:
        print("  " + s.lstrip("; "))
    print("whole kernel: " + fmt(census(items)))
    sl = slots(items)
    print(f"  VALU single-slot S={sl['S']} pairable D={sl['D']} transcendental T={sl['T']} "
          f"(S share {sl['S'] / max(1, sum(sl.values())):.2f})")
    if a.loops:
        stack = []
        for lo, hi, t in loops(items):
            while stack and not (stack[-1][0] <= lo and hi <= stack[-1][1]):
                stack.pop()
            c = census(items[lo:hi + 1])
            if sum(c.values()) >= a.min_body:
                sl = slots(items[lo:hi + 1])
                print(f"{'  ' * len(stack)}loop {t} (items {lo}-{hi}): " + fmt(c) +
                      f" | VALU S={sl['S']} D={sl['D']} T={sl['T']} quads>={quads(sl):.1f}")
            stack.append((lo, hi))


if __name__ == "__main__":
    sys.exit(main())
