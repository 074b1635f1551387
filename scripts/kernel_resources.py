#!/usr/bin/env python
"""Register / scratch / spill figures of the trace kernels from the gfx950
code-object metadata (hipcc -S with the Makefile's flags; runs on the CPU).

    python scripts/kernel_resources.py [--extra -DMM_AB_VARIANTS] [--filter wavepersist]

Prints one line per kernel: VGPRs, SGPRs, VGPR / SGPR spill counts, private
(scratch) bytes per lane, static LDS bytes.  bench.py reports the same VGPR /
scratch figures at run time through mm_scene_info (hipFuncGetAttributes).
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "mirror-maze_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extra", default="", help="extra hipcc flags (e.g. -DMM_AB_VARIANTS)")
    ap.add_argument("--filter", default="", help="substring of the mangled kernel name")
    ap.add_argument("--src", default="csrc/trace_kernels.hip")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-mllvm", "-amdgpu-use-amdgpu-trackers=1", f"-I{REPO / 'include'}", f"-I{PKG / 'csrc'}",
               "--cuda-device-only", "-S", "-o", str(out), str(PKG / args.src)] + args.extra.split()
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        text = out.read_text()
    # the amdhsa.kernels metadata block: one "- .args" entry per kernel
    meta = text[text.index("amdhsa.kernels:"):]
    fields = ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
              "group_segment_fixed_size")
    for ent in re.split(r"\n  - \.", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", ent)
        if not name or args.filter not in name.group(1):
            continue
        vals = {f: re.search(rf"\.{f}:\s+(\d+)", ent) for f in fields}
        vals = {f: (int(v.group(1)) if v else -1) for f, v in vals.items()}
        sym = name.group(1)
        try:
            sym = subprocess.run(["c++filt", sym], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        print(f"vgpr {vals['vgpr_count']:3d} sgpr {vals['sgpr_count']:3d} spill v/s {vals['vgpr_spill_count']:3d}/"
              f"{vals['sgpr_spill_count']:3d} scratch {vals['private_segment_fixed_size']:4d} B "
              f"lds {vals['group_segment_fixed_size']:5d} B  {sym[:150]}")


if __name__ == "__main__":
    sys.exit(main())
