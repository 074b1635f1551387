"""Which measurement records describe the working tree's product sources?
Lists every profiles/pmc_*.json and every bench line under a profiles/r*/
results directory with the source hash it carries against
`bench.py --src-hash`, so a stale record is visible before a round ends.

    python scripts/check_records.py [--round r04]
Exit status 1 when a top-level PMC record is stale (bench.py would then label
its lines "stale" and print a null roofline fraction).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main() -> int:
    from bench import src_hash

    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default=None, help="also check profiles/<round>/results/*.json")
    a = ap.parse_args()
    here = src_hash()
    print(f"product sources: {here}")
    stale = 0
    for f in sorted((REPO / "profiles").glob("pmc_*.json")):
        h = json.loads(f.read_text()).get("src_hash")
        ok = h == here
        stale += not ok
        print(f"  {'ok   ' if ok else 'STALE'} {f.relative_to(REPO)} ({h})")
    if a.round:
        for f in sorted((REPO / "profiles" / a.round / "results").glob("*.json")):
            lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
            if not lines:
                continue
            m = json.loads(lines[0]).get("roofline", {}).get("measured") or {}
            h = m.get("src_hash") if not m.get("stale") else m.get("profile_src_hash")
            ok = h == here and not m.get("stale")
            print(f"  {'ok   ' if ok else 'STALE'} {f.relative_to(REPO)} (measured {m.get('source')}, {h})")
    return 1 if stale else 0


if __name__ == "__main__":
    sys.exit(main())
