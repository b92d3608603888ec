#!/usr/bin/env python3
"""Rewrite committed bench lines (profiles/**/*.json) from the round-1/2 `roofline` schema to round 3's.

Round 1/2 put the reference-equivalent algorithmic FLOP rate in `roofline.frac` (C5: 2.70, above the peak: the BVH
skips work the reference does).  Round 3's `roofline.frac` is the executed VALU lane-op fraction (<= 1) from the
line's own PMC-derived `executed` block, or null where the line had none; the old figures move, unchanged, to
`roofline.effective_ref_flops`.  No measured number changes: fields are moved and the line says so.

    python tools/migrate_roofline.py            # rewrites in place, prints what it changed
"""
from __future__ import annotations

import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_LANE_OPS_T = 78.6


def migrate(rf: dict) -> dict:
    if "effective_ref_flops" in rf:
        return rf
    ex = rf.get("executed") or None
    out = {
        "bound": rf.get("bound", "valu"),
        "achieved": ex.get("achieved_T_lane_ops") if ex else None,
        "peak": PEAK_LANE_OPS_T, "unit": "T VALU lane-op/s",
        "frac": ex.get("frac_lane_ops") if ex else None,
        "traffic": rf.get("traffic"),
        "frac_kind": "executed VALU lane-ops / launch time / 78.6 T lane-op/s (from the line's `executed` block); null "
                     "where the line had no PMC record",
        "avg_launch_ms": rf.get("avg_launch_ms"),
        "executed": ex,
        "effective_ref_flops": {
            "achieved": rf.get("achieved"), "unit": rf.get("unit", "TFLOP/s"), "flops_per_launch": rf.get("flops_per_launch"),
            "peak": rf.get("peak"), "frac": rf.get("frac"), "frac_vs_nofma_peak": rf.get("frac_vs_nofma_peak"),
            "kind": "reference-equivalent algorithmic FLOPs / launch time: effective work, not utilisation"},
        "migrated": "round-3 schema (tools/migrate_roofline.py): the round-1/2 `frac` is effective_ref_flops.frac",
    }
    for k in ("kernel", "algo_hbm_bytes_per_launch", "algo_hbm_GBps"):
        if k in rf:
            out[k] = rf[k]
    return out


def main():
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*.json"), recursive=True)):
        text = open(p).read()
        if '"roofline"' not in text:
            continue
        try:  # one JSON document (indented) ...
            doc = json.loads(text)
            if isinstance(doc, dict) and isinstance(doc.get("roofline"), dict):
                old = doc["roofline"].get("frac")
                doc["roofline"] = migrate(doc["roofline"])
                open(p, "w").write(json.dumps(doc, indent=1 if "\n " in text else None) + "\n")
                print(os.path.relpath(p, ROOT), old, "->", doc["roofline"]["frac"])
            continue
        except ValueError:
            pass
        lines = text.splitlines()  # ... or JSON lines mixed with log text
        for i, line in enumerate(lines):
            if line.startswith("{") and '"roofline"' in line:
                d = json.loads(line)
                if isinstance(d.get("roofline"), dict):
                    old = d["roofline"].get("frac")
                    d["roofline"] = migrate(d["roofline"])
                    lines[i] = json.dumps(d)
                    print(os.path.relpath(p, ROOT), old, "->", d["roofline"]["frac"])
        open(p, "w").write("\n".join(lines) + ("\n" if text.endswith("\n") else ""))


if __name__ == "__main__":
    main()
