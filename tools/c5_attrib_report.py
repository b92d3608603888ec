#!/usr/bin/env python3
"""Summarise tools/c5_attrib.sh's output: per kernel (trace / bounce) and regroup setting, the mean per dispatch of
WRITE_SIZE, FETCH_SIZE (bytes) and the memory-instruction counts, next to the algorithmic writes (16 B per pixel,
split by which kernel writes the pixel) and the queue (64 B per parked trace, from the segment histogram).

    python tools/c5_attrib_report.py gpurun_out/<dir>/c5 [--out profiles/r03/c5_write_attribution.json]
"""
from __future__ import annotations

import argparse
import ast
import collections
import csv
import glob
import json
import os

PIXELS = 3840 * 2160


def per_kernel(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            kind = ("trace" if "trace_kernel<false" in name else "bounce" if "bounce_kernel" in name else
                    "stats" if "trace_kernel<true" in name else None)
            if kind:
                agg[kind][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    seg = ast.literal_eval(open(os.path.join(a.dir, "segstats_c5.txt")).read().strip().splitlines()[-1])
    parked = seg["alive_after"]["3"] if "3" in seg["alive_after"] else seg["alive_after"][3]
    out = {"pixels": PIXELS, "parked_traces_park3": parked, "queue_bytes_written_park3": parked * 64,
           "algo_write_bytes": PIXELS * 16, "runs": {}}
    for rg in (3, 0):
        run = {}
        for part in ("w", "f", "i"):
            for kind, cs in per_kernel(os.path.join(a.dir, f"{part}_rg{rg}")).items():
                run.setdefault(kind, {}).update(cs)
        for kind, cs in run.items():
            for c in ("WRITE_SIZE", "FETCH_SIZE"):
                if c in cs:
                    cs[c.lower() + "_bytes"] = int(cs.pop(c) * 1024)
        out["runs"][f"park{rg}"] = run
    r3, r0 = out["runs"]["park3"], out["runs"]["park0"]
    w3 = sum(k.get("write_size_bytes", 0) for n, k in r3.items() if n in ("trace", "bounce"))
    w0 = r0.get("trace", {}).get("write_size_bytes", 0)
    out["summary"] = {
        "write_bytes_park3_trace_plus_bounce": w3, "write_bytes_park0_trace": w0,
        "x_algorithmic_park3": round(w3 / (PIXELS * 16), 3), "x_algorithmic_park0": round(w0 / (PIXELS * 16), 3),
        "beyond_output_and_queue_park3": w3 - PIXELS * 16 - parked * 64,
        "beyond_output_park0": w0 - PIXELS * 16,
    }
    print(json.dumps(out, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
