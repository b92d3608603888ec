"""Summarise rocprofv3 --pmc CSVs of the trace kernel (+ its bounce kernel): per-frame means of each counter.

    python tools/pmc_summary.py [--kernel SUBSTR[,SUBSTR..]] [--out profiles/pmc/<name>.json
                                 --config SCENE W H DEPTH NGPUS SS] CSV...

With --out, also writes the HBM traffic record bench.py reads for `roofline.traffic`:
FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB per dispatch; the bytes are
taken as read + write.  (MI355X_MICROARCH.md: FETCH_SIZE counts exactly half the bytes of
16-B-per-lane streaming reads; this kernel's reads -- randDir dwords, texels, the scene --
are other widths, so FETCH_SIZE is used as reported, and the record says so.)
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflaxman_amd import _lib  # noqa: E402


def summarise(paths, kernel="trace_kernel<false,bounce_kernel"):
    """Per-frame counters: the mean per dispatch of each matching kernel (any of the comma-separated
    substrings), summed over the kernels -- the trace kernel and, on regrouped frames, its bounce kernel,
    each launched once per frame."""
    keys = kernel.split(",")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if any(k in name for k in keys):
                agg[r["Counter_Name"]][name].append(float(r["Counter_Value"]))
    return {c: sum(sum(v) / len(v) for v in per.values()) for c, per in sorted(agg.items())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="trace_kernel<false,bounce_kernel")
    ap.add_argument("--out")
    ap.add_argument("--config", nargs=6, help="SCENE W H DEPTH NGPUS SS (SS: samples per axis)")
    ap.add_argument("--lib-sha256", default=None, help="build the counters came from (default: the in-tree librfx.so)")
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    s = summarise(a.csv, a.kernel)
    if "SQ_ACTIVE_INST_VALU" in s and "SQ_THREAD_CYCLES_VALU" in s:
        s["valu_lane_util"] = s["SQ_THREAD_CYCLES_VALU"] / (64 * s["SQ_ACTIVE_INST_VALU"])
    print(json.dumps(s, indent=1))
    if a.out:
        scene, W, H, depth, n, ss = a.config
        rec = {
            "kernel": a.kernel, "config": [scene, int(W), int(H), int(depth), int(n), int(ss)],
            "lib_sha256": a.lib_sha256 or _lib.lib_sha256(),
            "device_sha256": None if a.lib_sha256 else _lib.device_sha256(),
            "fetch_bytes_per_launch": int(s["FETCH_SIZE"] * 1024), "write_bytes_per_launch": int(s["WRITE_SIZE"] * 1024),
            "hbm_bytes_per_launch": int((s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024),
            "note": "rocprofv3 FETCH_SIZE + WRITE_SIZE (KiB) per dispatch, separate --pmc passes; FETCH_SIZE uncorrected "
                    "(non-16B reads); Infinity-Cache hits may be counted",
            "counters": s,
        }
        json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
