"""Summarise rocprofv3 --pmc CSVs for the trace kernel (per-launch means of each counter)."""
import collections
import csv
import json
import sys


def summarise(paths, kernel="trace_kernel"):
    agg = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in sorted(agg.items())}


if __name__ == "__main__":
    s = summarise(sys.argv[1:])
    if "SQ_ACTIVE_INST_VALU" in s and "SQ_THREAD_CYCLES_VALU" in s:
        s["valu_lane_util"] = s["SQ_THREAD_CYCLES_VALU"] / (64 * s["SQ_ACTIVE_INST_VALU"])
    print(json.dumps(s, indent=1))
