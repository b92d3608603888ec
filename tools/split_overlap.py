"""Overlap of a split frame's launches (rocprofv3 --kernel-trace CSV of `bench.py --config shot128`): per trace launch
its stream, start, end and duration, how long the two streams' trace kernels ran at the same time, and how much of each
pre-pass ran beside the other stream's trace.  Usage: python tools/split_overlap.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted(({"name": r["Kernel_Name"], "stream": r.get("Stream_Id") or r.get("Queue_Id"),
                  "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])} for r in rows), key=lambda k: k["t0"])
    trace = [k for k in ks if "trace_kernel<" in k["name"]]
    pre = [k for k in ks if "rng_" in k["name"]]

    def overlap(a, b):
        return max(0, min(a["t1"], b["t1"]) - max(a["t0"], b["t0"]))

    tt = sum(overlap(a, b) for i, a in enumerate(trace) for b in trace[i + 1:] if a["stream"] != b["stream"])
    pp = sum(overlap(p, t) for p in pre for t in trace if p["stream"] != t["stream"])
    span = (trace[-1]["t1"] - trace[0]["t0"]) if trace else 0
    out = {"trace_launches": len(trace), "streams": sorted({k["stream"] for k in trace}),
           "trace_ms_mean": round(sum(k["t1"] - k["t0"] for k in trace) / max(len(trace), 1) / 1e6, 3),
           "span_ms": round(span / 1e6, 3),
           "trace_trace_overlap_ms": round(tt / 1e6, 3),
           "prepass_ms_total": round(sum(k["t1"] - k["t0"] for k in pre) / 1e6, 3),
           "prepass_beside_other_trace_ms": round(pp / 1e6, 3)}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
