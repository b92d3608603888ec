#!/usr/bin/env python3
"""Per-kernel register use of librfx's device code (CPU; hipcc only): VGPRs, VGPR / SGPR spills, scratch bytes per
lane and occupancy, from the compiler's kernel-resource-usage remarks, for every trace / bounce instantiation.

    python tools/resource_usage.py [TU ...]      # default: the plain-mode translation units
    python tools/resource_usage.py --json OUT    # also write the table as JSON

Kernel names are shortened to trace<STATS,MODE,CFG> / bounce<CFG> / bounce_lds<CFG> (the LDS-staged BVH form); CFG bits
(rfx_trace.h kCfg*): 1 cull, 2 >32 lights, 4 small scene, 8 planes, 16 park, 32 one light.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from reflaxman_amd import _build  # noqa: E402

FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
          "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill", "LDS Size [bytes/block]": "lds"}


def short(name: str) -> str:
    m = re.match(r"_ZN3rfx12trace_kernelILb(\d)ELi(\d+)ELi(\d+)EEEv", name)
    if m:
        return f"trace<{'stats' if m.group(1) == '1' else 'fast'},{m.group(2)},{m.group(3)}>"
    m = re.match(r"_ZN3rfx13bounce_kernelILi(\d+)EEEv", name)
    if m:
        return f"bounce<{m.group(1)}>"
    m = re.match(r"_ZN3rfx17bounce_kernel_ldsILi(\d+)EEEv", name)
    if m:
        return f"bounce_lds<{m.group(1)}>"
    return name


def usage(tu: str):
    flags = [f for f in _build.FLAGS if f != "-fPIC"] + os.environ.get("RFX_RU_DEFINES", "").split()
    with tempfile.TemporaryDirectory() as tmp:
        cmd = [_build.hipcc(), *flags, "--cuda-device-only", "-c", os.path.join(_build.CSRC, tu), "-o",
               os.path.join(tmp, "x.o"), "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-2000:])
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: \s*([^:]+?):\s*(\S+)\s*\[-Rpass-analysis", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2)
        if key == "Function Name":
            cur = {"kernel": short(val), "tu": tu}
            out.append(cur)
        elif cur is not None and key in FIELDS:
            cur[FIELDS[key]] = int(val)
    return [k for k in out if k["kernel"].startswith(("trace<", "bounce<", "bounce_lds<"))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tus", nargs="*", default=["rfx_trace_plain_fast.hip", "rfx_trace_plain_park.hip"])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = [k for tu in args.tus for k in usage(tu)]
    print(f"{'kernel':28s} {'vgpr':>5s} {'spill':>6s} {'sgpr_sp':>7s} {'scratch':>8s} {'occ':>4s}")
    for k in rows:
        print(f"{k['kernel']:28s} {k.get('vgpr', 0):5d} {k.get('vgpr_spill', 0):6d} {k.get('sgpr_spill', 0):7d} "
              f"{k.get('scratch', 0):8d} {k.get('occ', 0):4d}")
    if args.json:
        os.makedirs(os.path.dirname(os.path.abspath(args.json)), exist_ok=True)
        json.dump(rows, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
