"""Algorithmic work model of the trace loop, priced from the kernel's event counters.

Counting rule: every f32 + - x / sqrt is 1 FLOP, compares,
abs, clamps, selects and negations are 0, each powf is 1.  The weights are the
operations the trace loop *needs* per event in our formulation (closest-hit
candidates stop at their distance; drop/normal/reflection/texel are derived
once, for the winner) -- read off reflaxman_amd/csrc/rfx_trace.h, which
follows Scene.cpp:73-236 operation for operation.  The event counts come from
the stats build of the same kernel (``trace_kernel<true>``) and are tested
equal to the CPU restatement's (tests/test_gpu_parity.py).

Two views of the trace kernel's work (bench.py reports both):

* algorithmic FLOPs (``flops``): the reference's brute-force work -- every
  intersection test Scene::trace runs -- priced per event.  The kernel skips
  most of those tests exactly (wave-bundle culling), and a correctly rounded
  f32 divide or sqrt expands to ~10-15 VALU instructions, so FLOPs / time is an
  *effective* rate: it can exceed what the VALU executes (C5) or fall far
  below it (C1).  It is not a hardware utilisation.
* executed VALU work (``executed_work``): the instructions the kernel really
  issued, from a rocprofv3 --pmc record of the same workload and library build
  -- VALU lane-operations per second against the 78.6 T lane-op/s peak, and
  wave-instruction issue slots against 1024 SIMDs x 2.4 GHz / 2 cycles.
"""
from __future__ import annotations

import json
import os

COUNTER_NAMES = [
    "rays", "segments",
    "sph_tests", "sph_b", "sph_d", "sph_t",
    "tri_tests", "tri_z", "tri_s", "tri_t", "tri_in", "tri_d",
    "hit_sph", "hit_tri",
    "sh_sph_tests", "sh_sph_b", "sh_sph_d", "sh_sph_t",
    "sh_tri_tests", "sh_tri_z", "sh_tri_s", "sh_tri_t", "sh_tri_in",
    "l_eval", "l_facing", "l_lit", "l_spec", "l_pow",
    "dielectric", "metal", "continue", "sky",
    "tex_bilinear", "tex_checker", "tex_other",
    "pln_tests", "pln_t", "hit_pln", "sh_pln_tests", "sh_pln_t",
]

# FLOPs per event (see module docstring for the rule)
FLOP_WEIGHTS = {
    "rays": 24,         # rx, ry (2); + ss offset + jitter (4); view * ray (15); pixel sum (3)  [ss = 1]
    "segments": 10,     # |ray|^2 (5), 2*ray (3), 4a, 2a
    "sph_tests": 8,     # vco (3), b (5)                                       Sphere.cpp:50-52
    "sph_b": 9,         # c (6), d (3)  -- only when b <= 0 (b > 0 is an exact reject)
    "sph_d": 3,         # sqrt, -b - sqrt, / 2a                                Sphere.cpp:58
    "sph_t": 9,         # ray * t (3), |.| (6)                                 Sphere.cpp:62-63
    "tri_tests": 13,    # o - v0 (3), z rows of axTrans * (o - v0) and axTrans * ray (10)  Triangle.cpp:55-56
    "tri_z": 0,         # sign pre-check (compares only)
    "tri_s": 1,         # t = -ao.z / ar.z
    "tri_t": 25,        # x, y rows of both products (20), u, v (4), u + v (1)
    "tri_in": 8,        # ray * t (3), |.|^2 (5)
    "tri_d": 1,         # sqrt
    "hit_sph": 47,      # ray*t, drop, norm (9), reflect (20), |ray| |norm| |refl| (18)
    "hit_tri": 52,      # ray*t, drop (6), reflect (20), lengths (18), tuv * (u,v,0) + (tu0,tv0) (8)
    "sh_sph_tests": 8, "sh_sph_b": 9, "sh_sph_d": 3, "sh_sph_t": 9,
    "sh_tri_tests": 13, "sh_tri_z": 0, "sh_tri_s": 1, "sh_tri_t": 25, "sh_tri_in": 8,
    "l_eval": 8,        # dropToLight (3), . norm (5)                          Scene.cpp:121-124
    "l_facing": 16,     # shadow ray (6) + any-hit setup (10)                 Scene.cpp:128-129
    "l_lit": 30,        # |L|, cos, diffuse accumulate, angular radius        Scene.cpp:146-160
    "l_spec": 32,       # normalized(L) + jitter, |.|*|refl|, cos, clamp     Scene.cpp:162-166
    "l_pow": 12,        # exponent (4), powf (1), * refl, colour, accumulate Scene.cpp:172-176
    "dielectric": 33,   # ambient (3), Fresnel (11), finColor (10), mul (6), accumulate (3)
    "metal": 24,        # ambient (3), finColor (9), mul (6), accumulate (3)
    "continue": 16,     # normalized(reflect) + randDir * (1 - refl)          Scene.cpp:224
    "sky": 27,          # normalize (9), |n|+eps (3), u, v (6), accumulate (9)
    "tex_bilinear": 45, # fx, fy, fractions (6), 4 texels ARGB/255 (12), lerp (27)
    "tex_checker": 2,   # u*50, v*50
    "tex_other": 3,
    "pln_tests": 13,    # pos - o (3), norm . ray (5), norm . vop (5)            Plane.cpp:40-45
    "pln_t": 9,         # t (1), ray * t (3), |.|^2 (5)                          Plane.cpp:45-50
    "hit_pln": 45,      # sqrt (1), ray*t, drop (6), reflect (20), lengths (18)
    "sh_pln_tests": 13, "sh_pln_t": 9,
}

POW_EVENTS = ("l_pow", "dielectric")  # one powf each

# MI355X peaks (MI355X_MICROARCH.md: chip-level parameters)
PEAK_FP32_VALU_TFLOPS = 157.3   # spec, packed-FMA rate
PEAK_FP32_NOFMA_TFLOPS = 78.6   # separate v_mul/v_add (parity forbids contraction)
PEAK_HBM_GBS = 8000.0
# executed-work peaks: 256 CU x 4 SIMD-32 x 2.4 GHz -- one lane-op per lane per clock; a wave64 VALU
# instruction issues over 2 clocks (MI355X_MICROARCH.md, Wave scheduling)
PEAK_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
PEAK_VALU_WAVE_INSTS = 256 * 4 * 2.4e9 / 2

# algorithmic HBM bytes per pixel: f32 RGB framebuffer (12) + ARGB8 (4) written once
ALGO_BYTES_PER_PIXEL = 16


def flops(counts) -> int:
    """Algorithmic FLOPs for a dict/list of event counts."""
    if not isinstance(counts, dict):
        counts = dict(zip(COUNTER_NAMES, [int(c) for c in counts]))
    return int(sum(FLOP_WEIGHTS[k] * int(counts.get(k, 0)) for k in FLOP_WEIGHTS))


def summary(counts) -> dict:
    if not isinstance(counts, dict):
        counts = dict(zip(COUNTER_NAMES, [int(c) for c in counts]))
    rays = max(1, counts["rays"])
    return {
        "flops": flops(counts),
        "flops_per_ray": flops(counts) / rays,
        "segments_per_ray": counts["segments"] / rays,
        "shadow_rays_per_ray": counts["l_facing"] / rays,
        "isect_tests_per_ray": (counts["sph_tests"] + counts["tri_tests"] + counts.get("pln_tests", 0)) / rays,
        "shadow_tests_per_ray": (counts["sh_sph_tests"] + counts["sh_tri_tests"] + counts.get("sh_pln_tests", 0)) / rays,
        "pow_calls": sum(counts[k] for k in POW_EVENTS),
    }


def pmc_record(directory: str, config, lib_sha: str, device_sha: str = None):
    """The rocprofv3 --pmc record (tools/pmc_summary.py --out) of this workload and of this library build -- the
    same library file, or the same device code (its .hip_fatbin section, _lib.device_sha256) -- or None."""
    if not os.path.isdir(directory):
        return None
    for name in sorted(os.listdir(directory)):
        if not name.endswith(".json"):
            continue
        rec = json.load(open(os.path.join(directory, name)))
        if rec.get("config") != list(config):
            continue
        if rec.get("lib_sha256") == lib_sha or (device_sha and rec.get("device_sha256") == device_sha):
            return rec
    return None


def roofline(executed, traffic, flops_launch: float, trace_ms: float, px_launch: int) -> dict:
    """bench.py's `roofline` object for the trace kernel.  The bound is the FP32 VALU (no dense contraction, HBM
    traffic ~16 B/px): `achieved` is the executed VALU lane-op rate of one launch (PMC record of this workload and
    build, rated at this run's HIP-event launch time) against the 78.6 T lane-op/s peak, so `frac` is a hardware
    fraction <= 1 -- null when no PMC record matches.  The reference-equivalent algorithmic rate (SURVEY 8(d)
    counting rule over the reference's brute-force tests, which exact culling and the BVH skip) is reported beside
    it as `effective_ref_flops`: it is effective work, and exceeds the peak on C5."""
    t = trace_ms * 1e-3
    ach = flops_launch / t / 1e12
    out = {
        "bound": "valu",
        "achieved": executed["achieved_T_lane_ops"] if executed and "achieved_T_lane_ops" in executed else None,
        "peak": round(PEAK_VALU_LANE_OPS / 1e12, 1), "unit": "T VALU lane-op/s",
        "frac": executed["frac_lane_ops"] if executed and "frac_lane_ops" in executed else None,
        "traffic": traffic,
        "frac_kind": "executed VALU lane-ops per launch (SQ_INSTS_VALU x 64 x lane utilisation, rocprofv3 --pmc of this "
                     "workload and library build) / HIP-event launch time / 78.6 T lane-op/s (256 CU x 128 FP32 lanes "
                     "x 2.4 GHz, non-FMA: parity forbids contraction); null without a matching PMC record",
        "avg_launch_ms": round(trace_ms, 4),
        "executed": executed,
        "effective_ref_flops": {
            "achieved": round(ach, 3), "unit": "TFLOP/s", "flops_per_launch": int(flops_launch),
            "peak": PEAK_FP32_VALU_TFLOPS, "frac": round(ach / PEAK_FP32_VALU_TFLOPS, 4),
            "frac_vs_nofma_peak": round(ach / PEAK_FP32_NOFMA_TFLOPS, 4),
            "kind": "reference-equivalent algorithmic FLOPs / launch time: effective work, not utilisation"},
        "algo_hbm_bytes_per_launch": px_launch * ALGO_BYTES_PER_PIXEL,
        "algo_hbm_GBps": round(px_launch * ALGO_BYTES_PER_PIXEL / t / 1e9, 1),
    }
    return out


def executed_work(rec, trace_ms: float):
    """Executed VALU work of one trace launch from a PMC record, rated at this run's kernel time."""
    if not rec:
        return None
    c = rec["counters"]
    insts = c["SQ_INSTS_VALU"]
    util = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]) if c.get("SQ_ACTIVE_INST_VALU") else None
    lane_ops = insts * 64.0 * util if util else None
    t = trace_ms * 1e-3
    out = {"valu_wave_insts_per_launch": int(insts), "valu_lane_util": round(util, 4) if util else None,
           "valu_issue_frac": round(insts / t / PEAK_VALU_WAVE_INSTS, 4)}
    if lane_ops:
        out.update({"valu_lane_ops_per_launch": int(lane_ops), "achieved_T_lane_ops": round(lane_ops / t / 1e12, 2),
                    "peak_T_lane_ops": round(PEAK_VALU_LANE_OPS / 1e12, 1),
                    "frac_lane_ops": round(lane_ops / t / PEAK_VALU_LANE_OPS, 4)})
    out["source"] = rec.get("source", "rocprofv3 --pmc")
    return out
