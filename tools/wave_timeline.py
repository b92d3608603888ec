#!/usr/bin/env python3
"""The shape of one plain trace launch (diagnostic; needs a GPU): every wave's start and end on the chip's 100 MHz
clock, from the RFX_DEBUG_WAVES build (tools/build_diag.py -> lib/diag/librfx_waves.so), for the last of a few
frames of one view (per-view masks and the tile schedule at their defaults).

Prints, for the trace kernel (per 8x8 wave tile) and on regrouped large-scene frames the bounce kernel (per 64-trace
batch), the launch span (first wave start to last wave end), the dispatch ramp (how late waves start), the wave
durations (mean, percentiles, max), the waves still running over the last part of the span, and where the longest
waves start -- i.e. whether a launch is bound by its longest waves or by waiting for wave slots.

    python tools/wave_timeline.py [--scene default --width 640 --height 480 --depth 4 --frames 6 --tile-order 1]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from reflaxman_amd import _build, scenes  # noqa: E402
import ab  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz
BOUNCE_BASE = 1 << 17  # rfx_trace.h kBounceTimeBase: the bounce kernel's 64-trace batches


def summary(t, t0):
    """Span, start spread, durations and occupancy over time of one launch's waves (rows: start, end ticks)."""
    start, end = (t[:, 0] - t0) * TICK_US, (t[:, 1] - t0) * TICK_US
    dur = end - start
    span = end.max()
    q = lambda x, p: round(float(np.percentile(x, p)), 2)
    alive = lambda at: int(((start <= at) & (end > at)).sum())
    longest = np.argsort(-dur)[:8]
    return {
        "waves": int(len(t)), "span_us": round(float(span), 2),
        "start_us": {"p50": q(start, 50), "p90": q(start, 90), "max": round(float(start.max()), 2)},
        "duration_us": {"mean": round(float(dur.mean()), 2), "p50": q(dur, 50), "p90": q(dur, 90), "p99": q(dur, 99),
                        "max": round(float(dur.max()), 2)},
        "alive_at_fraction_of_span": {f: alive(f * span) for f in (0.1, 0.25, 0.5, 0.75, 0.9)},
        "longest_waves": [{"index": int(i), "start_us": round(float(start[i]), 2), "duration_us": round(float(dur[i]), 2)}
                          for i in longest],
        "wave_work_us_over_span": round(float(dur.sum() / span), 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="default")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--tile-order", type=int, default=None)
    a = ap.parse_args()
    path = os.path.join(_build.LIBDIR, "diag", "librfx_waves.so")
    r = ab.Runner("waves", path, scenes.get_scene(a.scene), a.width, a.height, a.depth, 1350490027,
                  tile_order=a.tile_order)
    r.render(a.frames)
    assert r.L.rfx_synchronize(r.r) == 0
    n = ((a.width + 7) // 8) * ((a.height + 7) // 8)
    cap = 1 << 18
    assert n <= BOUNCE_BASE, "frame too large for the timeline buffer"
    # each translation unit holds its own timeline: the plain kernels', and the parking trace and bounce kernels'
    t = np.zeros((cap, 2), np.int64)
    for fn in ("rfx_debug_wave_time_read", "rfx_debug_wave_time_read_park"):
        buf = (C.c_ulonglong * (2 * cap))()
        getattr(r.L, fn).argtypes = [C.c_void_p, C.c_int]
        assert getattr(r.L, fn)(buf, cap) == cap
        u = np.frombuffer(buf, np.uint64).reshape(cap, 2).astype(np.int64)
        t = np.where((u[:, 1] > t[:, 1])[:, None], u, t)  # the newer record of each slot
    tr = t[:n]
    t0 = tr[:, 0].min()
    out = {"frame": f"{a.scene} {a.width}x{a.height} d{a.depth}", "trace_kernel": summary(tr, t0)}
    b = t[BOUNCE_BASE:]
    b = b[(b[:, 0] >= t0) & (b[:, 1] > 0)]  # this frame's bounce batches (regrouped large-scene frames)
    if len(b):
        out["bounce_kernel"] = summary(b, b[:, 0].min())
    print(json.dumps(out, indent=1))
    r.close()


if __name__ == "__main__":
    main()
