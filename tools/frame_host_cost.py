#!/usr/bin/env python3
"""Cost of a frame by pre-pass form (needs a GPU): one renderer per form, the same frame K times, interleaved rounds in
one process -- the wall time to enqueue the K frames (no synchronisation) and the wall time until they are complete.
When enqueueing takes as long as rendering, the frame rate is bound by the host's launch path, not by the GPU.

Forms: "single" -- rfx_render_frame (rng_count recording each thread's accept flags, then rng_emit regenerating only
the accepted states); "two" -- rfx_frame_rng_count + rfx_render_frame_counted, the sliced pre-pass the multi-GPU ranks
use (rng_count, then rng_emit re-running the accept tests).  Both render the same pixels (tests/test_gpu_steady.py).
Round 3 also timed a one-launch form here (rng_scan_emit, commit d409089: count, decoupled look-back, emit) against
"two": DESIGN.md, measured and dropped.

    python tools/frame_host_cost.py [--scene default --width 640 --height 480 --depth 4 --frames 400]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="default")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from reflaxman_amd import _lib, scenes
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    L = _lib.load()
    scene, cam = build_scene(scenes.get_scene(a.scene))
    W, H = a.width, a.height
    rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    f = make_frame(cam, W, H, a.depth, 1)
    rs = {}
    for form in ("single", "two"):
        r = Renderer(sphere_seed=1350490027)
        r.set_scene(scene)
        rs[form] = r
    bps = C.c_uint64()
    _lib.check(L.rfx_frame_rng_blocks(rs["two"]._h, C.byref(f), 1, C.byref(bps)))
    counts = torch.zeros(bps.value, dtype=torch.int32, device="cuda")
    cp = C.c_void_p(counts.data_ptr())

    def frame(form, r):
        if form == "single":
            r.render_frame(f, rgb.data_ptr(), argb.data_ptr())
        else:
            _lib.check(L.rfx_frame_rng_count(r._h, C.byref(f), 0, 1, cp, None))
            _lib.check(L.rfx_render_frame_counted(r._h, C.byref(f), 1, cp, C.c_void_p(rgb.data_ptr()),
                                                  C.c_void_p(argb.data_ptr()), None, None))

    res = {m: {"enqueue_us": [], "frame_us": []} for m in rs}
    for _ in range(a.rounds):
        for m, r in rs.items():
            for _ in range(20):
                frame(m, r)
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                frame(m, r)
            t1 = time.perf_counter()
            r.synchronize()
            t2 = time.perf_counter()
            res[m]["enqueue_us"].append((t1 - t0) / a.frames * 1e6)
            res[m]["frame_us"].append((t2 - t0) / a.frames * 1e6)
    out = {"frame": f"{a.scene} {W}x{H} d{a.depth}", "frames": a.frames, "rounds": a.rounds}
    for m, v in res.items():
        out[m] = {k: round(sorted(x)[len(x) // 2], 2) for k, x in v.items()}
    print(json.dumps(out))
    for r in rs.values():
        r.close()


if __name__ == "__main__":
    main()
