#!/usr/bin/env python3
"""Host cost of a frame (needs a GPU): one renderer, the same frame K times -- the wall time to enqueue the K frames
(no synchronisation) against the wall time until they are complete, for each look-ahead mode.  When enqueueing takes
as long as rendering, the frame rate is bound by the host's launch path, not by the GPU.

    python tools/frame_host_cost.py [--scene default --width 640 --height 480 --depth 4 --frames 400]
"""
import argparse
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
    from reflaxman_amd import scenes
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    scene, cam = build_scene(scenes.get_scene(a.scene))
    W, H = a.width, a.height
    rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    f = make_frame(cam, W, H, a.depth, 1)
    rs = {}
    for mode in (0, 1, 2):
        r = Renderer(sphere_seed=1350490027)
        r.set_scene(scene)
        r.set_lookahead(mode)
        rs[mode] = r
    res = {m: {"enqueue_us": [], "frame_us": []} for m in rs}
    for _ in range(a.rounds):
        for m, r in rs.items():
            for _ in range(20):
                r.render_frame(f, rgb.data_ptr(), argb.data_ptr())
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                r.render_frame(f, rgb.data_ptr(), argb.data_ptr())
            t1 = time.perf_counter()
            r.synchronize()
            t2 = time.perf_counter()
            res[m]["enqueue_us"].append((t1 - t0) / a.frames * 1e6)
            res[m]["frame_us"].append((t2 - t0) / a.frames * 1e6)
    out = {"frame": f"{a.scene} {W}x{H} d{a.depth}", "frames": a.frames}
    for m, v in res.items():
        out[f"lookahead{m}"] = {k: round(sorted(x)[len(x) // 2], 2) for k, x in v.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
