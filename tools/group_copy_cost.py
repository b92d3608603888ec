#!/usr/bin/env python3
"""Per-frame cost of the device group's band copies (include/rfx.h rfx_group_render_frame): the C4 frame (7680x4320
d8) on an N-member group, f32 RGB + ARGB8 bands copied to member 0 (16 B/px: what the drop-in Render pays, since
Render::imagePixel reads the float image) against ARGB8-only frames (d_rgb NULL, 4 B/px: a display path), timed
interleaved in one process.

    python tools/group_copy_cost.py [--members 8] [--frames 20] [--rounds 3] [--devices 0,0,...]

On the one-GPU box every member is device 0, so a "peer" copy is a device-local copy: the difference is the copies'
HBM and queue cost, not xGMI transfer time (DESIGN.md gives the xGMI estimate beside it).  Prints one JSON line.
"""
from __future__ import annotations

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
    ap.add_argument("--members", type=int, default=8)
    ap.add_argument("--devices", default=None, help="comma-separated device per member (default: all 0)")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    args = ap.parse_args()
    import torch
    from reflaxman_amd import _lib, scenes
    from reflaxman_amd.render import build_scene, make_frame
    L = _lib.load()
    devs = [int(d) for d in args.devices.split(",")] if args.devices else [0] * args.members
    n = len(devs)
    scene, cam = build_scene(scenes.get_scene("synth16"))
    g = C.c_void_p()
    _lib.check(L.rfx_group_create(C.byref(g), (C.c_int * n)(*devs), n), "group_create")
    _lib.check(L.rfx_group_set_scene(g, scene._h), "group_set_scene")
    W, H = args.width, args.height
    f = make_frame(cam, W, H, 8, 1)
    rgb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    argb = torch.zeros(W * H, dtype=torch.int32, device="cuda")

    def frame(with_rgb):
        _lib.check(L.rfx_group_render_frame(g, C.byref(f), C.c_void_p(rgb.data_ptr() if with_rgb else 0),
                                            C.c_void_p(argb.data_ptr()), None), "group_render_frame")

    for _ in range(24):  # clock ramp, balancer re-cuts (every 8 frames)
        frame(True)
    torch.cuda.synchronize()
    res = {True: [], False: []}
    for _ in range(args.rounds):
        for mode in (True, False):
            for _ in range(3):
                frame(mode)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                frame(mode)
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / args.frames * 1e3)
    b = (C.c_uint32 * (n + 1))()
    _lib.check(L.rfx_group_get_bands(g, b))
    L.rfx_group_destroy(g)
    both, only = min(res[True]), min(res[False])
    px_to_0 = W * (H - (b[1] - b[0]))
    print(json.dumps({
        "frame": f"synth16 {W}x{H} d8 (C4)", "members": n, "devices": devs, "bands": list(b),
        "ms_per_frame_rgb_and_argb": round(both, 4), "ms_per_frame_argb_only": round(only, 4),
        "rgb_copy_ms_per_frame": round(both - only, 4),
        "rounds_ms": {"rgb_and_argb": [round(x, 4) for x in res[True]], "argb_only": [round(x, 4) for x in res[False]]},
        "bytes_to_member0_per_frame": {"rgb_and_argb": px_to_0 * 16, "argb_only": px_to_0 * 4},
        "note": "members on one device: band copies are device-local (HBM), not xGMI" if len(set(devs)) == 1 else
                "members on distinct devices: band copies over xGMI (hipMemcpyPeerAsync)"}))


if __name__ == "__main__":
    main()
