#!/usr/bin/env python3
"""Per-frame time of the counted multi-GPU frame path on one GPU (RCCL, world size 1), with its look-aheads off,
with count-ahead, and with count- and emit-ahead: how much of the RNG exchange leaves the critical path.

    python tools/emit_ahead_probe.py [--width 7680 --height 544 --frames 60 --rounds 3]

The default frame is an eighth of C4 (the rows one rank of 8 traces).  Prints one JSON line.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=544)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from reflaxman_amd import scenes
    from reflaxman_amd.dist import RfxStripOps, StripFrame
    from reflaxman_amd.render import Renderer, build_scene, make_frame

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        scene, cam = build_scene(scenes.get_scene("synth16"))
        W, H = a.width, a.height
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        modes = {"none": (False, False), "count_ahead": (True, False), "count_and_emit_ahead": (True, True)}
        frames = {}
        for name, (ca, ea) in modes.items():
            r = Renderer(device=0, sphere_seed=1350490027)
            r.set_scene(scene)
            r.set_stream(stream.cuda_stream)
            frames[name] = StripFrame(RfxStripOps(r, make_frame(cam, W, H, 8, 1), stream.cuda_stream), W, H, 8, 0, 1,
                                      dev, count_ahead=ca, emit_ahead=ea)
        for sf in frames.values():
            for _ in range(20):
                sf.step()
        torch.cuda.synchronize()
        res = {k: [] for k in modes}
        for _ in range(a.rounds):
            for name, sf in frames.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.frames):
                    sf.step()
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) / a.frames * 1e3)
        print(json.dumps({"frame": [W, H], "ms_per_frame": {k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()}}))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
