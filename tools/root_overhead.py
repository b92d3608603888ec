#!/usr/bin/env python3
"""Rank 0's extra work at N > 1, measured on one GPU (a proxy: the 8-GPU scaling run is the driver's).

    python tools/root_overhead.py [--nranks 8] [--frames 40]

Rank 0 of an N-rank C4 frame traces its strips like every rank, and in addition receives the other N - 1 ARGB8
strips (RCCL lands them in its HBM through a staging FIFO: about a read and a write of each strip) and
un-interleaves the N strips into the frame on a side stream (reflaxman_amd/dist.py StripFrame, pipelined).
This renders rank 0's strip frames back to back (a) alone and (b) with that traffic -- N - 1 device copies of a
strip into the gather buffers plus the N index_copy_ of the assembly, on a side stream as the pipeline runs
them -- and prints both per-frame times: (b) - (a) is what rank 0 pays beyond the other ranks.  The RNG counts of
all N slices are computed on this one device per frame in both (a) and (b).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from reflaxman_amd import _lib, scenes  # noqa: E402
from reflaxman_amd.dist import strip_row_to_y, strip_rows  # noqa: E402
from reflaxman_amd.render import Renderer, build_scene, make_frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--partition", choices=["strips", "bands"], default="strips",
                    help="bands: rank 0 traces rows [0, H / N) into the whole frame and receives the other bands in place")
    a = ap.parse_args()
    N, W, H, rb = a.nranks, a.width, a.height, 8
    L = _lib.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    side = torch.cuda.Stream(device=dev)
    scene, cam = build_scene(scenes.get_scene("synth16"))
    rr = Renderer(device=0, sphere_seed=1350490027)
    rr.set_scene(scene)
    rr.set_stream(st.cuda_stream)
    bands = a.partition == "bands"
    band = (H // N) // 8 * 8
    f = make_frame(cam, W, H, 8, 1, row_block=0 if bands else rb, rank=0, nranks=N,
                   pixel_begin=0, pixel_end=band * W if bands else 0)
    bps = C.c_uint64()
    _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), N, C.byref(bps)))
    counts = torch.zeros(N * bps.value, dtype=torch.int32, device=dev)
    rows = band if bands else strip_rows(H, rb, 0, N)
    maxr = H if bands else max(strip_rows(H, rb, r, N) for r in range(N))
    img = torch.zeros(maxr * W * 3, dtype=torch.float32, device=dev)
    argb = [torch.zeros(maxr * W, dtype=torch.int32, device=dev) for _ in range(2)]
    src = [torch.randint(0, 1 << 24, (maxr * W,), dtype=torch.int32, device=dev) for _ in range(N)]
    gl = [[torch.empty(maxr * W, dtype=torch.int32, device=dev) for _ in range(N)] for _ in range(2)]
    full = [torch.zeros(H, W, dtype=torch.int32, device=dev) for _ in range(2)]
    idx = [torch.tensor([strip_row_to_y(i, rb, r, N) for i in range(strip_rows(H, rb, r, N))], dtype=torch.int64,
                        device=dev) for r in range(N)]
    done = [None, None]

    def frame(k, assemble):
        b = k % 2
        if assemble and done[b] is not None:
            st.wait_event(done[b])
        for s in range(N):
            _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), s, N, C.c_void_p(counts.data_ptr()),
                                             C.c_void_p(st.cuda_stream)))
        _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), N, C.c_void_p(counts.data_ptr()),
                                              C.c_void_p(img.data_ptr()), C.c_void_p(argb[b].data_ptr()), None,
                                              C.c_void_p(st.cuda_stream)))
        if not assemble:
            return
        ev = torch.cuda.Event()
        ev.record(st)
        with torch.cuda.stream(side):
            side.wait_event(ev)
            if bands:  # the other bands land in their rows of rank 0's frame: no un-interleave
                argb[b][band * W:].copy_(src[1][band * W:])
                e2 = torch.cuda.Event()
                e2.record(side)
                done[b] = e2
                return
            gl[b][0].copy_(argb[b])  # rank 0's own strip: a local copy in the gather
            for r in range(1, N):
                gl[b][r].copy_(src[r])  # the received strips landing in HBM
            for r in range(N):
                n = idx[r].numel()
                full[b].index_copy_(0, idx[r], gl[b][r][: n * W].view(n, W))
            e2 = torch.cuda.Event()
            e2.record(side)
            done[b] = e2

    res = {"alone": [], "with_assembly": []}
    for _ in range(5):
        frame(0, True)
    torch.cuda.synchronize()
    # phases of rank 0's own frame (HIP events: the emit of the counted pre-pass, the trace), and the N counts
    rr.get_timing()
    rr.set_timing(True)
    for k in range(a.frames):
        frame(k, False)
    pre_ms, trace_ms, nfr = rr.get_timing()
    rr.set_timing(False)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(st)
    for k in range(a.frames):
        for s in range(N):
            _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), s, N, C.c_void_p(counts.data_ptr()),
                                             C.c_void_p(st.cuda_stream)))
    ev1.record(st)
    torch.cuda.synchronize()
    phases = {"emit_ms": pre_ms / max(nfr, 1), "trace_ms": trace_ms / max(nfr, 1),
              "counts_all_slices_ms": ev0.elapsed_time(ev1) / a.frames}
    for _ in range(a.rounds):
        for mode, asm in (("alone", False), ("with_assembly", True)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.frames):
                frame(k, asm)
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / a.frames * 1e3)
    out = {"nranks": N, "partition": a.partition, "frame": [W, H], "rank0_rows": rows, "ms_per_frame": {k: sorted(v)[len(v) // 2] for k, v in res.items()}}
    out["root_extra_frac"] = round(out["ms_per_frame"]["with_assembly"] / out["ms_per_frame"]["alone"] - 1, 4)
    out["phases_alone"] = {k: round(v, 4) for k, v in phases.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
