#!/usr/bin/env python3
"""A/B timing of librfx.so variant builds, interleaved in ONE process on ONE GPU.

    python tools/ab.py build                 # (CPU) compile reflaxman_amd/lib/variants/librfx_<name>.so
    python tools/ab.py run [--rounds R] ...  # (GPU) parity-check + interleaved timing of every built variant

Cross-run / cross-device timings differ by up to ~12% (DVFS, device spread), so
kernel changes are judged only by interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Every variant's first frame must
hash to the reference's full-frame SHA-256 before its timing counts.
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import hashlib
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from reflaxman_amd import _build, _lib, scenes  # noqa: E402

_HIP = C.CDLL("libamdhip64.so")

VARIANTS = {
    "base": [],
    "nopark": ["RFX_PARK_AFTER=0"],
    "park1": ["RFX_PARK_AFTER=1"],
    "park3": ["RFX_PARK_AFTER=3"],
    "bvhall": ["RFX_NARROW_BUNDLE_COS=2.0f"],
    "narrow99": ["RFX_NARROW_BUNDLE_COS=0.99f"],
    "narrow9999": ["RFX_NARROW_BUNDLE_COS=0.99999f"],
    "wg2": ["RFX_WG_WAVES=2"],
    "wg4": ["RFX_WG_WAVES=4"],
    "wpe8": ["RFX_WAVES_PER_EU=8"],
    "wpe6": ["RFX_WAVES_PER_EU=6"],
    "wg1": ["RFX_WG_WAVES=1"],
    "wpe7": ["RFX_WAVES_PER_EU=7"],
    "wg2wpe7": ["RFX_WG_WAVES=2", "RFX_WAVES_PER_EU=7"],
    "raster": ["RFX_TILE_ORDER_DEFAULT=0"],
    "rastercost": ["RFX_TILE_ORDER_DEFAULT=2"],
    "every1": ["RFX_TILE_SORT_EVERY=1"],
    "every2": ["RFX_TILE_SORT_EVERY=2"],
    "every8": ["RFX_TILE_SORT_EVERY=8"],
    "every16": ["RFX_TILE_SORT_EVERY=16"],
    "qsort": ["RFX_QUEUE_SORT=1"],
    "lpt16k": ["RFX_TILE_ORDER_MIN_TILES=16384"],
    "lpt4k": ["RFX_TILE_ORDER_MIN_TILES=4096"],
    "bg16": ["RFX_BOUNCE_GROUPS_PER_CU=16"],
    "bg8": ["RFX_BOUNCE_GROUPS_PER_CU=8"],
    "nolaunder": ["RFX_NO_LAUNDER"],
    "launderscene": ["RFX_NO_LAUNDER", "RFX_LAUNDER_SCENE"],
    "launderparams": ["RFX_NO_LAUNDER", "RFX_LAUNDER_PARAMS"],
    "primssaa": ["RFX_PRIM_SSAA=1"],
    "primlarge": ["RFX_PRIM_LARGE=1"],
    "ssaalds": ["RFX_SSAA_LDS_STATE"],
    "nolanes": ["RFX_SSAA_LANES=0"],
    "halves": ["RFX_HALF_BUNDLES"],
    "nolight1": ["RFX_ONE_LIGHT=0"],
    "noprimlanes": ["RFX_PRIM_LANES=0"],
    "nobvhfma": ["RFX_BVH_FMA=0"],
    "tlim": ["RFX_BVH_TLIM=1"],
    "noprewide": ["RFX_BVH_PREWIDE=0"],
    "pwlite": ["RFX_BVH_PREWIDE_KEEP=0"],
    "tlimlite": ["RFX_BVH_TLIM=1", "RFX_BVH_PREWIDE_KEEP=0"],
    "nocullfma": ["RFX_CULL_FMA=0"],
    "lanes8": ["RFX_LANES_WAVES_PER_EU=8"],
    "nb999": ["RFX_NARROW_BUNDLE_COS=0.999f"],
    "nocullsmall": ["RFX_NOCULL_MAX_TILES=8192"],
    "large6": ["RFX_WAVES_PER_EU_LARGE=6"],
    "large5": ["RFX_WAVES_PER_EU_LARGE=5"],
    "scanall": ["RFX_SCAN_EMIT_BLOCKS=0"],
    "chsum0": ["RFX_SSAA_CHANNEL_SUM=0"],
    "nochunkmask": ["RFX_PRIM_CHUNKS=0"],
    "fused0": ["RFX_RNG_FUSED=0"],
    "nohint": ["RFX_OCC_HINT=0"],
    "split1": ["RFX_SPLIT_STREAMS=1"],
    "leaf1": ["RFX_BVH_LEAF_PAIRS=1"],
    "leaf2": ["RFX_BVH_LEAF_PAIRS=2"],
    "leaf8": ["RFX_BVH_LEAF_PAIRS=8"],
    "lt28": ["RFX_LAUNCH_TRACES=(1ull<<28)"],
    "lt31": ["RFX_LAUNCH_TRACES=(1ull<<31)"],
    "lt29": ["RFX_LAUNCH_TRACES=(1ull<<29)"],
    "div0": ["RFX_DIV_FAST=0"],
    "divsingle": ["RFX_DIV_SINGLE=1"],
    "divall2": ["RFX_DIV_FAST=2", "RFX_DIV_SINGLE=1"],
    "ticket0": ["RFX_RNG_TICKET=0"],
    "lookback0": ["RFX_LOOKBACK_SPINS=0"],
    "tiles0": ["RFX_SCAN_TILES=0"],
    "fmax256": ["RFX_RNG_FUSED_MAX_BLOCKS=256"],
    "fmax512": ["RFX_RNG_FUSED_MAX_BLOCKS=512"],
    "divsel1": ["RFX_DIV_SEL=1"],
    "divfast2": ["RFX_DIV_FAST=2"],
    "intacc0": ["RFX_RNG_INT_ACCEPT=0"],
    "se4096": ["RFX_SCAN_EMIT_BLOCKS=4096"],
    "sortside4": ["RFX_TILE_SORT_MAIN=0", "RFX_TILE_SORT_EVERY=4"],
    "sortside16": ["RFX_TILE_SORT_MAIN=0", "RFX_TILE_SORT_EVERY=16"],
    "sortmain4": ["RFX_TILE_SORT_EVERY=4"],
    "sort32": ["RFX_TILE_SORT_EVERY=32"],
    "fmax1024": ["RFX_RNG_FUSED_MAX_BLOCKS=1024"],
    "fmax4096": ["RFX_RNG_FUSED_MAX_BLOCKS=4096"],
}


def build_scene_with(L, desc):
    fa = _lib.farr
    s = C.c_void_p(L.rfx_scene_create(*desc.diffuse))
    keep = []
    if desc.skybox is not None and desc.skybox.argb is not None:
        a = np.ascontiguousarray(desc.skybox.argb, np.uint32)
        keep.append(a)
        L.rfx_scene_set_skybox_argb(s, a.shape[1], a.shape[0], _lib.u32ptr(a))
    for (o, r, c, p) in desc.lights:
        L.rfx_scene_add_light(s, fa(o), r, fa(c), p)
    tex = []
    for t in desc.textures:
        if t.argb is None:
            tex.append(L.rfx_scene_add_texture_argb(s, 0, 0, None))
        else:
            a = np.ascontiguousarray(t.argb, np.uint32)
            keep.append(a)
            tex.append(L.rfx_scene_add_texture_argb(s, a.shape[1], a.shape[0], _lib.u32ptr(a)))
    for ob in desc.objects:
        mt, rgb, refl, tr = ob[-1]
        if ob[0] == "sphere":
            L.rfx_scene_add_sphere(s, fa(ob[1]), ob[2], mt, fa(rgb), refl, tr)
        elif ob[0] == "plane":
            L.rfx_scene_add_plane(s, fa(ob[1]), fa(ob[2]), mt, fa(rgb), refl, tr)
        else:
            L.rfx_scene_add_triangle(s, fa(ob[1]), fa(ob[2]), fa(ob[3]), mt, fa(rgb), refl, tr)
    for (oi, ti, uv) in desc.settex:
        L.rfx_triangle_set_texture(s, oi, tex[ti], fa(uv))
    eye, at, fov = desc.camera
    view = (C.c_float * 9)()
    L.rfx_camera_view(fa(eye), fa(at), view)
    return s, list(eye), list(view), fov


class Runner:
    def __init__(self, name, path, desc, W, H, depth, seed, tile_order=None, regroup=None, prim=None, ss=1, additive=0):
        self.name = name
        L = self.L = _lib.bind(path, partial=True)
        self.scene, eye, view, fov = build_scene_with(L, desc)
        self.r = C.c_void_p()
        rc = L.rfx_renderer_create(C.byref(self.r), 0)
        assert rc == 0, L.rfx_last_error()
        assert L.rfx_renderer_set_scene(self.r, self.scene) == 0, L.rfx_last_error()
        assert L.rfx_renderer_set_rng(self.r, seed, 0) == 0
        if tile_order is not None:
            assert L.rfx_renderer_set_tile_order(self.r, tile_order) == 0
        if regroup is not None:
            assert L.rfx_renderer_set_regroup(self.r, regroup) == 0
        if prim is not None:
            assert L.rfx_renderer_set_prim_masks(self.r, prim) == 0
        self.W, self.H = W, H
        self.img, self.argb = C.c_void_p(), C.c_void_p()
        assert L.rfx_device_alloc(self.r, W * H * 12, C.byref(self.img)) == 0
        assert L.rfx_device_alloc(self.r, W * H * 4, C.byref(self.argb)) == 0
        f = _lib.Frame()
        f.eye[:] = eye
        f.view[:] = view
        f.fov = fov
        f.width, f.height, f.reflect_num, f.sample_num, f.nranks = W, H, depth, ss, 1
        f.additive = additive  # jitter (Render.cpp:177-178); additive_counter 0: no accumulation
        self.frame = f

    def render(self, n=1):
        for _ in range(n):
            rc = self.L.rfx_render_frame(self.r, C.byref(self.frame), self.img, self.argb, None, None)
            assert rc == 0, self.L.rfx_last_error()

    def close(self):
        self.L.rfx_device_free(self.r, self.img)
        self.L.rfx_device_free(self.r, self.argb)
        self.L.rfx_renderer_destroy(self.r)
        self.L.rfx_scene_destroy(self.scene)

    def frame_hashes(self, n=1):
        """Render n frames (continuing the random stream); hashes of the last one."""
        self.render(n)
        assert self.L.rfx_synchronize(self.r) == 0
        rgb = np.empty(self.W * self.H * 3, np.float32)
        argb = np.empty(self.W * self.H, np.uint32)
        self.L.rfx_memcpy_d2h(self.r, rgb.ctypes.data_as(C.c_void_p), self.img, rgb.nbytes)
        self.L.rfx_memcpy_d2h(self.r, argb.ctypes.data_as(C.c_void_p), self.argb, argb.nbytes)
        return hashlib.sha256(rgb.tobytes()).hexdigest(), hashlib.sha256(argb.tobytes()).hexdigest()

    def timed(self, frames):
        self.L.rfx_renderer_set_timing(self.r, 1)
        _HIP.hipDeviceSynchronize()
        t0 = time.perf_counter()
        self.render(frames)
        _HIP.hipDeviceSynchronize()   # every stream: a speculative pre-pass counts too
        wall = (time.perf_counter() - t0) * 1e3 / frames
        pre, tr, n = C.c_double(), C.c_double(), C.c_uint64()
        self.L.rfx_renderer_get_timing(self.r, C.byref(pre), C.byref(tr), C.byref(n))
        self.L.rfx_renderer_set_timing(self.r, 0)
        return pre.value / n.value, tr.value / n.value, wall


def cmd_build(names):
    for n in names:
        p = _build.build_variant(n, VARIANTS[n])
        print("built", p)


def cmd_run(args):
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))["cases"]
    key = f"hash_{args.scene}_{args.width}x{args.height}_d{args.depth}" + (f"_ss{args.ss}" if args.ss != 1 else "") + \
        ("_jitter" if args.additive else "")
    desc = scenes.get_scene(args.scene)
    paths = sorted(glob.glob(os.path.join(_build.LIBDIR, "variants", "librfx_*.so")))
    names = [os.path.basename(p)[len("librfx_"):-3] for p in paths]
    if args.only:
        keep = set(args.only.split(","))
        paths, names = zip(*[(p, n) for p, n in zip(paths, names) if n in keep])
    # runtime variants: every build once per --regroup setting (rfx_renderer_set_regroup), named build@parkN
    regroups = [None] if not args.regroup else [int(v) for v in args.regroup.split(",")]
    prims = [None] if not args.prim else [int(v) for v in args.prim.split(",")]
    runners = [Runner(n + ("" if g is None else f"@park{g}") + ("" if q is None else f"@prim{q}"), p, desc, args.width,
                      args.height, args.depth, 1350490027, regroup=g, prim=q, ss=args.ss, additive=args.additive)
               for n, p in zip(names, paths) for g in regroups for q in prims]
    # parity of every variant: frame 1 against the reference's full-frame hash (when the manifest has one), and
    # frame 1 + LATER frames (rendered in the learned longest-tile-first order, after the tile sorts) against
    # the product build rendering the same frames in raster order
    later = max(2, args.later_frame)
    ref = Runner("raster", _build.LIB, desc, args.width, args.height, args.depth, 1350490027, tile_order=0, ss=args.ss,
                 additive=args.additive)
    ref_first = ref.frame_hashes(1)
    ref_later = ref.frame_hashes(later - 1)
    ref.close()
    parity = {}
    for r in runners:
        first = r.frame_hashes(1)
        ok = first == ref_first and (key not in man or first == (man[key]["sha_f32"], man[key]["sha_argb"]))
        parity[r.name] = ok and r.frame_hashes(later - 1) == ref_later
        r.render(args.warmup)
    times = {r.name: [] for r in runners}
    pre = {r.name: [] for r in runners}
    wall = {r.name: [] for r in runners}
    for _ in range(args.rounds):
        for r in runners:
            p, t, w = r.timed(args.frames)
            times[r.name].append(t)
            pre[r.name].append(p)
            wall[r.name].append(w)
    base = statistics.median(times[runners[0].name])
    out = []
    for r in runners:
        if not parity[r.name]:  # a variant that renders other pixels has no timing worth reporting
            out.append({"variant": r.name, "defines": VARIANTS.get(r.name.split("@")[0]), "parity_sha_ok": False,
                        "timings": None})
            continue
        med = statistics.median(times[r.name])
        out.append({"variant": r.name, "defines": VARIANTS.get(r.name.split("@")[0]), "parity_sha_ok": parity[r.name],
                    "trace_ms_median": round(med, 4), "trace_ms_min": round(min(times[r.name]), 4),
                    "prepass_ms_median": round(statistics.median(pre[r.name]), 4),
                    "frame_ms_median": round(statistics.median(wall[r.name]), 4),
                    "vs_first": round(med / base, 4),
                    "mrays_trace_only": round(args.width * args.height * args.ss ** 2 / (med * 1e-3) / 1e6, 1)})
    for o in out:
        print(json.dumps(o))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--only", default="")
    ap.add_argument("--scene", default="synth16")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--ss", type=int, default=1, help="samples per pixel ss x ss (SSAA frames)")
    ap.add_argument("--additive", type=int, default=0, help="1: jittered frames (Render.cpp:177-178)")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--later-frame", type=int, default=7, help="frame (1-based) also checked against raster order")
    ap.add_argument("--regroup", default="", help="comma list of park_after settings to run each build with (0 = off)")
    ap.add_argument("--prim", default="", help="comma list of rfx_renderer_set_prim_masks modes to run each build with")
    args = ap.parse_args()
    if args.cmd == "build":
        cmd_build(args.variants.split(","))
    else:
        cmd_run(args)


if __name__ == "__main__":
    main()
