#!/usr/bin/env python3
"""bench.py -- Mrays/s of ReflaxMan's per-pixel trace loop on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1..c5|shot|shot128]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` (N > 1) without a launcher starts the N ranks itself (a torch.distributed.run child job, rendezvous on
127.0.0.1) and exits with its code; under a launcher, --gpus must equal WORLD_SIZE (else exit 2).

Workload (BASELINE.json metric "Mrays/sec at 3840x2160 depth-8"): at N = 1 config
C3 -- the synth16 scene (16 spheres, ground + back-wall quads = 4 textured
triangles, the default sun light => shadow rays), 3840x2160, depth 8, 1 spp,
synthetic 512x512 TGA textures.  A step is one full frame of the hot path
(Render::renderBegin + renderNext(W*H)): the RNG pre-pass, the trace kernel and
the ARGB8 epilogue, inputs and outputs resident in HBM.  Every step renders
the *next* frame of the reference's global random stream, as the reference app
does.

N > 1: config C4 (BASELINE configs[3]) -- the C3 scene at a FIXED 7680x4320 d8
frame (strong scaling; --scaling weak grows the frame with N instead).  The
default partition is contiguous row bands, load-balanced from measured per-rank
trace times (BandFrame.balance) and received in place on rank 0 over RCCL p2p
(xGMI); --partition strips deals block-cyclic 8-row strips instead, gathered
and un-interleaved on rank 0.  The RNG pre-pass is sliced too: each rank counts
1/N of the random stream and one all-gather of ~1K block counts follows; that
count, the all-gather and the next frame's emit run a frame ahead on a side
stream (count-ahead / emit-ahead), and frame i's band transfer runs while frame
i+1 renders (--no-pipeline, --no-count-ahead, --no-emit-ahead turn these off).
value = traces of the whole frame / step time (max over ranks).  Rank 0 also
times the same C4 frame on its own GPU in the same run (the strong-scaling
baseline; the other ranks wait at a barrier) and checks both the first frame
and a steady-state frame after the timed loop against single-GPU renders.
Note: the driver's N = 1 point is C3 (3840x2160), not C4.

Also reported: the trace kernel's executed VALU lane-op rate against the
78.6 T lane-op/s peak (roofline, from the rocprofv3 --pmc record of the same
workload and library build) next to the reference-equivalent algorithmic
TFLOP/s, its HIP-event time, full-frame parity (SHA-256 of the first frame vs
the reference's, tests/golden/manifest.json), and the reference's own CPU path
timed on a bounded sample of the same frame on one host core.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec at 3840×2160 depth-8; max per-channel |Δ| vs CPU reference"
SEED = 1350490027


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# BASELINE.json configs (and the reference's screenshot workload): scene, width, height, depth, samples per pixel
# (ss x ss), description
CONFIGS = {
    "c1": ("default", 640, 480, 4, 1, "C1 default scene (Render::loadScene, textures absent -> checker)"),
    "c2": ("default", 1920, 1080, 4, 1, "C2 default scene"),
    "c3": ("synth16", 3840, 2160, 8, 1, "C3 synth16: 16 spheres + 4 textured triangles + sun"),
    "c4": ("synth16", 7680, 4320, 8, 1, "C4 synth16 (the C3 scene: 16 spheres + 4 textured triangles + sun)"),
    "c5": ("stress4096", 3840, 2160, 12, 1, "C5 stress4096: 4096 spheres + ground quad + sun"),
    "shot": ("default", 1920, 1080, 20, 4, "screenshot: Render's default scene, Full HD, 4x4 SSAA, depth 20 "
                                           "(Pulse.cpp:156-178, defaults.h:9)"),
    "shot128": ("default", 1920, 1080, 20, 128, "the reference's ReadMe screenshot (ReadMe.md:30-32): Render's default "
                                                "scene, Full HD, 128x128 SSAA, depth 20 (Pulse.cpp:10-34,156-178): "
                                                "3.4e10 samples per frame, rendered as launches of 2^30 traces"),
}
# cpu_baseline row strides: about 5 s of the reference's single-core trace time per config (C5's CPU rate is
# 0.0064 Mrays/s: every 270th row); SSAA configs time a band of rows instead: (first row or None = centred, rows).
# shot128's band is its first row (31.5 M samples, ~28 s on one core): a centred band would first advance the random
# stream over 1.7e10 draws.
CPU_STRIDE = {"c1": 1, "c2": 4, "c3": 2, "c4": 16, "c5": 270}
CPU_BAND_ROWS = {"shot": (None, 160), "shot128": (0, 1)}
# full-frame parity keys of configs whose manifest case is not named hash_<scene>_<W>x<H>_d<depth>_ss<ss>
PARITY_CASE = {"shot128": "pulse_screenshot_1920x1080_ss128"}
# steps / warmup when not given: a shot128 frame takes ~1.5 s
DEFAULT_STEPS = {"shot128": (3, 1)}


def frame_size(n: int, w0: int, h0: int, scaling: str):
    if n == 1 or scaling == "strong":
        return w0, h0
    s = math.sqrt(n)
    return int(round(w0 * s)), int(round(h0 * s))


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def ulp_diff(a: np.ndarray, b: np.ndarray) -> int:
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, np.int64(-2 ** 31) - ai, ai)
    bi = np.where(bi < 0, np.int64(-2 ** 31) - bi, bi)
    return int(np.abs(ai - bi).max()) if a.size else 0


def ulp_hist(a: np.ndarray, b: np.ndarray) -> dict:
    """Histogram of per-channel float ULP distances (buckets 0, 1, 2-15, 16-255, >=256)."""
    ai = a.reshape(-1).view(np.int32).astype(np.int64)
    bi = b.reshape(-1).view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, np.int64(-2 ** 31) - ai, ai)
    bi = np.where(bi < 0, np.int64(-2 ** 31) - bi, bi)
    d = np.abs(ai - bi)
    edges = [("0", 0, 0), ("1", 1, 1), ("2-15", 2, 15), ("16-255", 16, 255), (">=256", 256, None)]
    return {k: int(((d >= lo) & (d <= hi)).sum()) if hi is not None else int((d >= lo).sum()) for k, lo, hi in edges}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def u8_diff(a: np.ndarray, b: np.ndarray) -> int:
    ch = lambda x, s: ((x >> s) & 0xFF).astype(np.int32)
    return int(max(np.abs(ch(a, s) - ch(b, s)).max() for s in (0, 8, 16))) if a.size else 0


def cpu_baseline_band(desc, W, H, depth, ss, gpu_rgb, gpu_argb, rows, y0=None):
    """SSAA frames: the reference's CPU path (oracle/_ref/refharness bandss, Render::renderNext's pixel loop over the
    unmodified sources) on a band of `rows` rows of the same frame (centred unless y0 is given), one host core; the
    band is also compared with the GPU frame's."""
    harness = os.path.join(ROOT, "oracle", "_ref", "refharness")
    if not os.path.exists(harness):
        return None, None
    y0 = (H - rows) // 2 if y0 is None else y0
    with tempfile.TemporaryDirectory() as tmp:
        scene_path = desc.write(tmp)
        out = os.path.join(tmp, "band")
        r = subprocess.run([harness, "bandss", scene_path, str(W), str(H), str(depth), str(ss), "0", str(y0), str(rows),
                            out], env={**os.environ, "RFX_SPHERE_SEED": str(SEED)}, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            raise RuntimeError("refharness failed: " + r.stderr)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        rgb = np.fromfile(out + ".f32", np.float32).reshape(rows, W, 3)
        argb = np.fromfile(out + ".argb", np.uint32).reshape(rows, W)
    secs, n = info["trace_seconds"], info["traced_samples"]
    g_rgb, g_argb = gpu_rgb[y0:y0 + rows], gpu_argb[y0:y0 + rows]
    return {
        "value": round(n / secs / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "reference",
        "sample": f"rows {y0}..{y0 + rows - 1} ({rows} x {W} px x {ss * ss} samples) of the first frame; {secs:.1f} s "
                  f"of single-thread trace time; {cpu_model()}; "
                  f"{subprocess.run(['nproc'], capture_output=True, text=True).stdout.strip()} host CPUs visible",
    }, {"max_u8": u8_diff(g_argb, argb), "max_f32_ulp": ulp_diff(g_rgb, rgb), "f32_ulp_histogram": ulp_hist(g_rgb, rgb),
        "pixels": int(W * rows)}


def cpu_baseline(desc, W, H, depth, gpu_rgb, gpu_argb, stride):
    """The reference's CPU path (oracle/_ref/refharness, the unmodified sources) on every `stride`-th row of
    the same frame, one host core; its rows are also compared with the GPU frame's."""
    harness = os.path.join(ROOT, "oracle", "_ref", "refharness")
    count = (H + stride - 1) // stride
    with tempfile.TemporaryDirectory() as tmp:
        scene_path = desc.write(tmp)
        out = os.path.join(tmp, "rows")
        if os.path.exists(harness):
            kind = "reference"
            r = subprocess.run([harness, "rows", scene_path, str(W), str(H), str(depth), "0", str(stride), str(count), out],
                               env={**os.environ, "RFX_SPHERE_SEED": str(SEED)}, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                raise RuntimeError("refharness failed: " + r.stderr)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            rgb = np.fromfile(out + ".f32", np.float32).reshape(count, W, 3)
            argb = np.fromfile(out + ".argb", np.uint32).reshape(count, W)
            secs, px = info["trace_seconds"], info["traced_pixels"]
        else:  # no reference build on this host: the C restatement (bit-exact port), one thread, contiguous band
            kind = "port"
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as orc
            count = min(count, 256)
            y0 = (H - count) // 2
            t0 = time.perf_counter()
            rgb, argb = orc.render_band(desc, W, H, depth, y0, count, SEED, nthreads=1)
            secs, px = time.perf_counter() - t0, W * count
            stride, ys = 1, slice(y0, y0 + count)
    ys = slice(0, count * stride, stride) if kind == "reference" else ys
    g_rgb, g_argb = gpu_rgb[ys], gpu_argb[ys]
    sample = (f"rows 0,{stride},..,{(count - 1) * stride} ({count} x {W} px) of the first frame" if kind == "reference"
              else f"rows {ys.start}..{ys.stop - 1} of the first frame")
    return {
        "value": round(px / secs / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": kind,
        "sample": f"{sample}; {secs:.1f} s of single-thread trace time; {cpu_model()}; "
                  f"{subprocess.run(['nproc'], capture_output=True, text=True).stdout.strip()} host CPUs visible",
    }, {"max_u8": u8_diff(g_argb, argb), "max_f32_ulp": ulp_diff(g_rgb, rgb),
        "f32_ulp_histogram": ulp_hist(g_rgb, rgb), "pixels": int(px)}


def cpu_allcore(desc, W, H, depth, gpu_rgb, gpu_argb, rate_1core, seconds=8.0):
    """Context row (BASELINE.md:59-62, not the speedup denominator): the C restatement (bit-exact port) with
    its rows interleaved over every host thread this job may use, on a centred band sized from the 1-core
    rate to take about `seconds`; the band is also compared with the GPU frame's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    threads = max(1, min(64, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))
    rows = int(min(H, max(threads, rate_1core * 1e6 * threads * seconds / W)))
    y0 = (H - rows) // 2
    t0 = time.perf_counter()
    rgb, argb = orc.render_band(desc, W, H, depth, y0, rows, SEED, nthreads=threads)
    secs = time.perf_counter() - t0
    g = slice(y0, y0 + rows)
    same = bool(np.array_equal(gpu_rgb[g].view(np.uint32), rgb.view(np.uint32)) and np.array_equal(gpu_argb[g], argb))
    return {"value": round(W * rows / secs / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"rows {y0}..{y0 + rows - 1} of the first frame, rows interleaved over {threads} threads, "
                      f"{secs:.1f} s; {cpu_model()}", "bit_exact_vs_gpu": same}


def one_gpu_line(cfg_name, W, H, depth):
    """The committed 1-GPU bench line of the same frame (the newest profiles/rNN/configs/), a cross-check of the
    strong-scaling baseline this run measures itself, or None."""
    import glob
    dirs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "configs")), reverse=True)  # newest round
    for d in dirs:
        line = _one_gpu_line_in(d, cfg_name, W, H, depth)
        if line:
            return line
    return None


def _one_gpu_line_in(d, cfg_name, W, H, depth):
    for name in sorted(os.listdir(d)):
        if not name.startswith(cfg_name + "_") or not name.endswith(".json"):
            continue
        try:
            rec = json.loads(open(os.path.join(d, name)).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        c = rec.get("config", {})
        if rec.get("n_gpus") == 1 and (c.get("width"), c.get("height"), c.get("depth")) == (W, H, depth):
            return {"value": rec["value"], "unit": rec["unit"], "ms_per_step": rec["ms_per_step"],
                    "source": os.path.relpath(os.path.join(d, name), ROOT)}
    return None


class SingleGpu:
    """Rank 0's single-GPU renderer of the multi-rank frame (N > 1): the parity renders (the first frame and the
    steady-state frame, each from its stream state) and the strong-scaling baseline measured in the same run."""

    def __init__(self, Renderer, scene, frame, W, H, dev, stream):
        import torch
        self.torch = torch
        self.r = Renderer(device=dev.index, sphere_seed=SEED)
        self.r.set_scene(scene)
        self.r.set_stream(stream.cuda_stream)
        self.frame, self.stream = frame, stream
        self.img = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
        self.argb = torch.zeros(H * W, dtype=torch.int32, device=dev)

    def _frame(self):
        self.r.render_frame(self.frame, self.img.data_ptr(), self.argb.data_ptr(), 0, self.stream.cuda_stream)

    def render(self, sphere_seed: int):
        """The frame whose random stream starts at sphere_seed (synchronised)."""
        self.r.set_rng(sphere_seed, 0)
        self._frame()
        self.torch.cuda.synchronize()
        return self.img, self.argb

    def time(self, steps: int, warmup: int, prewarm_s: float, traces: int) -> dict:
        """Mrays/s of the whole frame on this GPU alone: untimed clock-ramp and warmup frames, then `steps` frames
        bracketed by synchronize (the bench's own 1-GPU step: pre-pass + trace + epilogue)."""
        sync = self.torch.cuda.synchronize
        sync()
        t = time.perf_counter()
        n = 0
        while time.perf_counter() - t < prewarm_s or n < warmup:
            self._frame()
            sync()
            n += 1
        t0 = time.perf_counter()
        for _ in range(steps):
            self._frame()
        sync()
        el = time.perf_counter() - t0
        return {"value": round(traces * steps / el / 1e6, 2), "unit": "Mrays/s", "ms_per_step": round(el / steps * 1e3, 4),
                "steps": steps, "untimed_frames_before": n,
                "kind": "measured in this run: rank 0 renders the same full frame on its GPU alone, the other ranks "
                        "waiting at a barrier"}

    def close(self):
        self.r.close()


def times_c4_denominator(world: int, cfg_name: str, custom: bool, no_c4: bool) -> bool:
    """Does this line carry c4_1gpu -- the C4 frame timed on one GPU in the same run?  The driver's default N = 1 line
    (C3) does, so that a scaling curve over the N > 1 lines (C4) has a same-config denominator."""
    return world == 1 and cfg_name == "c3" and not custom and not no_c4


LAUNCH_TRACES = 1 << 30  # rfx_host.cpp RFX_LAUNCH_TRACES (the library's default launch limit)


def split_launches(W: int, H: int, ss: int) -> int:
    """Launches rfx_render_frame makes of a W x H frame at ss x ss samples (rfx_host.cpp render_split)."""
    spp = ss * ss
    if W * H * spp <= LAUNCH_TRACES:
        return 1
    per = max(1, LAUNCH_TRACES // spp)
    if per >= W:
        per = per // W * W
        return -(-H // (per // W))
    return -(-(W * H) // per)


def launcher_command(n: int, argv: list, port: int) -> list:
    """The command that runs this bench as n ranks of one node (torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(n: int, argv: list) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run the N ranks as a child torch.distributed.run job and
    return its exit code; rank 0's JSON line reaches this process's stdout directly.  Nothing in this process has
    touched the GPU (torch is not even imported here), so the ranks own their devices."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = launcher_command(n, argv, port)
    log("launching", n, "ranks:", " ".join(cmd))
    return subprocess.run(cmd).returncode


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (GPUs of one node); N > 1 without WORLD_SIZE in the environment starts the N ranks "
                         "itself (torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=None, help="timed frames (default 50; shot128: 3)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed frames before them (default 5; shot128: 1)")
    ap.add_argument("--prewarm-ms", type=float, default=250.0,
                    help="untimed frames for about this long before the warmup steps (GPU clock ramp); 0: none")
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="BASELINE config (default: c3 on one GPU, c4 on more; shot: the reference's screenshot)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="N > 1: the config's fixed frame (strong) or a frame grown with N at its aspect (weak)")
    ap.add_argument("--scene", default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--ss", type=int, default=None, help="samples per pixel ss x ss (SSAA; default: the config's)")
    ap.add_argument("--no-first-view", action="store_true", help="N = 1: skip the first-view timing")
    ap.add_argument("--no-c4", action="store_true", help="N = 1 (C3): skip the same-run C4 frame (c4_1gpu)")
    ap.add_argument("--gather-rgb", action="store_true", help="N > 1: gather the float RGB strips to rank 0 too")
    ap.add_argument("--regroup", type=int, default=None,
                    help="ray regrouping: park traces after n segments (0 off; default: the library's choice)")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--cpu-stride", type=int, default=None,
                    help="cpu_baseline samples every n-th row (default per config: a ~5 s single-core sample)")
    ap.add_argument("--no-cpu-allcore", action="store_true", help="skip the all-core CPU context row")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (gloo: multi-rank rehearsal)")
    ap.add_argument("--one-device", action="store_true", help="all ranks on cuda:0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--no-pipeline", action="store_true", help="N > 1: gather each frame's strips before the next frame")
    ap.add_argument("--partition", choices=["bands", "strips"], default="bands",
                    help="N > 1: load-balanced contiguous bands received in place on rank 0 (default), or block-cyclic "
                         "row strips gathered and un-interleaved")
    ap.add_argument("--no-emit-ahead", action="store_true",
                    help="N > 1: emit each frame's randDirs on its critical path, not during the last trace")
    ap.add_argument("--no-count-ahead", action="store_true",
                    help="N > 1: count and all-gather each frame's RNG blocks on its critical path, not during the last trace")
    args = ap.parse_args(argv)

    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus is not None and args.gpus > 1 and world_env is None:
        return launch_ranks(args.gpus, argv)
    world = int(world_env or "1")
    if args.gpus is not None and args.gpus != world:
        log(f"--gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure another number of GPUs than asked")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    cfg_name = args.config or ("c3" if world == 1 else "c4")
    d_steps, d_warmup = DEFAULT_STEPS.get(cfg_name, (50, 5))
    args.steps = d_steps if args.steps is None else args.steps
    args.warmup = d_warmup if args.warmup is None else args.warmup
    c_scene, c_w, c_h, c_depth, c_ss, c_desc = CONFIGS[cfg_name]
    custom = any(v is not None for v in (args.scene, args.width, args.height, args.depth, args.ss))
    args.scene = args.scene or c_scene
    args.width = args.width or c_w
    args.height = args.height or c_h
    args.depth = args.depth or c_depth
    args.ss = args.ss or c_ss
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", str(rank)))

    import torch
    import torch.distributed as dist
    from reflaxman_amd import _lib, metrics, scenes
    from reflaxman_amd.render import Renderer, build_scene, make_frame

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    L = _lib.load()

    W, H = frame_size(world, args.width, args.height, args.scaling)
    depth, rb, ss = args.depth, args.row_block, args.ss
    if world > 1 and args.partition == "strips" and W * H * ss * ss > (1 << 31):
        raise SystemExit("bench.py: frames of more than 2^31 traces run as row-span passes of bands (--partition bands)")
    desc = scenes.get_scene(args.scene)
    scene, cam = build_scene(desc)
    rr = Renderer(device=local, sphere_seed=SEED)
    rr.set_scene(scene)
    if args.regroup is not None:
        rr.set_regroup(args.regroup)
    # one non-default stream, current for torch (collectives, copies) and passed to librfx (a NULL stream
    # would select the renderer's own non-blocking stream, unordered with torch's work)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    rr.set_stream(stream.cuda_stream)

    bands = world > 1 and args.partition == "bands"
    frame = make_frame(cam, W, H, depth, ss, row_block=rb if world > 1 and not bands else 0, rank=rank, nranks=world)
    traces = W * H * ss * ss  # one Scene::trace per sample (Render.cpp:181-187)
    if world > 1:
        # sliced RNG pre-pass (count own slice -> all-gather block counts -> emit own strips), trace of
        # the own strips, ARGB8 strip gather to rank 0 + device un-interleave (reflaxman_amd/dist.py)
        from reflaxman_amd.dist import BandFrame, RfxStripOps, StripFrame
        ops = RfxStripOps(rr, frame, stream.cuda_stream)
        common = dict(pipeline=False if args.no_pipeline else None, gather_rgb=args.gather_rgb,
                      count_ahead=False if args.no_count_ahead else None,
                      emit_ahead=False if args.no_emit_ahead else None)
        sf = BandFrame(ops, W, H, rank, world, dev, ss=ss, **common) if bands else \
            StripFrame(ops, W, H, rb, rank, world, dev, **common)
        rows, img, argb = sf.rows, sf.img, sf.argb
    else:
        rows = H
        img = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
        argb = torch.zeros(H * W, dtype=torch.int32, device=dev)
    log(f"rank {rank}/{world}: {args.scene} {W}x{H} d{depth}, strip rows {rows}")

    def step():
        if world > 1:
            return sf.step()
        rr.render_frame(frame, img.data_ptr(), argb.data_ptr(), 0, stream.cuda_stream)
        return None

    # ---- frame 0 (from the reference's default seed): parity evidence + event counts
    full0 = step()
    torch.cuda.synchronize()
    parity = {}
    one = None  # rank 0 at N > 1: a single-GPU renderer of the same frame (parity checks, strong-scaling baseline)
    if world > 1 and rank == 0:
        # the assembled multi-rank frame must equal a single-GPU render of the same frame (untimed)
        one = SingleGpu(Renderer, scene, make_frame(cam, W, H, depth, ss), W, H, dev, stream)
        img1, argb1 = one.render(SEED)
        parity["multi_rank_frame_equals_single_gpu"] = bool(torch.equal(full0.reshape(-1), argb1))
        if args.gather_rgb:
            parity["multi_rank_rgb_equals_single_gpu"] = bool(torch.equal(sf.rgb_full.reshape(-1), img1))
        man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))["cases"]
        key = f"hash_{args.scene}_{W}x{H}_d{depth}" + (f"_ss{ss}" if ss != 1 else "")
        key = PARITY_CASE.get(cfg_name, key) if not custom else key
        if key in man:
            parity["multi_rank_frame_vs_reference_sha256"] = {
                "argb8": sha(full0.reshape(-1).cpu().numpy().view(np.uint32).tobytes()) == man[key]["sha_argb"],
                "case": key}
        if os.environ.get("RFX_BENCH_DUMP"):
            np.save(os.path.join(os.environ["RFX_BENCH_DUMP"], "multi.npy"), full0.cpu().numpy())
            np.save(os.path.join(os.environ["RFX_BENCH_DUMP"], "single.npy"), argb1.view(H, W).cpu().numpy())
    first_rgb = first_argb = None
    if world == 1:
        first_rgb = img.view(H, W, 3).cpu().numpy()
        first_argb = argb[: H * W].view(H, W).cpu().numpy().view(np.uint32)
        man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))["cases"]
        key = f"hash_{args.scene}_{W}x{H}_d{depth}" + (f"_ss{ss}" if ss != 1 else "")
        key = PARITY_CASE.get(cfg_name, key) if not custom else key
        if key in man:
            ok_f = sha(first_rgb.tobytes()) == man[key]["sha_f32"]
            ok_a = sha(first_argb.tobytes()) == man[key]["sha_argb"]
            parity["full_frame_vs_reference_sha256"] = {"f32": ok_f, "argb8": ok_a, "case": key}
    # counted frames (the stats kernel) into scratch buffers at N > 1 (the step buffers may still be in pipelined
    # sends); each advances the random stream itself, on every rank
    cimg, cargb = (torch.empty_like(img), torch.empty_like(argb)) if world > 1 else (img, argb)

    def counted_frame():
        c = torch.zeros(_lib.RFX_NCOUNTERS, dtype=torch.int64, device=dev)
        if world > 1:
            sf.drop_lookahead()
        if world > 1 and bands and sf.passes:
            sf.step(c.data_ptr())  # a frame of row-span passes: the counters sum the passes' band launches
        else:
            rr.render_frame(frame, cimg.data_ptr(), cargb.data_ptr(), c.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        return c

    counters = counted_frame()
    cnt = counters.cpu().numpy().astype(np.uint64)
    if world > 1:
        c = torch.tensor(cnt.astype(np.int64), device=dev)
        dist.all_reduce(c)
        cnt = c.cpu().numpy().astype(np.uint64)
    work = metrics.summary(cnt)
    flops_frame = work["flops"]

    # ---- clock ramp: untimed frames for ~args.prewarm_ms before the W warmup steps (a few short frames leave the
    # GPU below its steady clock: C3 trace 0.766 ms after 2 warmup frames vs 0.721 ms after 50, same box).  The
    # count is rank 0's estimate, shared so that every rank runs the same collectives.
    prewarm = 0
    if args.prewarm_ms > 0:
        torch.cuda.synchronize()
        t_est = time.perf_counter()
        step()
        torch.cuda.synchronize()
        est = max(time.perf_counter() - t_est, 1e-5)
        prewarm = int(min(2000, args.prewarm_ms * 1e-3 / est))
        if world > 1:
            pw = torch.tensor([prewarm], dtype=torch.int64, device=dev)
            dist.broadcast(pw, 0)
            prewarm = int(pw.item())
        for _ in range(prewarm):
            step()
    flops_local = None
    if bands:
        # cut the bands from measured per-rank render times (rank 0's receive included), then keep them
        sf.balance(rounds=3, frames=8)
        log(f"rank {rank}: bands {sf.bounds}")
        # this rank's work in its final band, for the per-launch roofline
        flops_local = metrics.summary(counted_frame().cpu().numpy().astype(np.uint64))["flops"]
    # ---- warmup, then K timed steps (barrier + synchronize on both sides)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    rr.get_timing()
    # HIP events on every n-th timed frame (at least 5 samples): three event records per frame cost ~10 us of C1's
    # ~50 us frame, so timing every frame would slow the frames it measures
    timing_every = max(1, min(8, args.steps // 5))
    rr.set_timing(timing_every)
    if world > 1:
        sf.time_emits(True)
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    pre_ms, trace_ms, nfr = rr.get_timing()
    rr.set_timing(False)
    emit_side = None
    if world > 1:
        emit_side = sf.time_emits(False)  # ms per look-ahead emit on the side stream (None without emit-ahead)
        if emit_side is not None:
            pre_ms = emit_side * nfr  # the emit ran beside the trace, off the critical path
        t = torch.tensor([elapsed, trace_ms / max(nfr, 1), pre_ms / max(nfr, 1)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, trace_avg, pre_avg = t.tolist()
    else:
        trace_avg, pre_avg = trace_ms / max(nfr, 1), pre_ms / max(nfr, 1)

    steady = baseline = None
    if world > 1:
        # steady-state parity: one more step down the same path (look-aheads, masks, schedule, pipelined transfer),
        # against a single-GPU render of the same frame of the stream (its start state is the pending frame's)
        torch.cuda.synchronize()
        start = ops.rng_pending()
        fullk = step()
        torch.cuda.synchronize()
        if rank == 0:
            _, argbk = one.render(start)
            steady = {"frame": "the step after the timed steps (same path: look-aheads, masks, schedule, pipelined "
                               "transfer)", "stream_state_at_frame_start": start,
                      "equals_single_gpu": bool(torch.equal(fullk.reshape(-1), argbk))}
        # strong-scaling baseline measured in this run: rank 0 renders the same full frame on its own GPU while the
        # other ranks wait at the barrier
        if rank == 0:
            baseline = one.time(args.steps, args.warmup, prewarm_s=args.prewarm_ms * 1e-3, traces=traces)
        dist.barrier()
        if rank == 0:
            one.close()

    e2e = None
    if world == 1:
        # end to end with the frame handed back to the host: reported beside `value`, never as it.
        # (1) the display path: the ARGB8 plane (what a window shows, Pulse.cpp:455-458) of frame i copied to pinned
        #     host memory on a copy stream while frame i + 1 renders into the other of two device frame sets;
        # (2) both planes (f32 RGB + ARGB8) copied after each frame, serially.
        n_e2e = min(args.steps, 10)
        sets = [(img, argb), (torch.empty_like(img), torch.empty_like(argb))]
        h_argb = [torch.empty(argb.numel(), dtype=argb.dtype, pin_memory=True) for _ in range(2)]
        copy = torch.cuda.Stream(device=dev)
        done = [torch.cuda.Event(), torch.cuda.Event()]
        copied = [torch.cuda.Event(), torch.cuda.Event()]
        for e in done + copied:
            e.record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(n_e2e):
            k = i % 2
            stream.wait_event(copied[k])  # set k's last frame has reached the host
            rr.render_frame(frame, sets[k][0].data_ptr(), sets[k][1].data_ptr(), 0, stream.cuda_stream)
            done[k].record(stream)
            copy.wait_event(done[k])
            with torch.cuda.stream(copy):
                h_argb[k].copy_(sets[k][1], non_blocking=True)
            copied[k].record(copy)
        torch.cuda.synchronize()
        ovl_s = (time.perf_counter() - t1) / n_e2e
        h_rgb = torch.empty(img.numel(), dtype=img.dtype, pin_memory=True)
        h_argb1 = torch.empty(argb.numel(), dtype=argb.dtype, pin_memory=True)
        t1 = time.perf_counter()
        for _ in range(n_e2e):
            step()
            h_rgb.copy_(img, non_blocking=True)
            h_argb1.copy_(argb, non_blocking=True)
            torch.cuda.current_stream().synchronize()
        e2e_s = (time.perf_counter() - t1) / n_e2e
        # the r01/r02 keys keep their meaning (both planes, serial); the overlapped display path has its own key
        e2e = {"ms_per_frame": round(e2e_s * 1e3, 4), "Mrays_per_s": round(traces / e2e_s / 1e6, 2),
               "d2h_bytes_per_frame": int(img.numel() * 4 + argb.numel() * 4), "frames": n_e2e,
               "kind": "both planes (f32 RGB + ARGB8) to pinned host memory after each frame, serially",
               "overlapped_argb8": {"ms_per_frame": round(ovl_s * 1e3, 4), "Mrays_per_s": round(traces / ovl_s / 1e6, 2),
                                    "d2h_bytes_per_frame": int(argb.numel() * 4),
                                    "kind": "ARGB8 plane to pinned host memory, frame i's copy overlapped with frame "
                                            "i+1's render (the display path)"}}
        del sets

    first_view = None
    if world == 1 and not args.no_first_view:
        # what a view pays before the per-view state exists (the headline value is a still camera's steady state):
        # per-view primary masks off (a camera that moves every frame never has them), then also the tile schedule
        # reset to raster order (the very first frame of a grid, before any tile cost was measured)
        def new_view_step():
            # the renderer forgets the views it has seen (rfx_renderer_set_prim_masks clears them), so every frame is a
            # view's first: no per-view masks, except the chunk mode's, which are built for every view
            rr.set_prim_masks(1)
            step()

        def rate(n):
            for _ in range(3):
                new_view_step()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(n):
                new_view_step()
            torch.cuda.synchronize()
            el = (time.perf_counter() - t1) / n
            return {"ms_per_step": round(el * 1e3, 4), "value": round(traces / el / 1e6, 2)}
        n_fv = max(5, min(args.steps, 20))
        moving = rate(n_fv)
        rr.set_tile_order(0)
        cold = rate(n_fv)
        rr.set_tile_order(1)
        rr.set_prim_masks(1)
        first_view = {"unit": "Mrays/s", "frames": n_fv,
                      "moving_camera": {**moving, "kind": "every frame a view not seen before: no per-view primary masks "
                                                          "(built only when a view repeats; the chunk mode's per-pixel "
                                                          "masks are built for every view); tile schedule learned from "
                                                          "earlier frames of the grid"},
                      "cold": {**cold, "kind": "no per-view masks and raster tile order: a view's first frame before "
                                               "any per-view or per-grid state exists"},
                      "note": "value (above) is the steady state of a still camera: masks built on its second frame, "
                              "longest-first schedule from earlier frames' tile costs"}

    c4_1gpu = None
    if times_c4_denominator(world, cfg_name, custom, args.no_c4):
        # the denominator of a scaling curve: N > 1 lines render C4 (7680x4320), the N = 1 line C3 (3840x2160), so the
        # C4 frame is also timed here on this GPU, same steps and warmup, and checked against the reference's hash
        s4, w4, h4, d4, _, _ = CONFIGS["c4"]
        sc4, cam4 = build_scene(scenes.get_scene(s4))
        one4 = SingleGpu(Renderer, sc4, make_frame(cam4, w4, h4, d4, 1), w4, h4, dev, stream)
        _, argb4 = one4.render(SEED)
        man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))["cases"]
        key4 = f"hash_{s4}_{w4}x{h4}_d{d4}"
        ok4 = sha(argb4.cpu().numpy().view(np.uint32).tobytes()) == man[key4]["sha_argb"] if key4 in man else None
        c4_1gpu = one4.time(args.steps, args.warmup, prewarm_s=args.prewarm_ms * 1e-3, traces=w4 * h4)
        c4_1gpu.update({"config": f"C4 {s4} {w4}x{h4} d{d4}, 1 spp", "frame_vs_reference_sha256": {"argb8": ok4,
                                                                                                  "case": key4},
                        "kind": "the C4 frame (the N > 1 lines' fixed frame) on this GPU alone in this run: the "
                                "same-config denominator of value(N) / (N value(1))"})
        one4.close()
        del one4

    rgb_gather = None
    if world > 1 and bands and not args.gather_rgb:
        # the drop-in's path reads the float image (Render::imagePixel): the same bands with the f32 RGB plane sent to
        # rank 0 too (16 B/px instead of 4), timed the same way, reported beside the ARGB8-only value
        sf.set_gather_rgb(True)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        el = float(el.item())
        sf.set_gather_rgb(False)
        rgb_gather = {"value": round(traces * args.steps / el / 1e6, 2), "unit": "Mrays/s",
                      "ms_per_step": round(el / args.steps * 1e3, 4), "steps": args.steps,
                      "bytes_to_rank0_per_px": 16,
                      "kind": "bands with the f32 RGB plane gathered to rank 0 as well as ARGB8 (what a caller that "
                              "reads Render::imagePixel needs); same bands, same timing bracket"}

    if rank != 0:
        dist.destroy_process_group()
        return

    ms_step = elapsed / args.steps * 1e3
    mrays = traces * args.steps / elapsed / 1e6
    # the trace kernel of one rank processes its strip: per-launch FLOPs = frame FLOPs / world (balanced strips)
    # (bands: rank 0's counted work in its final band; strips: an equal share, the strips being balanced)
    if world > 1:
        rows = sf.rows
    flops_launch = flops_local if flops_local is not None else flops_frame / world
    achieved = flops_launch / (trace_avg * 1e-3) / 1e12
    px_launch = rows * W
    # HBM traffic and executed VALU work of the trace kernel: rocprofv3 --pmc passes of this very workload
    # and library build (tools/prof_round.sh -> profiles/pmc/), per launch; null when no such record exists
    pmc = metrics.pmc_record(os.path.join(ROOT, "profiles", "pmc"), [args.scene, W, H, depth, world, ss],
                             _lib.lib_sha256(), _lib.device_sha256())
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    passes = len(sf.passes) if world > 1 and bands and sf.passes else 0
    launches = split_launches(W, H, ss) if world == 1 else max(1, passes)
    if launches > 1 and world == 1:
        # a frame of several launches on two overlapping streams: a launch's HIP-event span includes the other stream's
        # work, so the per-launch time is the frame's wall time shared out over its launches
        trace_avg = ms_step / launches
        flops_launch = flops_frame / launches
        px_launch = W * H // launches
    elif launches > 1:
        # row-span passes (N > 1): rank 0 traces one band per pass, each timed by HIP events on its stream
        flops_launch = flops_launch / launches
        px_launch = sf.rows * W // launches
    executed = metrics.executed_work(pmc, trace_avg)
    roofline = metrics.roofline(executed, traffic, flops_launch, trace_avg, px_launch)
    if launches > 1:
        roofline["launches_per_frame"] = launches
        roofline["launch_time_kind"] = ("frame wall time / launches (the split frame's launches overlap on two streams)"
                                        if world == 1 else "rank 0's band launch of each row-span pass (HIP events)")
    roofline["kernel"] = ("rfx::trace_kernel (plain pixel mode, wave-bundle culling)" if ss == 1 else
                          "rfx::trace_kernel (SSAA pixel mode, wave-bundle culling)")
    if baseline is not None:
        baseline["efficiency"] = round(mrays / (world * baseline["value"]), 4)
    workload = (c_desc if not custom else f"{args.scene} scene") + f", {W}x{H}, depth {depth}, {ss * ss} spp"
    if world > 1:
        workload += f", {world} GPUs, fixed frame (strong scaling)" if args.scaling == "strong" else \
            f", {world} GPUs, frame grown with N (weak scaling)"
    out = {
        "metric": METRIC, "value": round(mrays, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "prewarm_frames": prewarm, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": workload, "name": None if custom else cfg_name.upper(),
                   "scene": args.scene, "width": W, "height": H, "depth": depth, "spp": ss * ss,
                   "parallelism": ((f"balanced-bands-x{world}" if bands else f"row-strips{rb}x{world}")
                                   + ("+pipelined-gather" if sf.pipeline else "")
                                   + ("+count-ahead" if sf.count_ahead else "")
                                   + ("+emit-ahead" if sf.emit_ahead else "")
                                   + (f"+row-span-passes-x{passes}" if passes else "")) if world > 1 else "single-gpu"},
        "roofline": roofline,
        "phases_ms": {"rng_prepass": round(pre_avg, 4), "trace": round(trace_avg, 4), "timed_every_nth_frame": timing_every,
                      **({"rng_prepass_kind": "look-ahead emit on the side stream, beside the previous trace (HIP "
                                              "events on that stream): off the critical path"}
                         if emit_side is not None else {}),
                      **({"split_kind": f"{launches} launches per frame on two streams: rng_prepass is the mean "
                                        "pre-pass per launch, timed on its stream while the other stream's trace holds "
                                        "the chip (so it spans most of that trace, off the critical path); trace is "
                                        "the frame's wall time / launches"}
                         if launches > 1 else {})},
        "work_per_ray": {k: round(v, 3) for k, v in work.items() if k != "flops"},
        # SURVEY §8(d) secondary metric: bounce segments + shadow rays per second (counted, frame 0's rates)
        "secondary_Msegments_per_s": round((work["segments_per_ray"] + work["shadow_rays_per_ray"]) * traces
                                           * args.steps / elapsed / 1e6, 1),
        "end_to_end_incl_d2h": e2e,
        **({"first_view": first_view} if first_view else {}),
        **({"c4_1gpu": c4_1gpu} if c4_1gpu else {}),
        **({"with_rgb_gather": rgb_gather} if rgb_gather else {}),
        "parity": parity,
        **({"band_bounds": sf.bounds} if bands else {}),
        **({"steady_state_parity": steady,
            "efficiency": baseline["efficiency"] if baseline else None,
            "efficiency_kind": "value / (N x strong_scaling_baseline.value): the same frame on one GPU of this run "
                               "(for C4, the driver's N = 1 line carries the same measurement as c4_1gpu)",
            "strong_scaling_baseline": baseline,
            "strong_scaling_baseline_committed": one_gpu_line(cfg_name, W, H, depth),
            "scale_note": (f"N > 1 renders {cfg_name.upper()} ({W}x{H}); the driver's N = 1 bench point is C3 "
                           "(3840x2160), whose line carries c4_1gpu, the C4 frame on one GPU in that run: efficiency "
                           "here is against strong_scaling_baseline, the same frame on one GPU of this run")}
           if world > 1 else {}),
    }
    if world == 1 and not args.no_cpu_baseline:
        log("cpu_baseline: reference CPU path on a row sample of the same frame ...")
        if ss != 1:
            y0b, nrows = CPU_BAND_ROWS.get(cfg_name, (None, 16)) if not custom else (None, 16)
            cb, delta = cpu_baseline_band(desc, W, H, depth, ss, first_rgb, first_argb, nrows, y0b)
        else:
            stride = args.cpu_stride or (2 if custom else CPU_STRIDE[cfg_name])
            cb, delta = cpu_baseline(desc, W, H, depth, first_rgb, first_argb, stride)
        out["cpu_baseline"] = cb  # None: an SSAA frame on a host without the reference build
        if cb is not None:
            out["parity"]["sample_vs_cpu_reference"] = delta
            out["max_abs_delta"] = {"u8": delta["max_u8"], "f32_ulp": delta["max_f32_ulp"]}
            out["speedup_vs_cpu_1core"] = round(mrays / cb["value"], 1)
        if cb is not None and not args.no_cpu_allcore and ss == 1:
            log("cpu_allcore: the C restatement on every host thread (context row) ...")
            out["cpu_allcore"] = cpu_allcore(desc, W, H, depth, first_rgb, first_argb, cb["value"])
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
