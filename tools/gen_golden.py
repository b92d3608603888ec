#!/usr/bin/env python3
"""Generate tests/golden/* from the *reference itself* (oracle/_ref/refharness).

Test infrastructure only.  Needs /root/reference (this container), never runs
on the GPU box.  Every fixture is data: seeded inputs + the outputs the
unmodified reference produced for them, stored as compressed .npz plus a JSON
manifest (flags, seeds, toolchain, output SHA-256s).

    python tools/gen_golden.py            # all cases
    python tools/gen_golden.py --only kat # subset by prefix
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from reflaxman_amd import scenes  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "refharness")
DEFAULT_SEED = 1350490027


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def run(args, env_extra=None):
    env = dict(os.environ)
    env.update({k: str(v) for k, v in (env_extra or {}).items()})
    subprocess.run([HARNESS] + [str(a) for a in args], check=True, env=env)


def render_case(tmp, scene_arg, W, H, depth, ss, additive, frames, sphere_seed, jitter_seed):
    out = os.path.join(tmp, "out")
    run(["render", scene_arg, W, H, depth, ss, int(additive), frames, out],
        {"RFX_SPHERE_SEED": sphere_seed, "RFX_JITTER_SEED": jitter_seed})
    rgb = np.fromfile(out + ".f32", dtype=np.float32).reshape(H, W, 3)
    argb = np.fromfile(out + ".argb", dtype=np.uint32).reshape(H, W)
    return rgb, argb


def band_case(tmp, scene_arg, W, H, depth, y0, rows, sphere_seed):
    out = os.path.join(tmp, "band")
    run(["band", scene_arg, W, H, depth, y0, rows, out], {"RFX_SPHERE_SEED": sphere_seed})
    rgb = np.fromfile(out + ".f32", dtype=np.float32).reshape(rows, W, 3)
    argb = np.fromfile(out + ".argb", dtype=np.uint32).reshape(rows, W)
    return rgb, argb


def banded_frame(tmp, scene_arg, W, H, depth, ss, frame, sphere_seed, workers=None, band_rows=None):
    """Frame `frame` (0-based, non-additive frames, ss x ss samples) of the reference, rendered as row bands by
    parallel `refharness bandss` processes (each advances the random stream over every draw before its band) and
    concatenated.  Used for the full-size hashes the single-threaded reference would take tens of minutes for."""
    from concurrent.futures import ThreadPoolExecutor
    workers = workers or os.cpu_count() or 8
    band_rows = band_rows or max(1, -(-H // (workers * 4)))  # ~4 bands per worker: the cost varies along y
    bands = [(y, min(band_rows, H - y)) for y in range(0, H, band_rows)]
    env = dict(os.environ, RFX_SPHERE_SEED=str(sphere_seed))

    def one(b):
        y0, rows = b
        out = os.path.join(tmp, f"bss_{frame}_{y0}")
        subprocess.run([HARNESS, "bandss", scene_arg, str(W), str(H), str(depth), str(ss), str(frame), str(y0),
                        str(rows), out], check=True, env=env, capture_output=True)
        rgb = np.fromfile(out + ".f32", dtype=np.float32).reshape(rows, W, 3)
        argb = np.fromfile(out + ".argb", dtype=np.uint32).reshape(rows, W)
        os.remove(out + ".f32")
        os.remove(out + ".argb")
        return rgb, argb

    with ThreadPoolExecutor(workers) as ex:
        parts = list(ex.map(one, bands))
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def kat_io(tmp, mode, inp, extra=(), out_dtype=np.float32):
    fi = os.path.join(tmp, "kat.in")
    fo = os.path.join(tmp, "kat.out")
    np.ascontiguousarray(inp, np.float32).tofile(fi)
    if mode in ("kat_skybox", "kat_texture"):
        run([mode, *extra, fi, fo])
    else:
        run([mode, fi, fo, *extra])
    return np.fromfile(fo, dtype=out_dtype)


# ---------------------------------------------------------------- KAT inputs
def sphere_inputs(rng, n=4000):
    o = rng.uniform(-10, 10, (n, 3))
    c = rng.uniform(-10, 10, (n, 3))
    r = rng.uniform(0.05, 4, (n, 1))
    tgt = c + rng.normal(0, 1, (n, 3)) * r * rng.uniform(0, 1.5, (n, 1))  # aim near the sphere
    d = (tgt - o) * rng.choice([1e-3, 1.0, 640.0, 1e10], size=(n, 1))
    rec = np.concatenate([o, d, c, r, np.zeros((n, 1))], axis=1)
    # edge cases: inside, on-surface (DELTA boundary), tangent, away, zero ray, tiny radius, huge shadow rays
    k = n // 8
    rec[:k, 0:3] = rec[:k, 6:9] + rng.normal(0, 0.1, (k, 3)) * rec[:k, 9:10]          # inside
    rec[k:2 * k, 0:3] = rec[k:2 * k, 6:9] + np.array([1, 0, 0]) * (rec[k:2 * k, 9:10] + rng.choice([0, 5e-5, 1e-4, 2e-4], (k, 1)))
    rec[2 * k:3 * k, 3:6] = -rec[2 * k:3 * k, 3:6]                                      # pointing away (mostly)
    rec[3 * k:3 * k + 16, 3:6] = 0                                                      # zero ray
    rec[3 * k + 16:3 * k + 32, 9] = 1e-20                                               # radius clamp
    return rec.astype(np.float32)


def tri_inputs(rng, n=4000):
    v = rng.uniform(-10, 10, (n, 9))
    o = rng.uniform(-10, 10, (n, 3))
    bary = rng.uniform(-0.2, 1.2, (n, 2))
    p = v[:, 0:3] + bary[:, 0:1] * (v[:, 3:6] - v[:, 0:3]) + bary[:, 1:2] * (v[:, 6:9] - v[:, 0:3])
    d = (p - o) * rng.choice([1e-3, 1.0, 640.0, 1e10], size=(n, 1))
    uv = rng.uniform(0, 1, (n, 6))
    rec = np.concatenate([o, d, v, uv], axis=1)
    k = n // 8
    # edges: exactly on an edge in barycentric terms, parallel rays, degenerate triangles, origin on the plane
    e = rec[:k]
    pe = e[:, 6:9] + 0.5 * (e[:, 9:12] - e[:, 6:9])
    e[:, 3:6] = pe - e[:, 0:3]
    rec[k:2 * k, 12:15] = rec[k:2 * k, 6:9] + 1e-4 * rng.normal(0, 1, (k, 3))           # near-degenerate
    nrm = np.cross(rec[2 * k:3 * k, 9:12] - rec[2 * k:3 * k, 6:9], rec[2 * k:3 * k, 12:15] - rec[2 * k:3 * k, 6:9])
    rec[2 * k:3 * k, 3:6] = np.cross(nrm, rng.normal(0, 1, (k, 3)))                    # parallel to plane
    rec[3 * k:3 * k + 32, 0:3] = rec[3 * k:3 * k + 32, 6:9]                            # origin at a vertex
    return rec.astype(np.float32)


def plane_inputs(rng, n=2000):
    o = rng.uniform(-10, 10, (n, 3))
    d = rng.normal(0, 1, (n, 3)) * rng.choice([1e-3, 1.0, 640.0, 1e10], size=(n, 1))
    pos = rng.uniform(-10, 10, (n, 3))
    nn = rng.normal(0, 1, (n, 3))
    rec = np.concatenate([o, d, pos, nn], axis=1)
    k = n // 8
    rec[:k, 3:6] = np.cross(rec[:k, 9:12], rng.normal(0, 1, (k, 3)))                    # parallel
    return rec.astype(np.float32)


def skybox_inputs(rng, n=3000):
    axes = []
    for v in [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1), (1, 1, 0), (1, 0, 1), (0, 1, 1),
              (1, 1, 1), (-1, -1, -1), (-1, 1, 0), (0, -1, 1), (1, 0, -1), (0, 0, 0), (2, 2, 1), (1e-30, 0, 0)]:
        axes.append(v)
    r = rng.normal(0, 1, (n, 3)) * rng.choice([1e-3, 1.0, 1e4], size=(n, 1))
    return np.concatenate([np.array(axes, np.float64), r]).astype(np.float32)


def texture_inputs(rng, n=3000):
    eps = np.float32(1.1920929e-07)
    special = [0.0, 1.0, 1 - eps, 1 - eps / 2, 0.5, 1e-30, -1e-7, 1 + 1e-7, 0.02, 0.98, 0.999999]
    sp = np.array([(a, b) for a in special for b in special], np.float64)
    r = rng.uniform(0, 1, (n, 2))
    return np.concatenate([sp, r]).astype(np.float32)


def argb_inputs(rng, n=4000):
    base = rng.uniform(0, 1, (n, 3))
    k = np.arange(256) / 255.999
    spec = np.stack([k, np.nextafter(k.astype(np.float32), np.float32(2)), np.nextafter(k.astype(np.float32), np.float32(-1))], axis=1)
    big = rng.uniform(1, 40, (64, 3))  # additive sums > 1 (copyImage of an accumulated frame)
    return np.concatenate([base, spec, big, [[0, 0, 0], [1, 1, 1]]]).astype(np.float32)


def camera_inputs(rng, n=200):
    eye = rng.uniform(-20, 20, (n, 3))
    at = eye + rng.normal(0, 1, (n, 3)) * rng.uniform(0.1, 10, (n, 1))
    fov = rng.uniform(0.3, 2.0, (n, 1))
    rows = np.concatenate([eye, at, fov], axis=1)
    rows[0] = [7.427, 3.494, -3.773, 6.5981, 3.127, -3.352, 1.05]
    return rows.astype(np.float32)


def pow_inputs(rng, n=40000):
    # Scene.cpp:175 -- base (2^-63, 1], exponent 1 + 3*refl*|L|/r  (1 .. ~120 for the sun)
    x1 = np.concatenate([rng.uniform(0, 1, n // 2), 10.0 ** rng.uniform(-19, 0, n // 4), [1.0, 0.5, 1e-19]])
    y1 = np.concatenate([rng.uniform(1, 120, n // 2 + n // 4), [1.0, 113.0, 50.0]])
    # Scene.cpp:196 -- base (1 - cos) in [0, 1], exponent 3
    x2 = np.concatenate([rng.uniform(0, 1, n // 4), [0.0, 1.0, 2 ** -24, 1 - 2 ** -24]])
    y2 = np.full(x2.shape, 3.0)
    return np.concatenate([np.stack([x1, y1], 1), np.stack([x2, y2], 1)]).astype(np.float32)


def tga_cases() -> dict:
    """Hand-made TGA files for Texture::loadFromTGAFile (Texture.cpp:34-108): file name -> bytes."""
    import struct
    tex = scenes.synth_texture("t", 5, 3, 5150).argb

    def hdr(idlen=0, cmt=0, itype=2, cmorg=0, cmlen=0, cmbits=0, w=5, h=3, bpp=32, desc=0):
        return struct.pack("<bbbhhbhhhhbb", idlen, cmt, itype, cmorg, cmlen, cmbits, 0, 0, w, h, bpp, desc)

    def px(bpp, a=tex):
        b, g, r, al = a & 0xFF, (a >> 8) & 0xFF, (a >> 16) & 0xFF, (a >> 24) & 0xFF
        ch = [b, g, r, al] if bpp == 32 else [b, g, r]
        return np.stack(ch, -1).astype(np.uint8).tobytes()

    big = scenes.synth_texture("b", 300, 250, 6160).argb  # > 32768 pixels: the reader's buffer refills
    c = {
        "t32.tga": hdr() + px(32),
        "t24.tga": hdr(bpp=24) + px(24),
        "t32_id.tga": hdr(idlen=7) + b"ident!!" + px(32),
        "t24_cmap.tga": hdr(cmlen=4, cmbits=24) + bytes(12) + px(24),
        "t32_origin.tga": hdr(desc=0x20) + px(32),
        "t32_big.tga": hdr(w=300, h=250) + px(32, big),
        "t32_trailing.tga": hdr() + px(32) + b"extra bytes",
        "short_pixels.tga": hdr() + px(32)[:-1],
        "short_header.tga": hdr()[:10],
        "type10.tga": hdr(itype=10) + px(32),
        "bpp16.tga": hdr(bpp=16) + px(32),
        "empty.tga": b"",
        "not_tga.bmp": hdr() + px(32),
        "zero_w.tga": hdr(w=0) + px(32),
    }
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    os.makedirs(GOLDEN, exist_ok=True)
    man_path = os.path.join(GOLDEN, "manifest.json")
    manifest = json.load(open(man_path)) if os.path.exists(man_path) else {"cases": {}}
    manifest["provenance"] = {
        "generator": "tools/gen_golden.py",
        "reference": "/root/reference (BaZzz01010101/ReflaxMan v1 snapshot), src/common/*.cpp unmodified",
        "build": "g++ -std=c++11 -O2 -ffp-contract=off -fno-fast-math -DNDEBUG (oracle/Makefile)",
        "compiler": subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
        "libc": platform.libc_ver(),
        "cpu": platform.processor() or platform.machine(),
        "powf": "glibc 2.35 powf@@GLIBC_2.27 (FMA ifunc variant on this host)",
        "seed_hook": "oracle/ref_seed_shim.h: RFX_SPHERE_SEED -> Vector3.cpp stream, RFX_JITTER_SEED -> Render.cpp stream",
        "generated_unix": int(time.time()),
    }
    cases = manifest["cases"]
    rng = np.random.default_rng(20261015)

    with tempfile.TemporaryDirectory() as tmp:
        sc_dir = os.path.join(tmp, "scenes")
        scene_files = {}
        for name in ("default", "synth16", "synth16_sky", "stress4096", "lights3", "lights40", "nolight", "mesh100",
                     "planes", "planes300"):
            desc = scenes.get_scene(name)
            scene_files[name] = desc.write(sc_dir)

        def want(key):
            return key.startswith(args.only)

        def save_render(key, scene, W, H, depth, ss=1, additive=False, frames=1, seed=DEFAULT_SEED, jseed=0,
                        store=True, use_file=True):
            if not want(key):
                return
            t0 = time.time()
            arg = scene_files[scene] if (use_file or scene != "default") else "default"
            rgb, argb = render_case(tmp, arg, W, H, depth, ss, additive, frames, seed, jseed)
            ent = dict(kind="render", scene=scene, W=W, H=H, depth=depth, ss=ss, additive=additive, frames=frames,
                       sphere_seed=seed, jitter_seed=jseed, sha_f32=sha(rgb.tobytes()), sha_argb=sha(argb.tobytes()),
                       stored=store)
            if store:
                np.savez_compressed(os.path.join(GOLDEN, key + ".npz"), rgb=rgb, argb=argb)
            cases[key] = ent
            print(f"{key}: {time.time() - t0:.1f}s", flush=True)

        # 1. default scene, depths 1/4/8/12 (loadScene path and scene-file path must agree)
        for d in (1, 4, 8, 12):
            save_render(f"render_default_160x120_d{d}", "default", 160, 120, d, use_file=False)
        save_render("render_default_file_160x120_d4", "default", 160, 120, 4, use_file=True)
        save_render("render_default_320x240_d4", "default", 320, 240, 4, use_file=False)
        # 2. SSAA and block preview
        save_render("render_default_160x120_d4_ss2", "default", 160, 120, 4, ss=2, use_file=False)
        save_render("render_default_161x121_d4_ssm4", "default", 161, 121, 4, ss=-4, use_file=False)
        save_render("render_default_160x120_d4_ssm3", "default", 160, 120, 4, ss=-3, use_file=False)
        # SSAA rates of the screenshot menu (Pulse.cpp:24-34) beyond 2x2: the one-lane-per-sample modes (4, 8) and the
        # 64-samples-per-chunk mode (16, 32), additive jitter among them; 3x3 (the per-pixel sample loop) with planes
        save_render("render_default_64x40_d8_ss4", "default", 64, 40, 8, ss=4, use_file=False)
        save_render("render_default_40x24_d6_ss8", "default", 40, 24, 6, ss=8, use_file=False)
        save_render("render_default_17x9_d8_ss16_add2", "default", 17, 9, 8, ss=16, additive=True, frames=2, jseed=5150,
                    use_file=False)
        save_render("render_default_6x5_d4_ss32", "default", 6, 5, 4, ss=32, use_file=False)
        # the top of the menu (64, 128, 256 per axis: 4096 .. 65536 samples per pixel) at the screenshot depth, and 64
        # with additive jitter over two frames
        save_render("render_default_3x2_d20_ss64", "default", 3, 2, 20, ss=64, use_file=False)
        save_render("render_default_2x2_d20_ss128", "default", 2, 2, 20, ss=128, use_file=False)
        save_render("render_default_1x1_d20_ss256", "default", 1, 1, 20, ss=256, use_file=False)
        save_render("render_default_2x1_d8_ss64_add2", "default", 2, 1, 8, ss=64, additive=True, frames=2, jseed=2718,
                    use_file=False)
        save_render("render_planes_40x24_d6_ss3", "planes", 40, 24, 6, ss=3)
        # 3. additive progressive refinement (jitter stream explicit), 3 frames
        save_render("render_default_160x120_d15_add3", "default", 160, 120, 15, additive=True, frames=3,
                    jseed=987654321, use_file=False)
        save_render("render_default_96x64_d4_ss2_add2", "default", 96, 64, 4, ss=2, additive=True, frames=2,
                    jseed=42, use_file=False)
        # 7. a second seed + ragged sizes
        save_render("render_default_160x120_d4_seed2", "default", 160, 120, 4, seed=12345, use_file=False)
        save_render("render_default_1x1_d4", "default", 1, 1, 4, use_file=False)
        save_render("render_default_7x3_d8", "default", 7, 3, 8, use_file=False)
        # 5. synthetic scenes (bilinear TGA textures on planes; skybox atlas)
        save_render("render_synth16_320x180_d8", "synth16", 320, 180, 8)
        save_render("render_synth16_sky_160x90_d8", "synth16_sky", 160, 90, 8)
        # 6. stress
        save_render("render_stress4096_64x36_d12", "stress4096", 64, 36, 12)
        # light loop (3 lights; 40 > 32: the many-lights kernel), no light, > 64 triangles (general object loops),
        # planes (the addPlane extension; the reference's Plane in the reference's Scene::trace)
        save_render("render_lights3_160x90_d8", "lights3", 160, 90, 8)
        save_render("render_lights40_96x54_d8", "lights40", 96, 54, 8)
        save_render("render_nolight_160x120_d4", "nolight", 160, 120, 4)
        save_render("render_mesh100_160x90_d8", "mesh100", 160, 90, 8)
        save_render("render_planes_160x90_d8", "planes", 160, 90, 8)
        save_render("render_planes_64x36_d6_ss2_add2", "planes", 64, 36, 6, ss=2, additive=True, frames=2, jseed=77)
        save_render("render_planes300_96x54_d8", "planes300", 96, 54, 8)
        # large scenes (pair BVH, > 64 triangles) in the one-lane-per-sample and 64-samples-per-chunk SSAA modes
        save_render("render_stress4096_48x27_d12_ss2", "stress4096", 48, 27, 12, ss=2)
        save_render("render_stress4096_24x14_d8_ss4_add2", "stress4096", 24, 14, 8, ss=4, additive=True, frames=2,
                    jseed=31337)
        save_render("render_stress4096_6x4_d8_ss16", "stress4096", 6, 4, 8, ss=16)
        save_render("render_planes300_40x24_d6_ss2", "planes300", 40, 24, 6, ss=2)
        save_render("render_mesh100_40x24_d6_ss2_add2", "mesh100", 40, 24, 6, ss=2, additive=True, frames=2, jseed=9)
        # full-size hashes only (C1, C3; the default 4K d8 too -- SURVEY Appendix B)
        save_render("hash_default_640x480_d4", "default", 640, 480, 4, store=False, use_file=False)
        save_render("hash_synth16_3840x2160_d8", "synth16", 3840, 2160, 8, store=False)
        save_render("hash_default_3840x2160_d8", "default", 3840, 2160, 8, store=False, use_file=False)
        save_render("hash_default_1920x1080_d4", "default", 1920, 1080, 4, store=False, use_file=False)
        # C4: the C3 scene at 7680x4320 d8 (BASELINE configs[3])
        save_render("hash_synth16_7680x4320_d8", "synth16", 7680, 4320, 8, store=False)

        # C2's depth-1 leg (BASELINE configs[1], "primary rays only")
        save_render("hash_default_1920x1080_d1", "default", 1920, 1080, 1, store=False, use_file=False)

        # Full frames the single-threaded reference needs tens of CPU-minutes for, rendered as parallel row bands
        # (refharness bandss) and concatenated.  First the band path is checked against Render::renderNext itself
        # (the render mode) on small frames: SSAA, a second frame of the stream, the large-scene path.
        def save_banded(key, scene, W, H, depth, ss, frames, use_file=True):
            if not want(key):
                return
            arg = scene_files[scene] if (use_file or scene != "default") else "default"
            for (sW, sH, sd, sss, sfr) in ((96, 64, 4, ss, frames), (64, 36, min(depth, 12), 1, 2)):
                rr, ra = render_case(tmp, arg, sW, sH, sd, sss, False, sfr, DEFAULT_SEED, 0)
                br, ba = banded_frame(tmp, arg, sW, sH, sd, sss, sfr - 1, DEFAULT_SEED, band_rows=7)
                assert rr.tobytes() == br.tobytes() and np.array_equal(ra, ba), (key, "bandss != renderNext")
            t0 = time.time()
            rgb, argb = banded_frame(tmp, arg, W, H, depth, ss, frames - 1, DEFAULT_SEED)
            cases[key] = dict(kind="render", scene=scene, W=W, H=H, depth=depth, ss=ss, additive=False, frames=frames,
                              sphere_seed=DEFAULT_SEED, jitter_seed=0, sha_f32=sha(rgb.tobytes()),
                              sha_argb=sha(argb.tobytes()), stored=False,
                              generated="refharness bandss: parallel row bands of Render::renderNext's pixel loop, "
                                        "concatenated; checked equal to the render mode on small frames",
                              cpu_wall_s=round(time.time() - t0, 1))
            print(f"{key}: {time.time() - t0:.1f}s", flush=True)

        # C5 (BASELINE configs[4]) frame 0 and frame 1 (the stream continued), full size
        save_banded("hash_stress4096_3840x2160_d12", "stress4096", 3840, 2160, 12, 1, 1)
        save_banded("hash_stress4096_3840x2160_d12_f2", "stress4096", 3840, 2160, 12, 1, 2)
        # the reference's screenshot workload (Pulse.cpp:156-178: renderBegin(20, ss, false), Full HD, 4x4 SSAA)
        save_banded("hash_default_1920x1080_d20_ss4", "default", 1920, 1080, 20, 4, 1, use_file=False)

        # Screenshots of 2^32 samples and more (the renderer splits them into launches of fewer traces).  The
        # reference's own Pulse would take hours on one core for these, so the frame is banded as above and its BMP is
        # written by the reference's Texture::saveToFile (refharness savetex) from the frame's Color::argb words, which
        # is what Pulse::screenshotRenderSave does (Pulse.cpp:200-205).  The route is first checked against the BMP the
        # reference's Pulse itself wrote at 800x600 2x2 (pulse_screenshot_800x600_ss2).
        def shot_bmp(argb, W, H):
            src, fn = os.path.join(tmp, "shot.u32"), os.path.join(tmp, "shot.bmp")
            np.ascontiguousarray(argb, np.uint32).tofile(src)
            subprocess.run([HARNESS, "savetex", str(W), str(H), src, fn], check=True, capture_output=True)
            return open(fn, "rb").read()

        def save_shot(key, res_key, ss_key, W, H, ss, heavy=False):
            if not want(key) or (heavy and args.only != key):  # heavy: only when asked for by its full name
                return
            ref = cases["pulse_screenshot_800x600_ss2"]
            _, a2 = banded_frame(tmp, "default", 800, 600, 20, 2, 0, ref["RFX_SPHERE_SEED"])
            assert sha(shot_bmp(a2, 800, 600)) == ref["sha_bmp"], "banded frame + savetex != the reference Pulse's BMP"
            t0 = time.time()
            workers = int(os.environ.get("RFX_GEN_WORKERS", "0")) or None  # leave cores free for other work
            rgb, argb = banded_frame(tmp, "default", W, H, 20, ss, 0, ref["RFX_SPHERE_SEED"], workers=workers)
            data = shot_bmp(argb, W, H)
            cases[key] = dict(kind="pulse", res_key=res_key, ss_key=ss_key, W=W, H=H, ss=ss, depth=20, bytes=len(data),
                              sha_bmp=sha(data), file=ref["file"], RFX_SPHERE_SEED=ref["RFX_SPHERE_SEED"],
                              RFX_JITTER_SEED=ref["RFX_JITTER_SEED"], sha_f32=sha(rgb.tobytes()),
                              sha_argb=sha(argb.tobytes()), samples=W * H * ss * ss,
                              generated="refharness bandss (parallel row bands of Render::renderNext's pixel loop) + "
                                        "refharness savetex; route checked against pulse_screenshot_800x600_ss2",
                              cpu_wall_s=round(time.time() - t0, 1))
            print(f"{key}: {time.time() - t0:.1f}s", flush=True)

        # 800x600 at 128x128 (menu keys 1 and 8): 7.9e9 samples
        save_shot("pulse_screenshot_800x600_ss128", 1, 8, 800, 600, 128)
        # the screenshot the reference's ReadMe shows (ReadMe.md:30-32): Full HD (key 8) at 128x128 (key 8), 3.4e10 samples
        # (about 4 hours on this container's 8 cores: generated only with --only pulse_screenshot_1920x1080_ss128)
        save_shot("pulse_screenshot_1920x1080_ss128", 8, 8, 1920, 1080, 128, heavy=True)

        # C4 band: 4 rows at the middle of the 8K frame (stream advanced over the 2160 rows above)
        key = "band_synth16_7680x4320_d8_y2160_r4"
        if want(key):
            t0 = time.time()
            rgb, argb = band_case(tmp, scene_files["synth16"], 7680, 4320, 8, 2160, 4, DEFAULT_SEED)
            np.savez_compressed(os.path.join(GOLDEN, key + ".npz"), rgb=rgb, argb=argb)
            cases[key] = dict(kind="band", scene="synth16", W=7680, H=4320, depth=8, y0=2160, rows=4,
                              sphere_seed=DEFAULT_SEED, sha_f32=sha(rgb.tobytes()), sha_argb=sha(argb.tobytes()))
            print(f"{key}: {time.time() - t0:.1f}s", flush=True)

        # file formats: the bytes Texture::saveToFile writes (BMP, TGA) and what Texture::loadFromFile reads
        # back from hand-made TGA files (24/32 bpp, id field, colour-map fields, origin bit, broken files)
        if want("file"):
            img = scenes.synth_texture("img", 7, 5, 99).argb
            src = os.path.join(tmp, "img.u32")
            img.tofile(src)
            outs = {}
            for ext in ("bmp", "tga", "png"):
                fn = os.path.join(tmp, "out." + ext)
                r = subprocess.run([HARNESS, "savetex", "7", "5", src, fn], check=True, capture_output=True, text=True)
                ok = int(r.stdout.strip())
                outs[ext] = (ok, np.fromfile(fn, np.uint8) if ok else np.zeros(0, np.uint8))
            np.savez_compressed(os.path.join(GOLDEN, "file_save.npz"), argb=img, bmp=outs["bmp"][1], tga=outs["tga"][1],
                                ok=np.array([outs["bmp"][0], outs["tga"][0], outs["png"][0]], np.int32))
            cases["file_save"] = dict(kind="file", what="Texture(7, 5) + saveToFile(.bmp / .tga / .png)")
            loads = {}
            for name, data in tga_cases().items():
                fn = os.path.join(tmp, name)
                open(fn, "wb").write(data)
                fo = os.path.join(tmp, "load.out")
                run(["loadtex", fn, fo])
                loads[name] = (data, np.fromfile(fo, np.uint32))
            arrays = {}
            for i, (name, (data, out)) in enumerate(sorted(loads.items())):
                arrays[f"in{i}"] = np.frombuffer(data, np.uint8)
                arrays[f"out{i}"] = out
            np.savez_compressed(os.path.join(GOLDEN, "file_load.npz"), names=np.array(sorted(loads)), **arrays)
            cases["file_load"] = dict(kind="file", what="Texture::loadFromFile on hand-made TGA files",
                                      names=sorted(loads))
            print("file fixtures", flush=True)

        # the reference's own application controller (Pulse.cpp, unmodified, headless platform) taking a
        # screenshot through its menus: 800x600 (key 1), SSAA 2x2 (key 2), depth 20 -- the BMP file's SHA-256
        if want("pulse"):
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import pulse_build
            exe = pulse_build.build("reference", os.path.join(tmp, "pulse_ref"))
            shot = os.path.join(tmp, "shot") + "/"
            os.makedirs(shot)
            seeds = {"RFX_SPHERE_SEED": DEFAULT_SEED, "RFX_JITTER_SEED": 424238335}
            r = subprocess.run([exe, shot, "1", "2"], check=True, capture_output=True, text=True,
                               env={**os.environ, **{k: str(v) for k, v in seeds.items()}})
            data = open(r.stdout.strip(), "rb").read()
            cases["pulse_screenshot_800x600_ss2"] = dict(kind="pulse", res_key=1, ss_key=2, W=800, H=600, ss=2,
                                                         depth=20, bytes=len(data), sha_bmp=sha(data),
                                                         file=os.path.basename(r.stdout.strip()), **seeds)
            print("pulse screenshot", flush=True)

        # an interactive session of the same Pulse (still frames, a key press that abandons a frame, motion frames in
        # block preview, release, deceleration, still frames again): the hash of every completed frame as the window
        # reads it.  TICK 1000 us keeps sampleNum at -1 (a fast renderer's path); 2000 us walks it down to -8.
        if want("pulse_session"):
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import pulse_build
            exe = pulse_build.build("reference", os.path.join(tmp, "pulse_ref_s"))
            seeds = {"RFX_SPHERE_SEED": DEFAULT_SEED, "RFX_JITTER_SEED": 424238335}
            for tick in (1000, 2000):
                W, H = 640, 480
                r = subprocess.run([exe, tmp + "/", "session", str(W), str(H), str(tick)], check=True,
                                   capture_output=True, text=True, env={**os.environ, **{k: str(v) for k, v in seeds.items()}})
                frames = [l.split() for l in r.stdout.splitlines() if l.startswith("frame ")]
                cases[f"pulse_session_{W}x{H}_tick{tick}"] = dict(
                    kind="pulse_session", W=W, H=H, tick_us=tick, execs=[int(f[3]) for f in frames],
                    hashes=[f[7] for f in frames], **seeds)
                print(f"pulse session tick {tick}: {len(frames)} frames", flush=True)

        # stress bands (4K width) with stream advance
        for y0 in (0, 1080):
            key = f"band_stress4096_3840x2160_d12_y{y0}_r4"
            if want(key):
                t0 = time.time()
                rgb, argb = band_case(tmp, scene_files["stress4096"], 3840, 2160, 12, y0, 4, DEFAULT_SEED)
                np.savez_compressed(os.path.join(GOLDEN, key + ".npz"), rgb=rgb, argb=argb)
                cases[key] = dict(kind="band", scene="stress4096", W=3840, H=2160, depth=12, y0=y0, rows=4,
                                  sphere_seed=DEFAULT_SEED, sha_f32=sha(rgb.tobytes()), sha_argb=sha(argb.tobytes()))
                print(f"{key}: {time.time() - t0:.1f}s", flush=True)

        # 8. KATs
        def save_kat(key, **arrays):
            np.savez_compressed(os.path.join(GOLDEN, key + ".npz"), **arrays)
            cases[key] = dict(kind="kat", arrays=sorted(arrays))
            print(key, flush=True)

        if want("kat"):
            out = os.path.join(tmp, "rand.bin")
            run(["rand", 20000, out], {"RFX_SPHERE_SEED": DEFAULT_SEED})
            save_kat("kat_rand", seed=np.array([DEFAULT_SEED], np.uint32),
                     dirs=np.fromfile(out, np.float32).reshape(-1, 3))
            rec = sphere_inputs(rng)
            save_kat("kat_sphere", inp=rec, out=kat_io(tmp, "kat_sphere", rec).reshape(-1, 15))
            rec = tri_inputs(rng)
            save_kat("kat_triangle", inp=rec, out=kat_io(tmp, "kat_triangle", rec).reshape(-1, 15))
            tex = scenes.synth_texture("kat", 64, 48, 31337).argb
            scenes.write_tga(os.path.join(tmp, "kat.tga"), tex)
            save_kat("kat_triangle_tex", inp=rec, tex=tex,
                     out=kat_io(tmp, "kat_triangle", rec, extra=[os.path.join(tmp, "kat.tga")]).reshape(-1, 15))
            save_kat("kat_triangle_checker", inp=rec,
                     out=kat_io(tmp, "kat_triangle", rec, extra=["-"]).reshape(-1, 15))
            rec = plane_inputs(rng)
            save_kat("kat_plane", inp=rec, out=kat_io(tmp, "kat_plane", rec).reshape(-1, 15))
            rays = skybox_inputs(rng)
            save_kat("kat_skybox_checker", inp=rays, out=kat_io(tmp, "kat_skybox", rays, extra=["-"]).reshape(-1, 3))
            sky = scenes.synth_texture("sky", 256, 192, 4242).argb
            scenes.write_tga(os.path.join(tmp, "sky.tga"), sky)
            save_kat("kat_skybox_tex", inp=rays, tex=sky,
                     out=kat_io(tmp, "kat_skybox", rays, extra=[os.path.join(tmp, "sky.tga")]).reshape(-1, 3))
            uv = texture_inputs(rng)
            save_kat("kat_texture_checker", inp=uv, out=kat_io(tmp, "kat_texture", uv, extra=["-"]).reshape(-1, 3))
            save_kat("kat_texture_tex", inp=uv, tex=tex,
                     out=kat_io(tmp, "kat_texture", uv, extra=[os.path.join(tmp, "kat.tga")]).reshape(-1, 3))
            # 24-bpp TGA path (alpha forced to 0xFF by the loader)
            scenes.write_tga(os.path.join(tmp, "kat24.tga"), tex, bpp=24)
            save_kat("kat_texture_tex24", inp=uv, tex=(tex & 0x00FFFFFF) | 0xFF000000,
                     out=kat_io(tmp, "kat_texture", uv, extra=[os.path.join(tmp, "kat24.tga")]).reshape(-1, 3))
            cols = argb_inputs(rng)
            save_kat("kat_argb", inp=cols, out=kat_io(tmp, "kat_argb", cols, out_dtype=np.uint32))
            cam = camera_inputs(rng)
            save_kat("kat_camera", inp=cam, out=kat_io(tmp, "kat_camera", cam).reshape(-1, 9))
            pw = pow_inputs(rng)
            save_kat("kat_pow", inp=pw, out=kat_io(tmp, "kat_pow", pw))

        # record the scene-file hashes so generator drift is detected
        manifest["scene_sha256"] = {n: sha(open(p, "rb").read()) for n, p in scene_files.items()}

    json.dump(manifest, open(man_path, "w"), indent=1, sort_keys=True)
    total = sum(os.path.getsize(os.path.join(GOLDEN, f)) for f in os.listdir(GOLDEN))
    print(f"golden dir: {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
