"""Shared helpers: drive the GPU renderer and the CPU oracle on the same case."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    return json.load(open(os.path.join(GOLDEN, "manifest.json")))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gpu_render(desc, W, H, depth, ss=1, additive=False, frames=1, sphere_seed=1350490027, jitter_seed=0,
               chunks=None, device=0, tile_order=None, each_frame=None, regroup=None, prim_masks=None,
               regroup_sort=None, launch_traces=None):
    """Render through the Python mirror of Render (reflaxman_amd.render.Render) on the GPU.

    chunks: None -> one renderNext(W*H) per frame; else a list of renderNext sizes cycled until done.
    Returns (imagePixels float32 HxWx3, copyImage ARGB HxW, renderer)."""
    from reflaxman_amd.render import Render, build_scene
    r = Render(device=device, sphere_seed=sphere_seed, jitter_seed=jitter_seed, load_default_scene=False)
    r.scene, r.camera = build_scene(desc)
    r.setImageSize(W, H)
    if tile_order is not None:
        r._r.set_tile_order(tile_order)
    if regroup is not None:
        r._r.set_regroup(regroup)
    if regroup_sort is not None:
        r._r.set_regroup_sort(regroup_sort)
    if prim_masks is not None:
        r._r.set_prim_masks(prim_masks)
    if launch_traces is not None:
        r._r.set_launch_traces(launch_traces)
    for _ in range(frames):
        r.renderBegin(depth, ss, additive)
        if chunks is None:
            while r.renderNext(W * H):
                pass
        else:
            i = 0
            while r.renderNext(chunks[i % len(chunks)]):
                i += 1
        if each_frame is not None:
            r.synchronize()
            each_frame(r.imagePixels(), r.copyImage())
    r.synchronize()
    return r.imagePixels(), r.copyImage(), r
