"""Frames of any sample count: spans of more traces than one launch takes render as consecutive launches
(rfx_render_frame, include/rfx.h) and a device group's frame as consecutive row-span passes (rfx_group_render_frame).

The reference traces every sample of every pixel serially with no trace count (Render.cpp:136-215, Pulse.cpp:10-34 offers
SSAA up to 256x256 at up to 7680x4320), so a frame's pixels and both random streams must come out the same whatever the
launch size.  Small frames are forced through the split with tiny launch limits and compared with the reference's
stored frames (SSAA 2..256, additive jitter, accumulation, the per-pixel sample loop, a large scene); the full-size case
is a 800x600 128x128 screenshot (7.9e9 samples, over 2^32) hashed against the reference's banded frame.
"""
import ctypes as C
import os

import numpy as np
import pytest

from helpers import GOLDEN, gpu_render, manifest, sha
from reflaxman_amd import _lib, scenes

pytestmark = pytest.mark.gpu
CASES = manifest()["cases"]


def _golden(key):
    return np.load(os.path.join(GOLDEN, key + ".npz"))


@pytest.mark.parametrize("key,limit,chunks", [
    ("render_default_160x120_d4", 5000, None),             # whole-row launches (31 rows)
    ("render_default_160x120_d4", 100, None),              # launches of 100 pixels: spans start mid-row
    ("render_default_160x120_d15_add3", 3000, None),       # additive jitter, accumulation over 3 frames
    ("render_default_160x120_d4_ss2", 4 * 700, None),      # one lane per sample, 2x2
    ("render_default_64x40_d8_ss4", 16 * 50, None),        # 4x4, spans cutting the lanes' pixel blocks
    ("render_default_40x24_d6_ss8", 64 * 30, None),        # 8x8
    ("render_default_17x9_d8_ss16_add2", 256 * 5, None),   # 64-sample chunks, additive over 2 frames
    ("render_default_6x5_d4_ss32", 1024 * 4, None),
    ("render_planes_40x24_d6_ss3", 9 * 100, None),         # the per-pixel sample loop, planes
    ("render_default_3x2_d20_ss64", 4096, None),           # one pixel per launch
    ("render_default_2x2_d20_ss128", 1, None),             # a limit below one pixel: still one pixel per launch
    ("render_default_1x1_d20_ss256", 1, None),
    ("render_default_2x1_d8_ss64_add2", 4096, None),
    ("render_stress4096_48x27_d12_ss2", 4 * 200, None),    # the pair BVH per lane
    ("render_default_160x120_d4_ss2", 4 * 700, [7, 1000, 13]),  # Pulse-style chunks, each split again
])
def test_split_launches_equal_reference(key, limit, chunks):
    c = CASES[key]
    rgb, argb, r = gpu_render(scenes.get_scene(c["scene"]), c["W"], c["H"], c["depth"], c["ss"], c["additive"],
                              c["frames"], c["sphere_seed"], c.get("jitter_seed", 0), chunks=chunks, launch_traces=limit)
    g = _golden(key)
    assert np.array_equal(argb, g["argb"]), key
    assert rgb.tobytes() == g["rgb"].tobytes(), key
    r.close()


@pytest.mark.parametrize("key", ["render_default_3x2_d20_ss64", "render_default_2x2_d20_ss128",
                                 "render_default_1x1_d20_ss256", "render_default_2x1_d8_ss64_add2"])
def test_top_menu_rates_chunked(key):
    """SSAA 64/128/256 (the top of Pulse's menu) one renderNext pixel at a time, at the default launch limit."""
    c = CASES[key]
    rgb, argb, r = gpu_render(scenes.get_scene(c["scene"]), c["W"], c["H"], c["depth"], c["ss"], c["additive"],
                              c["frames"], c["sphere_seed"], c.get("jitter_seed", 0), chunks=[1])
    g = _golden(key)
    assert np.array_equal(argb, g["argb"]) and rgb.tobytes() == g["rgb"].tobytes(), key
    r.close()


def _renderer(scene, seed=1350490027, jitter=99):
    from reflaxman_amd.render import Renderer
    r = Renderer(sphere_seed=seed, jitter_seed=jitter)
    r.set_scene(scene)
    return r


def test_split_streams_counters_and_rewind():
    """A split frame leaves both random streams where one launch leaves them, counts the same events (stats kernel),
    and rfx_frame_rng_rewind returns both streams to the frame's start (the saved start state, not a seed flip)."""
    import torch
    from reflaxman_amd.render import build_scene, make_frame
    scene, cam = build_scene(scenes.get_scene("default"))
    W, H = 96, 64
    f = make_frame(cam, W, H, 6, 4, additive=True, additive_counter=1)
    out = {}
    for limit in (0, 16 * 333):
        r = _renderer(scene)
        r.set_launch_traces(limit)
        start = r.get_rng()
        rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
        argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(_lib.RFX_NCOUNTERS, dtype=torch.int64, device="cuda")
        r.render_frame(f, rgb.data_ptr(), argb.data_ptr(), cnt.data_ptr())
        r.synchronize()
        end = r.get_rng()
        assert end != start
        _lib.check(_lib.load().rfx_frame_rng_rewind(r._h))
        assert r.get_rng() == start, limit
        # the rewound frame renders again to the same pixels
        rgb2 = torch.zeros_like(rgb)
        r.render_frame(f, rgb2.data_ptr(), 0)
        r.synchronize()
        assert torch.equal(rgb, rgb2) and r.get_rng() == end
        out[limit] = (rgb.cpu().numpy().tobytes(), argb.cpu().numpy().tobytes(), end, cnt.cpu().numpy().tolist())
        r.close()
    assert out[0] == out[16 * 333]


def test_split_frame_on_a_device_group():
    """A device group's frame of more traces than one pass takes (3 members on device 0, launch limit forced low):
    consecutive row-span passes with the random stream continued, equal to the single renderer's frames over 3 frames
    (4x4 SSAA, additive accumulation), then rewound on member 0 and rendered again."""
    import torch
    from reflaxman_amd.render import build_scene, make_frame
    scene, cam = build_scene(scenes.get_scene("default"))
    W, H = 200, 150
    L = _lib.load()
    g = C.c_void_p()
    devs = (C.c_int * 3)(0, 0, 0)
    _lib.check(L.rfx_group_create(C.byref(g), devs, 3), "group_create")
    _lib.check(L.rfx_group_set_scene(g, scene._h))
    r0 = C.c_void_p(L.rfx_group_renderer(g, 0))
    _lib.check(L.rfx_renderer_set_rng(r0, 1350490027, 99))
    _lib.check(L.rfx_renderer_set_launch_traces(r0, 16 * 200 * 7))  # passes of 3 x 7 rows, the last one shorter
    one = _renderer(scene)
    rgb, argb = torch.zeros(H * W * 3, device="cuda"), torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rgb1, argb1 = torch.zeros_like(rgb), torch.zeros_like(argb)
    for k in range(1, 4):
        f = make_frame(cam, W, H, 5, 4, additive=True, additive_counter=k)
        _lib.check(L.rfx_group_render_frame(g, C.byref(f), C.c_void_p(rgb.data_ptr()), C.c_void_p(argb.data_ptr()),
                                            None), "group_render_frame")
        one.render_frame(f, rgb1.data_ptr(), argb1.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(rgb, rgb1) and torch.equal(argb, argb1), k
    # rewind the last group frame on member 0 (the saved start state) and render a fresh non-additive frame from it
    _lib.check(L.rfx_frame_rng_rewind(r0))
    _lib.check(L.rfx_frame_rng_rewind(one._h))
    f = make_frame(cam, W, H, 5, 4)
    _lib.check(L.rfx_group_render_frame(g, C.byref(f), C.c_void_p(rgb.data_ptr()), C.c_void_p(argb.data_ptr()), None))
    one.render_frame(f, rgb1.data_ptr(), argb1.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(rgb, rgb1) and torch.equal(argb, argb1)
    L.rfx_group_destroy(g)
    one.close()


def test_group_passes_narrower_than_the_group():
    """Split group frames whose passes hold fewer rows than members (3 members, passes of 2 rows, the last of 1): the
    members a pass leaves out keep an older stream state, so the next pass -- and the next whole frame, which takes
    every member -- must hand member 0's state over again.  Two split frames, then two frames in one pass, each equal
    to the single renderer's."""
    import torch
    from reflaxman_amd.render import build_scene, make_frame
    scene, cam = build_scene(scenes.get_scene("default"))
    W, H, ss = 40, 9, 4
    L = _lib.load()
    g = C.c_void_p()
    devs = (C.c_int * 3)(0, 0, 0)
    _lib.check(L.rfx_group_create(C.byref(g), devs, 3), "group_create")
    _lib.check(L.rfx_group_set_scene(g, scene._h))
    r0 = C.c_void_p(L.rfx_group_renderer(g, 0))
    _lib.check(L.rfx_renderer_set_rng(r0, 1350490027, 99))
    one = _renderer(scene)
    rgb, argb = torch.zeros(H * W * 3, device="cuda"), torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rgb1, argb1 = torch.zeros_like(rgb), torch.zeros_like(argb)
    for k, limit in enumerate([W * ss * ss * 2 // 3, W * ss * ss * 2 // 3, 0, 0]):
        _lib.check(L.rfx_renderer_set_launch_traces(r0, limit))  # 3 x limit traces per pass: 2 rows, then 1 row
        f = make_frame(cam, W, H, 6, ss)
        _lib.check(L.rfx_group_render_frame(g, C.byref(f), C.c_void_p(rgb.data_ptr()), C.c_void_p(argb.data_ptr()),
                                            None), "group_render_frame")
        one.render_frame(f, rgb1.data_ptr(), argb1.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(rgb, rgb1) and torch.equal(argb, argb1), k
    L.rfx_group_destroy(g)
    one.close()


@pytest.mark.parametrize("case", ["pulse_screenshot_800x600_ss128", "pulse_screenshot_1920x1080_ss128"])
def test_screenshot_over_2_32_samples(case):
    """800x600 at 128x128 samples, depth 20 (Pulse's menu keys 1 and 8): 7.9e9 samples in one rfx_render_frame, split
    into launches at the default limit; and the reference's ReadMe screenshot, 1920x1080 at 128x128 (3.4e10 samples).
    SHA-256 of the floats and the ARGB8 image equal the reference's frame (tools/gen_golden.py, banded refharness)."""
    c = CASES[case]
    assert c["samples"] >= 1 << 32
    rgb, argb, r = gpu_render(scenes.get_scene("default"), c["W"], c["H"], c["depth"], c["ss"],
                              sphere_seed=c["RFX_SPHERE_SEED"])
    assert sha(argb) == c["sha_argb"]
    assert sha(rgb) == c["sha_f32"]
    r.close()


@pytest.mark.parametrize("nranks,launch_traces", [(2, 0), (4, 0), (8, 800 * 128 * 128 * 3 // 8)])
def test_rank_passes_assemble_the_screenshot(nranks, launch_traces):
    """The multi-process path's SSAA frames (reflaxman_amd/dist.py BandFrame row-span passes) with the ranks emulated
    in one process: the 800x600 128x128 screenshot (7.9e9 samples) as passes over row spans (dist.pass_plan: 2^31
    traces per pass; with 8 ranks and a launch limit of 3/8 row, passes of 3 rows, so 5 of 8 ranks sit every pass out
    and take rank 0's stream state), each span cut into equal bands (dist.pass_bands), every rank counting every slice
    of the span's stream (the all-gather emulated), each band emitted and traced into its rank's whole-frame buffers
    and copied into one frame as rank 0 receives it: SHA-256 of the f32 and ARGB8 frames equal the reference's."""
    import torch
    from reflaxman_amd import dist as rdist
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    c = CASES["pulse_screenshot_800x600_ss128"]
    W, H, depth, ss = c["W"], c["H"], c["depth"], c["ss"]
    lt = launch_traces or rdist.LAUNCH_TRACES
    plan = rdist.pass_plan(W, H, ss, nranks, lt)
    assert plan and len(plan) > 1
    s, cam = build_scene(scenes.get_scene("default"))
    L = _lib.load()
    rs = [Renderer(sphere_seed=c["RFX_SPHERE_SEED"]) for _ in range(nranks)]
    for r in rs:
        r.set_scene(s)
    fr = [make_frame(cam, W, H, depth, ss, row_block=0, rank=k, nranks=nranks) for k in range(nranks)]
    bufs = [(torch.zeros(H * W * 3, device="cuda"), torch.zeros(H * W, dtype=torch.int32, device="cuda"))
            for _ in range(nranks)]
    img = torch.zeros(H * W * 3, device="cuda")
    argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    cnt = None
    sat_out = 0
    for y0, y1 in plan:
        bd = rdist.pass_bands(y0, y1, nranks)
        m = len(bd) - 1
        for k in range(nranks):
            fr[k].span_begin, fr[k].span_end = y0 * W, y1 * W
            a, b = rdist.pass_rows(bd, k, y1)
            fr[k].pixel_begin, fr[k].pixel_end = a * W, b * W
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(rs[0]._h, C.byref(fr[0]), nranks, C.byref(bps)))
        if cnt is None:  # the first pass is the largest
            cnt = [torch.zeros(nranks * bps.value, dtype=torch.int32, device="cuda") for _ in range(nranks)]
        for k in range(nranks):
            for sl in range(nranks):
                _lib.check(L.rfx_frame_rng_count(rs[k]._h, C.byref(fr[k]), sl, nranks, C.c_void_p(cnt[k].data_ptr()),
                                                 None), "rng_count")
        for k in range(m):
            _lib.check(L.rfx_render_frame_counted(rs[k]._h, C.byref(fr[k]), nranks, C.c_void_p(cnt[k].data_ptr()),
                                                  C.c_void_p(bufs[k][0].data_ptr()), C.c_void_p(bufs[k][1].data_ptr()),
                                                  None, None), "render_frame_counted")
        if m < nranks:
            sat_out += 1
            st = rs[0].get_rng()
            for k in range(m, nranks):
                rs[k].set_rng(*st)
        for k in range(m):
            rs[k].synchronize()
            img[bd[k] * W * 3:bd[k + 1] * W * 3] = bufs[k][0][bd[k] * W * 3:bd[k + 1] * W * 3]
            argb[bd[k] * W:bd[k + 1] * W] = bufs[k][1][bd[k] * W:bd[k + 1] * W]
    torch.cuda.synchronize()
    assert (sat_out > 0) == (launch_traces != 0)
    assert sha(argb.cpu().numpy().view(np.uint32)) == c["sha_argb"]
    assert sha(img.cpu().numpy()) == c["sha_f32"]
    for r in rs:
        r.close()
