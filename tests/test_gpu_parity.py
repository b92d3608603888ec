"""GPU parity: the HIP renderer (through librfx.so's C-ABI) against the reference.

Bit-exact bar: the f32 framebuffer and the ARGB8 image must equal, byte for
byte, what the unmodified reference produced (tests/golden/, made by
oracle/_ref) -- at small sizes directly, at full BASELINE sizes by SHA-256 --
and what the CPU restatement (oracle/) produces on the same seeded inputs.
Float tolerance is therefore 0 ULP (the north star allows <= 1 ULP).
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, gpu_render, manifest, sha
from reflaxman_amd import scenes

pytestmark = pytest.mark.gpu

CASES = manifest()["cases"]
_SCENES = {}


def scene(name):
    if name not in _SCENES:
        _SCENES[name] = scenes.get_scene(name)
    return _SCENES[name]


def run_case(c, **kw):
    return gpu_render(scene(c["scene"]), c["W"], c["H"], c["depth"], c["ss"], c["additive"], c["frames"],
                      c["sphere_seed"], c.get("jitter_seed", 0), **kw)


@pytest.mark.parametrize("key", sorted(k for k, c in CASES.items() if c["kind"] == "render" and c.get("stored")))
def test_golden_bitexact(key):
    c = CASES[key]
    rgb, argb, r = run_case(c)
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    diff = argb != g["argb"]
    assert not diff.any(), f"{key}: {diff.sum()} ARGB8 pixels differ, first at {np.argwhere(diff)[:3].tolist()}"
    ulp = np.abs(rgb.view(np.int32).astype(np.int64) - g["rgb"].view(np.int32).astype(np.int64))
    assert ulp.max() == 0, f"{key}: max float ULP {ulp.max()} ({(ulp > 0).sum()} channels)"
    r.close()


@pytest.mark.parametrize("key", ["hash_default_640x480_d4", "hash_default_1920x1080_d1", "hash_default_1920x1080_d4",
                                 "hash_synth16_3840x2160_d8", "hash_default_3840x2160_d8",
                                 "hash_synth16_7680x4320_d8", "hash_stress4096_3840x2160_d12",
                                 "hash_stress4096_3840x2160_d12_f2", "hash_default_1920x1080_d20_ss4"])
def test_full_size_hash(key):
    """BASELINE configs C1, C2 (depth 1 and 4), C3, C4, C5 (frame 0, and frame 1 with the stream continued: the
    image after two frames) and the reference's screenshot workload (Full HD, 4x4 SSAA, depth 20), plus the default
    scene at 4K d8, at full size and the library defaults, bit-exact by SHA-256.  C5 runs the large-scene path as
    shipped: park after 2 segments, the LDS-staged bounce kernel, the longest-first schedule (learned from frame 0 on
    frame 1)."""
    c = CASES[key]
    rgb, argb, r = run_case(c)
    if c["scene"] == "stress4096":
        assert r._r.bounce_form() == 2, key  # the regrouped frame's LDS-staged bounce kernel ran
    assert sha(argb) == c["sha_argb"], key
    assert sha(rgb) == c["sha_f32"], key
    r.close()


def test_c5_full_frames_steady_state():
    """C5 over three frames at the defaults, per-view state included: frame 0 (first view: per-launch bundles, raster
    tile order), frame 1 (the view repeats: the schedule is sorted from frame 0's costs) hash to the reference's
    frames 0 and 1; frame 2 equals a frame rendered without regrouping or schedule from the same stream state."""
    c0, c1 = CASES["hash_stress4096_3840x2160_d12"], CASES["hash_stress4096_3840x2160_d12_f2"]
    got = []
    _, _, r = gpu_render(scene("stress4096"), 3840, 2160, 12, frames=3, sphere_seed=c0["sphere_seed"],
                         each_frame=lambda rgb, argb: got.append((sha(rgb), sha(argb))))
    r.close()
    assert got[0] == (c0["sha_f32"], c0["sha_argb"])
    assert got[1] == (c1["sha_f32"], c1["sha_argb"])
    plain = []
    _, _, r = gpu_render(scene("stress4096"), 3840, 2160, 12, frames=3, sphere_seed=c0["sphere_seed"], regroup=0,
                         tile_order=0, prim_masks=0, each_frame=lambda rgb, argb: plain.append((sha(rgb), sha(argb))))
    r.close()
    assert plain == got


@pytest.mark.parametrize("key", sorted(k for k, c in CASES.items() if c["kind"] == "band"))
def test_stress_band(key):
    """C5 (4096 spheres, 4K, depth 12): full GPU frame; the reference's 4-row bands must match bit-exactly."""
    c = CASES[key]
    rgb, argb, r = gpu_render(scene(c["scene"]), c["W"], c["H"], c["depth"], sphere_seed=c["sphere_seed"])
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    y0, rows = c["y0"], c["rows"]
    assert np.array_equal(argb[y0:y0 + rows], g["argb"])
    assert rgb[y0:y0 + rows].tobytes() == g["rgb"].tobytes()
    r.close()


@pytest.mark.parametrize("chunks", [[1], [7, 1000, 13], [4096], [19200 - 1, 1]])
def test_chunked_render_next(chunks):
    """Pulse-style chunked renderNext (Pulse.cpp:131-145) gives the reference's image for any chunk pattern: plain,
    block-preview and additive frames, and SSAA frames whose spans cut through the lanes modes' pixel blocks."""
    for key in ("render_default_160x120_d4", "render_default_161x121_d4_ssm4", "render_default_160x120_d15_add3",
                "render_default_160x120_d4_ss2", "render_default_64x40_d8_ss4", "render_default_17x9_d8_ss16_add2"):
        c = CASES[key]
        rgb, argb, r = run_case(c, chunks=chunks)
        g = np.load(os.path.join(GOLDEN, key + ".npz"))
        assert np.array_equal(argb, g["argb"]), (key, chunks)
        assert rgb.tobytes() == g["rgb"].tobytes(), (key, chunks)
        r.close()


def test_rand_dirs_prepass():
    """The parallel LCG pre-pass reproduces the reference's serial randomInsideSphere stream."""
    from reflaxman_amd.render import Renderer
    g = np.load(os.path.join(GOLDEN, "kat_rand.npz"))
    rr = Renderer()
    dirs, after = rr.rand_dirs(int(g["seed"][0]), g["dirs"].shape[0])
    assert dirs.tobytes() == g["dirs"].tobytes()
    import oracle as orc
    _, s_after = orc.rand_dirs(int(g["seed"][0]), g["dirs"].shape[0])
    assert after == s_after
    # tiny and ragged counts
    for n in (1, 2, 3, 63, 64, 65, 4097):
        d, a = rr.rand_dirs(12345, n)
        od, oa = orc.rand_dirs(12345, n)
        assert d.tobytes() == od.tobytes() and a == oa, n
    rr.close()


@pytest.mark.parametrize("W,H,ss,frames", [(1, 1, 1, 3), (7, 9, 1, 2), (65, 63, 1, 2), (640, 480, 1, 2),
                                           (1999, 2000, 1, 2), (2000, 2000, 1, 1), (2100, 2100, 1, 1), (333, 200, 8, 1),
                                           (512, 511, 2, 2), (300, 200, 4, 1)])
def test_rng_stream_state_per_frame_size(W, H, ss, frames):
    """The render path's pre-pass -- the one-pass kernel (rng_fused: count, decoupled look-back scan, scatter) up to
    RFX_RNG_FUSED_MAX_BLOCKS = 256 blocks (640x480 is 166), the two-kernel form beyond -- carries
    the reference's randomInsideSphere stream: after each frame the renderer's sphere seed equals the serial stream
    advanced by the frame's W*H*ss^2 accepted triples (oracle orc_rand_dirs), frame after frame; no error flag."""
    import oracle as orc
    desc = scene("default")
    _, _, r = gpu_render(desc, W, H, 1, ss, frames=frames, sphere_seed=4242)
    _, after = orc.rand_dirs(4242, W * H * ss * ss * frames)
    assert r.getRng()[0] == after
    r.close()


def test_concurrent_renderers_share_one_device():
    """Three renderers render C1 frames (640x480 depth 4, the one-pass pre-pass: 166 blocks) on their own streams of one
    device at once, beside a fourth renderer's C3 frame that holds the chip's slots, with no synchronisation between
    them: the pre-pass's look-back takes its block order from an ordered ticket, so its blocks finish whatever order
    the workgroups are dispatched in and whatever else is resident.  Each C1 frame hashes to the reference's frame and
    no renderer reports an error."""
    import torch
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    c1 = CASES["hash_default_640x480_d4"]
    s1, cam1 = build_scene(scene("default"))
    s3, cam3 = build_scene(scene("synth16"))
    big = Renderer()
    big.set_scene(s3)
    rs = [Renderer() for _ in range(3)]
    for r in rs:
        r.set_scene(s1)
    W, H = 640, 480
    f1, f3 = make_frame(cam1, W, H, 4), make_frame(cam3, 3840, 2160, 8)
    bufs = [(torch.zeros(H * W * 3, device="cuda"), torch.zeros(H * W, dtype=torch.int32, device="cuda")) for _ in rs]
    big_rgb = torch.zeros(3840 * 2160 * 3, device="cuda")
    torch.cuda.synchronize()
    big.render_frame(f3, big_rgb.data_ptr())
    for r, (rgb, argb) in zip(rs, bufs):
        r.render_frame(f1, rgb.data_ptr(), argb.data_ptr())
    for r in rs + [big]:
        r.synchronize()
    for rgb, argb in bufs:
        assert sha(rgb.cpu().numpy()) == c1["sha_f32"]
        assert sha(argb.cpu().numpy().view(np.uint32)) == c1["sha_argb"]
    for r in rs + [big]:
        r.close()


@pytest.mark.parametrize("name,W,H,depth,ss,additive,chunks", [
    ("synth16", 640, 360, 8, 1, False, None),      # plain frames: record, reuse the sorted order, re-sort
    ("default", 200, 150, 4, 2, True, None),       # SSAA + additive accumulation
    ("default", 161, 121, 4, -4, False, None),     # block preview
    ("synth16", 320, 180, 8, 1, False, [5000, 777]),  # chunked renderNext: the grid changes every call
])
def test_tile_order_changes_no_pixel(name, W, H, depth, ss, additive, chunks):
    """The longest-tile-first schedule (default) renders every frame exactly as raster order does."""
    frames = []
    for mode in (0, 3):  # raster order vs longest-first on every launch size
        got = []
        _, _, r = gpu_render(scene(name), W, H, depth, ss, additive, 9, tile_order=mode, chunks=chunks,
                             each_frame=lambda rgb, argb: got.append((rgb.tobytes(), argb.tobytes())))
        r.close()
        frames.append(got)
    assert len(frames[0]) == 9 and frames[0] == frames[1]


def test_tile_order_default_full_size():
    """C3 at full size, where the default schedule is on: 6 frames, bit-identical to raster order."""
    frames = []
    for mode in (0, 1):
        got = []
        _, _, r = gpu_render(scene("synth16"), 3840, 2160, 8, frames=6, tile_order=mode,
                             each_frame=lambda rgb, argb: got.append((sha(rgb), sha(argb))))
        r.close()
        frames.append(got)
    assert len(frames[0]) == 6 and frames[0] == frames[1]
    assert frames[0][0] == (CASES["hash_synth16_3840x2160_d8"]["sha_f32"], CASES["hash_synth16_3840x2160_d8"]["sha_argb"])


def test_rng_state_carries_across_frames():
    """Two back-to-back frames (non-additive) continue the global stream like the reference."""
    import oracle as orc
    desc = scene("default")
    rgb, argb, r = gpu_render(desc, 96, 72, 4, frames=2, sphere_seed=777, jitter_seed=5)
    o = orc.OracleRender(desc, 777, 5)
    o.set_image_size(96, 72)
    o.render(4, 1)
    o.render(4, 1)
    assert rgb.tobytes() == o.image_pixels().tobytes()
    assert r.getRng()[0] == o.sphere_seed.value
    r.close()


@pytest.mark.parametrize("nranks,row_block", [(2, 8), (3, 5), (4, 16), (8, 8)])
def test_strip_partition_assembles_to_whole_frame(nranks, row_block):
    """Block-cyclic strips rendered rank by rank re-assemble to the 1-GPU frame bit-exactly."""
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    import ctypes as C
    desc = scene("synth16")
    W, H, depth = 200, 123, 8
    s, cam = build_scene(desc)
    L = _lib.load()

    def render(rank, nr):
        rr = Renderer(sphere_seed=1350490027)
        rr.set_scene(s)
        rows = L.rfx_strip_rows(H, row_block, rank, nr) if nr > 1 else H
        n = W * rows
        d_img, d_argb = C.c_void_p(), C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, n * 12, C.byref(d_img)))
        _lib.check(L.rfx_device_alloc(rr._h, n * 4, C.byref(d_argb)))
        f = make_frame(cam, W, H, depth, 1, row_block=row_block if nr > 1 else 0, rank=rank, nranks=nr)
        rr.render_frame(f, d_img.value, d_argb.value)
        img = np.empty((rows, W, 3), np.float32)
        argb = np.empty((rows, W), np.uint32)
        _lib.check(L.rfx_memcpy_d2h(rr._h, img.ctypes.data_as(C.c_void_p), d_img, n * 12))
        _lib.check(L.rfx_memcpy_d2h(rr._h, argb.ctypes.data_as(C.c_void_p), d_argb, n * 4))
        rr.synchronize()
        L.rfx_device_free(rr._h, d_img)
        L.rfx_device_free(rr._h, d_argb)
        rr.close()
        return img, argb

    whole, whole_argb = render(0, 1)
    img = np.zeros_like(whole)
    argb = np.zeros_like(whole_argb)
    for rank in range(nranks):
        part, part_argb = render(rank, nranks)
        ys = [L.rfx_strip_row_to_y(i, row_block, rank, nranks) for i in range(part.shape[0])]
        img[ys] = part
        argb[ys] = part_argb
    assert img.tobytes() == whole.tobytes()
    assert np.array_equal(argb, whole_argb)


@pytest.mark.parametrize("nranks,row_block,ss,masks", [(2, 8, 1, 1), (3, 5, 1, 1), (4, 16, 2, 1), (8, 8, 1, 1),
                                                       (3, 5, 2, 2), (2, 3, 4, 2), (2, 8, 1, 2)])
def test_sliced_rng_prepass_multi_rank(nranks, row_block, ss, masks):
    """The multi-GPU pre-pass (slice counts -> all-gather -> filtered emit), emulated rank by rank in one
    process: the assembled strips equal the 1-GPU frame and every rank carries the same stream state.  masks 2: the
    ranks build their per-view masks before the launch, over strips whose height is no multiple of the lanes mode's
    pixel block (sampleNum 2: 4-row blocks over 5-row strips; 4: 2-row blocks over 3-row strips)."""
    import ctypes as C
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    desc = scene("synth16")
    W, H, depth = 160, 101, 8
    s, cam = build_scene(desc)
    L = _lib.load()

    def fetch(rr, d, n, dtype):
        a = np.empty(n, dtype)
        _lib.check(L.rfx_memcpy_d2h(rr._h, a.ctypes.data_as(C.c_void_p), d, a.nbytes))
        return a

    whole = Renderer(sphere_seed=97531)
    whole.set_scene(s)
    d_img, d_argb = C.c_void_p(), C.c_void_p()
    _lib.check(L.rfx_device_alloc(whole._h, W * H * 12, C.byref(d_img)))
    _lib.check(L.rfx_device_alloc(whole._h, W * H * 4, C.byref(d_argb)))
    whole.render_frame(make_frame(cam, W, H, depth, ss), d_img.value, d_argb.value)
    ref = fetch(whole, d_img, W * H * 3, np.float32).reshape(H, W, 3)
    ref_argb = fetch(whole, d_argb, W * H, np.uint32).reshape(H, W)
    ref_seed = whole.get_rng()[0]

    img = np.zeros_like(ref)
    argb = np.zeros_like(ref_argb)
    for rank in range(nranks):
        rr = Renderer(sphere_seed=97531)
        rr.set_scene(s)
        rr.set_prim_masks(masks)
        f = make_frame(cam, W, H, depth, ss, row_block=row_block, rank=rank, nranks=nranks)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), nranks, C.byref(bps)))
        d_cnt = C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, nranks * bps.value * 4, C.byref(d_cnt)))
        for sl in range(nranks):  # what the all-gather assembles from every rank's slice
            _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), sl, nranks, d_cnt, None))
        rows = L.rfx_strip_rows(H, row_block, rank, nranks)
        p_img, p_argb = C.c_void_p(), C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, max(rows, 1) * W * 12, C.byref(p_img)))
        _lib.check(L.rfx_device_alloc(rr._h, max(rows, 1) * W * 4, C.byref(p_argb)))
        _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), nranks, d_cnt, p_img, p_argb, None, None))
        part = fetch(rr, p_img, rows * W * 3, np.float32).reshape(rows, W, 3)
        part_argb = fetch(rr, p_argb, rows * W, np.uint32).reshape(rows, W)
        ys = [L.rfx_strip_row_to_y(i, row_block, rank, nranks) for i in range(rows)]
        img[ys] = part
        argb[ys] = part_argb
        assert rr.get_rng()[0] == ref_seed, rank
        rr.close()
    assert img.tobytes() == ref.tobytes()
    assert np.array_equal(argb, ref_argb)
    whole.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_strips_with_tile_order_over_frames(nranks):
    """Strip frames (the multi-GPU path, ranks emulated in one process) with the longest-first schedule on
    every launch (mode 3): each of 5 consecutive frames assembles to the raster-order 1-GPU frame."""
    import ctypes as C
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    desc = scene("synth16")
    W, H, depth, rb, frames = 200, 120, 8, 8, 5
    s, cam = build_scene(desc)
    L = _lib.load()

    def fetch(rr, d, n):
        a = np.empty(n, np.uint32)
        _lib.check(L.rfx_memcpy_d2h(rr._h, a.ctypes.data_as(C.c_void_p), d, a.nbytes))
        return a

    whole = Renderer(sphere_seed=4242)
    whole.set_scene(s)
    whole.set_tile_order(0)
    d_img, d_argb = C.c_void_p(), C.c_void_p()
    _lib.check(L.rfx_device_alloc(whole._h, W * H * 12, C.byref(d_img)))
    _lib.check(L.rfx_device_alloc(whole._h, W * H * 4, C.byref(d_argb)))
    refs = []
    for _ in range(frames):
        whole.render_frame(make_frame(cam, W, H, depth, 1), d_img.value, d_argb.value)
        refs.append(fetch(whole, d_argb, W * H).reshape(H, W))
    got = [np.zeros((H, W), np.uint32) for _ in range(frames)]
    for rank in range(nranks):
        rr = Renderer(sphere_seed=4242)
        rr.set_scene(s)
        rr.set_tile_order(3)
        f = make_frame(cam, W, H, depth, 1, row_block=rb, rank=rank, nranks=nranks)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), nranks, C.byref(bps)))
        d_cnt = C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, nranks * bps.value * 4, C.byref(d_cnt)))
        rows = L.rfx_strip_rows(H, rb, rank, nranks)
        p_img, p_argb = C.c_void_p(), C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, rows * W * 12, C.byref(p_img)))
        _lib.check(L.rfx_device_alloc(rr._h, rows * W * 4, C.byref(p_argb)))
        ys = [L.rfx_strip_row_to_y(i, rb, rank, nranks) for i in range(rows)]
        for k in range(frames):
            for sl in range(nranks):  # what the all-gather assembles from every rank's slice
                _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), sl, nranks, d_cnt, None))
            _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), nranks, d_cnt, p_img, p_argb, None, None))
            got[k][ys] = fetch(rr, p_argb, rows * W).reshape(rows, W)
        rr.close()
    for k in range(frames):
        assert np.array_equal(got[k], refs[k]), k
    whole.close()


def test_event_counters_match_oracle():
    """The stats kernel's event counts equal the CPU restatement's (same algorithm, same branches)."""
    import ctypes as C
    import oracle as orc
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    for name, W, H, depth in (("default", 64, 48, 8), ("synth16", 64, 36, 8), ("synth16_sky", 48, 27, 6),
                              ("planes", 64, 36, 8), ("planes300", 48, 27, 6), ("lights3", 48, 27, 8),
                              ("lights40", 32, 18, 6), ("mesh100", 48, 27, 6), ("nolight", 48, 36, 4)):
        desc = scene(name)
        o = orc.OracleRender(desc, 4242, 0)
        o.set_image_size(W, H)
        oc = np.zeros(len(orc.COUNTER_NAMES), np.uint64)
        o.render(depth, 1, counters=oc)
        s, cam = build_scene(desc)
        rr = Renderer(sphere_seed=4242)
        rr.set_scene(s)
        img = np.zeros((H, W, 3), np.float32)
        gc = np.zeros(len(orc.COUNTER_NAMES), np.uint64)
        f = make_frame(cam, W, H, depth, 1)
        L = _lib.load()
        _lib.check(L.rfx_render_frame_host(rr._h, C.byref(f), _lib.fptr(img), None, _lib.u64ptr(gc)))
        assert img.tobytes() == o.image.tobytes()
        # more than 32 spheres: the kernel visits them in Morton order, so the shadow any-hit (which stops at
        # the first occluder) runs a different number of tests than the oracle's insertion order; its boolean
        # and every other counter are order-independent
        skip = {k for k in orc.COUNTER_NAMES if k.startswith("sh_")} if desc.n_spheres > 32 else set()
        bad = {k: (int(a), int(b)) for k, a, b in zip(orc.COUNTER_NAMES, gc, oc) if a != b and k not in skip}
        assert not bad, (name, bad)
        rr.close()


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_c4_strips_assemble_to_reference_hash(nranks):
    """C4 (the C3 scene at 7680x4320 d8, BASELINE configs[3]) as the multi-GPU path renders it -- each rank
    counts its slice of the random stream, the counts are exchanged (emulated: every rank counts every slice),
    each rank emits and traces only its 8-row block-cyclic strips -- assembled in one process: SHA-256 of the
    f32 frame and of the ARGB8 frame equal the reference's."""
    import ctypes as C
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    c = CASES["hash_synth16_7680x4320_d8"]
    W, H, depth, rb = c["W"], c["H"], c["depth"], 8
    s, cam = build_scene(scene("synth16"))
    L = _lib.load()
    img = np.zeros((H, W, 3), np.float32)
    argb = np.zeros((H, W), np.uint32)
    for rank in range(nranks):
        rr = Renderer(sphere_seed=c["sphere_seed"])
        rr.set_scene(s)
        f = make_frame(cam, W, H, depth, 1, row_block=rb, rank=rank, nranks=nranks)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), nranks, C.byref(bps)))
        d_cnt = C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, nranks * bps.value * 4, C.byref(d_cnt)))
        for sl in range(nranks):
            _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), sl, nranks, d_cnt, None))
        rows = L.rfx_strip_rows(H, rb, rank, nranks)
        p_img, p_argb = C.c_void_p(), C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, rows * W * 12, C.byref(p_img)))
        _lib.check(L.rfx_device_alloc(rr._h, rows * W * 4, C.byref(p_argb)))
        _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), nranks, d_cnt, p_img, p_argb, None, None))
        part = np.empty((rows, W, 3), np.float32)
        part_argb = np.empty((rows, W), np.uint32)
        _lib.check(L.rfx_memcpy_d2h(rr._h, part.ctypes.data_as(C.c_void_p), p_img, part.nbytes))
        _lib.check(L.rfx_memcpy_d2h(rr._h, part_argb.ctypes.data_as(C.c_void_p), p_argb, part_argb.nbytes))
        ys = np.array([L.rfx_strip_row_to_y(i, rb, rank, nranks) for i in range(rows)])
        img[ys] = part
        argb[ys] = part_argb
        for p in (d_cnt, p_img, p_argb):
            L.rfx_device_free(rr._h, p)
        rr.close()
    assert sha(argb) == c["sha_argb"]
    assert sha(img) == c["sha_f32"]


@pytest.mark.parametrize("bounds", [[0, 2000, 4320], [0, 1000, 2200, 2208, 4320],
                                    [0, 600, 1096, 1600, 2160, 2704, 3240, 3800, 4320]])
def test_c4_bands_assemble_to_reference_hash(bounds):
    """C4 under the band partition (rfx.h: nranks > 1, row_block 0), with uneven bands as the balancer cuts them
    (one of them 8 rows): each rank counts its slice of the random stream (the exchange emulated: every rank counts
    every slice), emits and traces only its rows into a whole-frame buffer, and the bands are copied into one
    frame, as rank 0 receives them: SHA-256 of the f32 frame and of the ARGB8 frame equal the reference's."""
    import ctypes as C
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    c = CASES["hash_synth16_7680x4320_d8"]
    W, H, depth = c["W"], c["H"], c["depth"]
    nranks = len(bounds) - 1
    s, cam = build_scene(scene("synth16"))
    L = _lib.load()
    img = np.zeros((H, W, 3), np.float32)
    argb = np.zeros((H, W), np.uint32)
    for rank in range(nranks):
        y0, y1 = bounds[rank], bounds[rank + 1]
        rr = Renderer(sphere_seed=c["sphere_seed"])
        rr.set_scene(s)
        f = make_frame(cam, W, H, depth, 1, row_block=0, rank=rank, nranks=nranks, pixel_begin=y0 * W,
                       pixel_end=y1 * W)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), nranks, C.byref(bps)))
        d_cnt, p_img, p_argb = C.c_void_p(), C.c_void_p(), C.c_void_p()
        _lib.check(L.rfx_device_alloc(rr._h, nranks * bps.value * 4, C.byref(d_cnt)))
        for sl in range(nranks):
            _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), sl, nranks, d_cnt, None))
        _lib.check(L.rfx_device_alloc(rr._h, H * W * 12, C.byref(p_img)))
        _lib.check(L.rfx_device_alloc(rr._h, H * W * 4, C.byref(p_argb)))
        _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), nranks, d_cnt, p_img, p_argb, None, None))
        part = np.empty((H, W, 3), np.float32)
        part_argb = np.empty((H, W), np.uint32)
        _lib.check(L.rfx_memcpy_d2h(rr._h, part.ctypes.data_as(C.c_void_p), p_img, part.nbytes))
        _lib.check(L.rfx_memcpy_d2h(rr._h, part_argb.ctypes.data_as(C.c_void_p), p_argb, part_argb.nbytes))
        img[y0:y1] = part[y0:y1]
        argb[y0:y1] = part_argb[y0:y1]
        for p in (d_cnt, p_img, p_argb):
            L.rfx_device_free(rr._h, p)
        rr.close()
    assert sha(argb) == c["sha_argb"]
    assert sha(img) == c["sha_f32"]


def test_textures_loaded_from_tga_files(tmp_path):
    """The scene's textures read from TGA files by the library's loader (Scene.addTexture /
    setSkyboxTexture, Texture.cpp:34-108) -- the files the reference read for the same golden."""
    key = "render_synth16_sky_160x90_d8"
    c = CASES[key]
    from reflaxman_amd.render import Render, build_scene
    r = Render(sphere_seed=c["sphere_seed"], jitter_seed=0, load_default_scene=False)
    r.scene, r.camera = build_scene(scene(c["scene"]), texture_dir=str(tmp_path))
    assert r.scene.counts() == (16, 4, 1, 3)
    r.setImageSize(c["W"], c["H"])
    r.renderBegin(c["depth"], 1, False)
    while r.renderNext(c["W"] * c["H"]):
        pass
    r.synchronize()
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    assert np.array_equal(r.copyImage(), g["argb"])
    assert r.imagePixels().tobytes() == g["rgb"].tobytes()
    r.close()


@pytest.mark.parametrize("key,park,qsort", [("hash_synth16_3840x2160_d8", 1, 1), ("hash_synth16_3840x2160_d8", 2, 1),
                                            ("hash_default_640x480_d4", 1, 1), ("hash_synth16_7680x4320_d8", 3, 1),
                                            ("hash_synth16_3840x2160_d8", 1, 0), ("hash_default_640x480_d4", 2, 0)])
def test_regrouped_frame_matches_reference_hash(key, park, qsort):
    """Ray regrouping (traces parked after `park` segments, resumed by the packed bounce kernel -- in bucket order or
    in park order) on the small-scene configs, where it is off by default: the full frame still hashes to the
    reference's."""
    c = CASES[key]
    rgb, argb, r = run_case(c, regroup=park, regroup_sort=qsort)
    assert sha(argb) == c["sha_argb"], key
    assert sha(rgb) == c["sha_f32"], key
    r.close()


@pytest.mark.parametrize("key", sorted(k for k, c in CASES.items() if c["kind"] == "band" and c["scene"] == "stress4096"))
@pytest.mark.parametrize("regroup,qsort", [(0, None), (3, 1), (2, 1)])
def test_stress_band_other_regrouping(key, regroup, qsort):
    """C5 with regrouping off, and with the parked traces sorted into buckets (the default takes them in park
    order): the reference's bands again."""
    c = CASES[key]
    rgb, argb, r = gpu_render(scene(c["scene"]), c["W"], c["H"], c["depth"], sphere_seed=c["sphere_seed"],
                              regroup=regroup, regroup_sort=qsort)
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    y0, rows = c["y0"], c["rows"]
    assert np.array_equal(argb[y0:y0 + rows], g["argb"])
    assert rgb[y0:y0 + rows].tobytes() == g["rgb"].tobytes()
    r.close()


@pytest.mark.parametrize("key", sorted(k for k, c in CASES.items() if c["kind"] == "band" and c["scene"] == "stress4096"))
def test_stress_band_chunk_lists(key):
    """C5 with prim_masks 2: the per-view chunk lists of the primary bundles (prim_cull_large_kernel).  They exist only
    in an RFX_PRIM_LARGE build (measured slower, compiled out by default): in the default build this path has no parity
    coverage, and the test is skipped rather than repeating test_stress_band."""
    from reflaxman_amd import _lib
    if not _lib.load().rfx_build_options() & 1:  # RFX_BUILD_PRIM_LARGE
        pytest.skip("default build: RFX_PRIM_LARGE compiled out (no per-view chunk lists to test)")
    c = CASES[key]
    rgb, argb, r = gpu_render(scene(c["scene"]), c["W"], c["H"], c["depth"], sphere_seed=c["sphere_seed"], prim_masks=2)
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    y0, rows = c["y0"], c["rows"]
    assert np.array_equal(argb[y0:y0 + rows], g["argb"])
    assert rgb[y0:y0 + rows].tobytes() == g["rgb"].tobytes()
    r.close()


@pytest.mark.parametrize("big", [False, True])
def test_regrouped_large_scene_equals_unregrouped(big):
    """The bounce kernel's two forms on large scenes: with the BVH staged in LDS (4096 spheres fit) and walking it in
    global memory (a scene whose BVH has more than the ~2,100 nodes the LDS holds: 4,400 spheres per sphere pair of a
    leaf, rfx_build_options).  Regrouped frames (park after 1 and 2) equal the frame traced without regrouping, bit for
    bit, over two frames of the random stream."""
    from reflaxman_amd import _lib
    leaf_pairs = (_lib.load().rfx_build_options() >> 8) & 0xFF
    n_spheres = 4400 * leaf_pairs if big else 4096
    desc = scenes.stress_scene(n_spheres)
    ref, _, r0 = gpu_render(desc, 320, 180, 12, frames=2, regroup=0)
    assert r0._r.bounce_form() == 0
    r0.close()
    for park in (1, 2):
        rgb, _, r = gpu_render(desc, 320, 180, 12, frames=2, regroup=park)
        assert rgb.tobytes() == ref.tobytes(), (n_spheres, park)
        # the form the test is about ran (a refused LDS launch falls back to the global form silently otherwise)
        assert r._r.bounce_form() == (1 if big else 2), (n_spheres, park)
        r.close()


@pytest.mark.parametrize("key", ["hash_synth16_3840x2160_d8", "hash_default_640x480_d4", "hash_synth16_7680x4320_d8",
                                 "hash_default_1920x1080_d20_ss4"])
def test_primary_masks_match_reference_hash(key):
    """Precomputed primary-bundle cull masks (rfx_renderer_set_prim_masks 2: built before the launch, so the
    very first frame uses them): the full frame still hashes to the reference's."""
    c = CASES[key]
    rgb, argb, r = run_case(c, prim_masks=2)
    assert sha(argb) == c["sha_argb"], key
    assert sha(rgb) == c["sha_f32"], key
    r.close()


@pytest.mark.parametrize("key", sorted(k for k, c in CASES.items()
                                       if c["kind"] == "render" and c.get("stored") and c["ss"] >= 1
                                       and c["W"] * c["H"] > 1))
def test_primary_masks_on_goldens(key):
    """Every stored golden but the block previews with the masks built before every launch (prim_masks 2): one-sample
    frames and the one-lane-per-sample frames (sampleNum 2, 4, 8, jittered sampleNum 1: prim_cull_kernel<., true>) use
    them; sampleNum 3, 5, 6, 7 and > 8 use them only in an RFX_PRIM_SSAA build (compiled out by default, measured
    slower), so there the test pins that the setting changes nothing."""
    c = CASES[key]
    rgb, argb, r = run_case(c, prim_masks=2)
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    assert np.array_equal(argb, g["argb"]), key
    assert rgb.tobytes() == g["rgb"].tobytes(), key
    r.close()


@pytest.mark.parametrize("ss,additive", [(1, False), (2, False), (1, True), (3, True), (4, False), (2, True), (8, False)])
def test_primary_masks_over_repeated_views(ss, additive):
    """A still camera over 4 frames (masks built on the second and reused), one-sample, SSAA and additive (jittered,
    accumulating) frames: every frame equals the frame rendered without masks (sampleNum 3 takes masks only in an
    RFX_PRIM_SSAA build; 2, 4, 8 and jittered 1 take the lanes masks, jittered ones without the shadow masks)."""
    desc = scene("synth16")
    W, H, depth = (640, 360, 8) if ss == 1 else (320, 184, 8)
    frames = {}
    for mode in (0, 1):
        out = []
        _, _, r = gpu_render(desc, W, H, depth, ss=ss, additive=additive, frames=4, prim_masks=mode, jitter_seed=99,
                             each_frame=lambda rgb, argb: out.append((rgb.tobytes(), argb.tobytes())))
        r.close()
        frames[mode] = out
    assert frames[0] == frames[1]


def test_primary_masks_full_size_frames():
    """C3 at full size over 6 frames (masks built on the second frame and reused): every frame equals the frame
    rendered without masks (the first also equals the reference's hash)."""
    c = CASES["hash_synth16_3840x2160_d8"]
    hashes = {}
    for mode in (0, 1):
        out = []
        _, _, r = gpu_render(scene(c["scene"]), c["W"], c["H"], c["depth"], frames=6, prim_masks=mode,
                             sphere_seed=c["sphere_seed"],
                             each_frame=lambda rgb, argb: out.append((sha(rgb), sha(argb))))
        r.close()
        hashes[mode] = out
    assert hashes[0][0] == (c["sha_f32"], c["sha_argb"])
    assert hashes[0] == hashes[1]


def _float_accept_counts(seed, nthreads):
    """Per pre-pass thread (16 triples, 48 draws from its jumped start), the accepted triples by the reference's float
    test (Vector3.cpp:182-185: x = float(k) / (float(0x7FFF) / 2) - 1, rejected when x*x + y*y + z*z > 1), and the
    number of triples that fall on the integer test's shell (where rng_count runs the float test itself)."""
    def jump(n):
        a, c, A, Cc = 214013, 2531011, 1, 0
        while n:
            if n & 1:
                A, Cc = (a * A) & 0xFFFFFFFF, (a * Cc + c) & 0xFFFFFFFF
            c, a, n = (a * c + c) & 0xFFFFFFFF, (a * a) & 0xFFFFFFFF, n >> 1
        return np.uint32(A), np.uint32(Cc)
    half = np.float32(np.float32(0x7FFF) / np.float32(2))
    x_of = (np.arange(1 << 15, dtype=np.float32) / half - np.float32(1)).astype(np.float32)
    S = np.empty(nthreads, np.uint32)
    S[0] = seed
    k = 1
    cnt = np.zeros(nthreads, np.int64)
    shell = 0
    with np.errstate(over="ignore"):
        while k < nthreads:
            A, Cc = jump(48 * k)
            m = min(k, nthreads - k)
            S[k:k + m] = A * S[:m] + Cc
            k *= 2
        s = S
        for _ in range(16):
            acc = np.zeros(nthreads, np.float32)
            n = np.zeros(nthreads, np.int64)
            for d in range(3):
                s = np.uint32(214013) * s + np.uint32(2531011)
                kk = ((s >> 16) & 0x7FFF).astype(np.int64)
                x = x_of[kk]
                acc = (acc + x * x).astype(np.float32) if d else (x * x).astype(np.float32)
                n += (2 * kk - 32767) ** 2
            cnt += ~(acc > np.float32(1))
            shell += int((np.abs(n - 32767 * 32767) <= 1024).sum())
    return cnt, shell


def test_rng_count_blocks_equal_the_float_test():
    """rng_count's per-block accept counts (rfx_frame_rng_count, one slice) for the C3 frame from the default seed against
    the reference's float test restated in numpy: every block of the launch (about 4,100) equal, with triples on the
    integer test's shell among them (so its float fallback is what decided those)."""
    import ctypes as C
    from reflaxman_amd import _lib
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    L = _lib.load()
    s, cam = build_scene(scene("synth16"))
    rr = Renderer(sphere_seed=1350490027)
    rr.set_scene(s)
    f = make_frame(cam, 3840, 2160, 8)
    nblk = C.c_uint64()
    _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), 1, C.byref(nblk)))
    d_cnt = C.c_void_p()
    _lib.check(L.rfx_device_alloc(rr._h, nblk.value * 4, C.byref(d_cnt)))
    _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), 0, 1, d_cnt, None))
    got = np.empty(nblk.value, np.uint32)
    _lib.check(L.rfx_memcpy_d2h(rr._h, got.ctypes.data_as(C.c_void_p), d_cnt, got.nbytes))
    rr.close()
    per_thread, shell = _float_accept_counts(1350490027, nblk.value * 256)
    want = per_thread.reshape(-1, 256).sum(1)
    assert nblk.value >= 4054 and shell >= 10
    assert np.array_equal(got.astype(np.int64), want)
