"""The single-pass RNG pre-pass (rng_scan_emit: count, decoupled look-back scan and emit in one launch) against the
two-launch form (rng_count + rng_emit, which the multi-GPU slices keep) and the oracle's serial stream.

The reference draws one randomInsideSphere triple per trace from one serial LCG stream (Scene.cpp:75,
Vector3.cpp:176-186, trace_math.h:34-39); the pre-pass must hand trace i the i-th accepted triple and leave the
stream state after the frame's last one.  Checked here:

* rfx_rand_dirs (the same kernel) against the oracle's serial stream at sizes from one block to ~10k blocks (many
  64-block look-back windows), repeated with the size changing between launches (granule epochs, ticket reset);
* the same under uneven load: a torch workload keeps the GPU busy on another stream while the pre-pass runs;
* rfx_render_frame (single pass) and rfx_frame_rng_count + rfx_render_frame_counted (two launches) render the
  same frames bit for bit, over frames whose size changes, and leave the same stream state.
"""
import ctypes as C

import numpy as np
import pytest

from reflaxman_amd import _lib, scenes

pytestmark = pytest.mark.gpu

SEED = 1350490027


def _oracle_dirs(seed, n):
    import oracle as orc
    return orc.rand_dirs(seed, n)


def test_scan_emit_matches_serial_stream_across_sizes():
    from reflaxman_amd.render import Renderer
    rr = Renderer()
    # 1 block .. ~10k blocks (2^24 triples), then smaller again: each launch a new epoch over reused granules
    for n in (1, 4095, 4096, 70_000, 2_000_003, 20_000_000, 300_001, 5):
        seed = (SEED * 7 + n) & 0xFFFFFFFF
        d, a = rr.rand_dirs(seed, n)
        od, oa = _oracle_dirs(seed, n)
        assert a == oa, n
        assert d.tobytes() == od.tobytes(), n
    rr.close()


def test_scan_emit_under_uneven_load():
    """The look-back's granules are polled while another stream's kernels hold most of the chip."""
    import torch
    from reflaxman_amd.render import Renderer
    rr = Renderer()
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    n = 3_000_000
    od, oa = _oracle_dirs(SEED, n)
    for k in range(6):
        with torch.cuda.stream(side):
            for _ in range(4):
                a = torch.tanh(a @ a * 1e-3)
        d, after = rr.rand_dirs(SEED, n)
        assert after == oa and d.tobytes() == od.tobytes(), k
    torch.cuda.synchronize()
    rr.close()


@pytest.mark.parametrize("name,sizes,depth", [
    ("default", [(640, 480), (96, 54), (1920, 1080), (640, 480)], 4),
    ("synth16", [(3840, 2160), (320, 180), (3840, 2160)], 8),
])
def test_single_pass_frames_equal_two_launch_frames(name, sizes, depth):
    import torch
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    L = _lib.load()
    desc = scenes.get_scene(name)
    one, two = Renderer(sphere_seed=SEED), Renderer(sphere_seed=SEED)
    sc, cam = build_scene(desc)
    one.set_scene(sc)
    two.set_scene(sc)
    for W, H in sizes:
        f = make_frame(cam, W, H, depth, 1)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(two._h, C.byref(f), 1, C.byref(bps)))
        counts = torch.zeros(bps.value, dtype=torch.int32, device="cuda")
        out = []
        for rr, single in ((one, True), (two, False)):
            print(f"{name} {W}x{H} single={single}", flush=True)
            rgb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
            argb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            if single:
                rr.render_frame(f, rgb.data_ptr(), argb.data_ptr())
            else:
                _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), 0, 1, C.c_void_p(counts.data_ptr()), None))
                _lib.check(L.rfx_render_frame_counted(rr._h, C.byref(f), 1, C.c_void_p(counts.data_ptr()),
                                                      C.c_void_p(rgb.data_ptr()), C.c_void_p(argb.data_ptr()),
                                                      None, None))
            rr.synchronize()
            print("  synchronized", flush=True)
            out.append((rgb.cpu().numpy().tobytes(), argb.cpu().numpy().tobytes()))
        assert out[0] == out[1], (W, H)
        assert one.get_rng() == two.get_rng(), (W, H)
    one.close()
    two.close()
