"""Look-ahead of rfx_render_frame (rfx.h rfx_renderer_set_lookahead): the next frame's RNG pre-pass runs on a side
stream beside this frame's trace, into the second randDir buffer, and the next call with the same frame plan traces
from it.  It must change no pixel and no stream state (trace_math.h:34-39: the reference's stream carries across
frames): the same call sequence with look-ahead on every frame (mode 2) and off (mode 0) gives identical frames and
states -- repeats that take the look-ahead, plan changes that forget it, state queries and resets in between, event
counts, SSAA + additive, block preview, cursor spans, and rfx_frame_rng_rewind of a frame whose successor was already
emitted ahead.  C1 at full size with the default (mode 1: on below 16384 wave tiles) hashes to the reference.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import manifest, sha
from reflaxman_amd import _lib, scenes

pytestmark = pytest.mark.gpu
SEED = 1350490027


def _sequence(mode, scene, cam):
    import torch
    from reflaxman_amd.render import Renderer, make_frame
    L = _lib.load()
    r = Renderer(sphere_seed=SEED, jitter_seed=99)
    r.set_scene(scene)
    r.set_lookahead(mode)
    W, H = 160, 120
    rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(_lib.RFX_NCOUNTERS, dtype=torch.int64, device="cuda")
    out = []

    def frame(f, counters=False):
        r.render_frame(f, rgb.data_ptr(), argb.data_ptr(), cnt.data_ptr() if counters else 0)
        torch.cuda.synchronize()
        out.append((sha(rgb.cpu().numpy()), sha(argb.cpu().numpy())))

    plain = make_frame(cam, W, H, 6, 1)
    for _ in range(3):
        frame(plain)                                   # the second and third take the look-ahead
    frame(make_frame(cam, W, H, 6, 1, pixel_begin=0, pixel_end=5000))  # another plan: forgets it
    frame(make_frame(cam, W, H, 6, 1, pixel_begin=5000, pixel_end=W * H))
    frame(plain)
    out.append(r.get_rng())                            # a state query forgets the pending look-ahead
    frame(plain)
    frame(plain, counters=True)                        # event counts from emitted-ahead randDirs
    out.append(tuple(int(x) for x in cnt.cpu().numpy()))
    for k in (1, 2, 3):                                # SSAA 2x2, additive accumulation (jitter stream)
        frame(make_frame(cam, W, H, 4, 2, additive=True, additive_counter=k))
    frame(make_frame(cam, W, H, 4, -3))                # block preview
    frame(make_frame(cam, W, H, 4, -3))
    frame(plain)
    frame(plain)
    _lib.check(L.rfx_frame_rng_rewind(r._h))          # undo a frame whose successor was emitted ahead ...
    frame(plain)                                       # ... and render it again: the same frame
    frame(plain)
    r.set_rng(4242, 7)                                 # a reset forgets it too
    frame(plain)
    frame(plain)
    out.append(r.get_rng())
    r.close()
    return out


def test_lookahead_changes_no_frame_and_no_state():
    from reflaxman_amd.render import build_scene
    scene, cam = build_scene(scenes.get_scene("default"))
    off = _sequence(0, scene, cam)
    on = _sequence(2, scene, cam)
    assert len(on) == len(off)
    for i, (a, b) in enumerate(zip(on, off)):
        assert a == b, i
    # the rewound frame (the 15th) was rendered again identically (the 16th)
    frames = [x for x in on if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], str)]
    assert len(frames) == 19 and frames[14] == frames[15], "the rewound frame differs from its first rendering"


def test_lookahead_c1_full_size_frames():
    """C1 (640x480 d4) with the default look-ahead (on: 4,800 wave tiles): 6 frames equal the frames without it, the
    first equals the reference's SHA-256."""
    import torch
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    c = manifest()["cases"]["hash_default_640x480_d4"]
    scene, cam = build_scene(scenes.get_scene("default"))
    W, H = c["W"], c["H"]
    hashes = {}
    for mode in (1, 0):
        r = Renderer(sphere_seed=c["sphere_seed"])
        r.set_scene(scene)
        r.set_lookahead(mode)
        rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
        argb = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        f = make_frame(cam, W, H, c["depth"], 1)
        hs = []
        for _ in range(6):
            r.render_frame(f, rgb.data_ptr(), argb.data_ptr())
            torch.cuda.synchronize()
            hs.append((sha(rgb.cpu().numpy()), sha(argb.cpu().numpy().view(np.uint32))))
        hashes[mode] = hs
        r.close()
    assert hashes[1][0] == (c["sha_f32"], c["sha_argb"])
    assert hashes[1] == hashes[0]
