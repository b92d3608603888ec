"""Multi-GPU steady state, emulated in one process on one GPU: frames >= 1, not just frame 0.

N ranks, each with its own renderer and its own two streams (a main stream and the side stream of the
look-aheads), replay the per-frame choreography of reflaxman_amd/dist.py at its defaults over 8 frames
(Render.cpp:136-215 partitioned; the random stream carried across frames, trace_math.h:34-39):

* frame 0: every rank counts its slice of the random stream, the counts are exchanged (device copies between the
  ranks' count arrays, ordered by events, standing in for the RCCL all-gather), then emit + trace on the main stream;
* from then on, right after each trace is enqueued, the NEXT frame's count, exchange and emit run on the side
  stream (count-ahead + emit-ahead: rfx_frame_rng_emit into the renderer's second randDir buffer, after the trace
  before the current one), and the main stream traces it with rfx_render_frame_emitted;
* bands only: after frame 2 the bands are re-cut (as BandFrame.balance() does): every rank drops the look-ahead it
  has already emitted (rfx_frame_rng_discard restores the stream state) and the next frame counts afresh;
* frame 5 is bench.py's counted frame: look-aheads dropped, rfx_render_frame with event counters on every rank;
* per-view primary masks (built when a view repeats, so from each rank's second frame of a band on) and the
  longest-tile-first schedule (mode 1 at C4 size, forced with mode 3 on the smaller frames) stay at work.

Each frame's bands (or strips) are assembled on a third stream while the next frame renders (double-buffered
outputs) and compared bit for bit with the same-index frame of a single-GPU renderer; frame 0 at C4 size also
equals the reference's SHA-256 (tests/golden/manifest.json).
"""
import ctypes as C

import numpy as np
import pytest

from helpers import manifest, sha
from reflaxman_amd import _lib, scenes
from reflaxman_amd.dist import equal_bounds, strip_row_to_y, strip_rows

pytestmark = pytest.mark.gpu

SEED = 1350490027
RECUT_AFTER = 2
COUNTED_FRAME = 5
FRAMES = 8


class _Rank:
    def __init__(self, torch, L, scene, cam, W, H, D, rank, world, partition, bounds, tile_order, dev):
        from reflaxman_amd.render import Renderer, make_frame
        self.torch, self.L, self.rank, self.world, self.W, self.H = torch, L, rank, world, W, H
        self.rr = Renderer(sphere_seed=SEED)
        self.rr.set_scene(scene)
        if tile_order is not None:
            self.rr.set_tile_order(tile_order)
        self.main = torch.cuda.Stream(device=dev)
        self.side = torch.cuda.Stream(device=dev)
        self.rr.set_stream(self.main.cuda_stream)
        self.bands = partition == "bands"
        if self.bands:
            self.f = make_frame(cam, W, H, D, 1, row_block=0, rank=rank, nranks=world)
            self.set_rows(bounds)
            self.rows = H
        else:
            self.f = make_frame(cam, W, H, D, 1, row_block=8, rank=rank, nranks=world)
            self.rows = strip_rows(H, 8, rank, world)
        bps = C.c_uint64()
        _lib.check(L.rfx_frame_rng_blocks(self.rr._h, C.byref(self.f), world, C.byref(bps)))
        self.bps = bps.value
        self.counts = torch.zeros(world * self.bps, dtype=torch.int32, device=dev)
        self.img = [torch.zeros(self.rows * W * 3, dtype=torch.float32, device=dev) for _ in range(2)]
        self.argb = [torch.zeros(self.rows * W, dtype=torch.int32, device=dev) for _ in range(2)]
        ev = lambda: torch.cuda.Event()
        self.emitted, self.counted, self.copied = ev(), ev(), ev()
        self.trace_done = [ev(), ev()]
        for e in (self.emitted, self.counted, self.copied, *self.trace_done):
            e.record(self.main)  # the hipEvent_t exists from its first record
        self.emit_ready = False
        self.n = 0

    def set_rows(self, bounds):
        self.y0, self.y1 = bounds[self.rank], bounds[self.rank + 1]
        self.f.pixel_begin, self.f.pixel_end = self.y0 * self.W, self.y1 * self.W

    def count(self, stream, ranks):
        for q in ranks:  # every rank has copied this rank's previous counts
            stream.wait_event(q.copied)
        _lib.check(self.L.rfx_frame_rng_count(self.rr._h, C.byref(self.f), self.rank, self.world,
                                              C.c_void_p(self.counts.data_ptr()), C.c_void_p(stream.cuda_stream)))
        self.counted.record(stream)

    def emit(self, stream):
        _lib.check(self.L.rfx_frame_rng_emit(self.rr._h, C.byref(self.f), self.world, C.c_void_p(self.counts.data_ptr()),
                                             C.c_void_p(stream.cuda_stream), C.c_void_p(self.emitted.cuda_event)))

    def drop_lookahead(self):
        self.main.wait_stream(self.side)
        if self.emit_ready:
            _lib.check(self.L.rfx_frame_rng_discard(self.rr._h))
            self.emit_ready = False


def _exchange(torch, ranks, stream_of):
    """The all-gather of the slice counts: each rank's slice copied into every other rank's array."""
    for r in ranks:
        s = stream_of(r)
        with torch.cuda.stream(s):
            for q in ranks:
                if q is r:
                    continue
                s.wait_event(q.counted)
                sl = slice(q.rank * q.bps, (q.rank + 1) * q.bps)
                r.counts[sl].copy_(q.counts[sl])
        r.copied.record(s)


def _run(partition, world, W, H, D, tile_order, bounds=None, recut=None):
    import torch
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L = _lib.load()
    scene, cam = build_scene(scenes.get_scene("synth16"))
    bounds = bounds or equal_bounds(H, world)
    ranks = [_Rank(torch, L, scene, cam, W, H, D, r, world, partition, bounds, tile_order, dev) for r in range(world)]
    asm = torch.cuda.Stream(device=dev)
    asm_done = [torch.cuda.Event(), torch.cuda.Event()]
    for e in asm_done:
        e.record(asm)
    ys = None
    if partition == "strips":
        ys = [torch.tensor([strip_row_to_y(i, 8, r.rank, world) for i in range(r.rows)], dtype=torch.int64, device=dev)
              for r in ranks]
    frames = []  # assembled (rgb, argb) per frame
    cnt = torch.zeros(_lib.RFX_NCOUNTERS, dtype=torch.int64, device=dev)
    for i in range(FRAMES):
        k = i % 2
        if partition == "bands" and i == RECUT_AFTER + 1:
            bounds = recut
            for r in ranks:
                r.drop_lookahead()
                r.set_rows(bounds)
        if i == COUNTED_FRAME:
            for r in ranks:  # bench.py counted_frame(): look-aheads dropped, rfx_render_frame with counters
                r.drop_lookahead()
                r.main.wait_event(asm_done[k])
                r.rr.render_frame(r.f, r.img[k].data_ptr(), r.argb[k].data_ptr(), cnt.data_ptr(), r.main.cuda_stream)
                r.n += 1
                r.trace_done[r.n % 2].record(r.main)
        else:
            if not ranks[0].emit_ready:  # nothing emitted ahead: count, exchange and emit on the main streams
                for r in ranks:
                    r.count(r.main, ranks)
                _exchange(torch, ranks, lambda r: r.main)
                for r in ranks:
                    r.emit(r.main)
            else:
                for r in ranks:
                    r.main.wait_event(r.emitted)
            for r in ranks:
                r.emit_ready = False
                r.main.wait_event(asm_done[k])  # frame i - 2's assembly has read buffer set k
                _lib.check(L.rfx_render_frame_emitted(r.rr._h, C.byref(r.f), C.c_void_p(r.img[k].data_ptr()),
                                                      C.c_void_p(r.argb[k].data_ptr()), None,
                                                      C.c_void_p(r.main.cuda_stream)))
                r.n += 1
                r.trace_done[r.n % 2].record(r.main)
            # the next frame's count, exchange and emit on the side streams, while this frame traces (a re-cut or
            # the counted frame discards it again, as dist.py's drop_lookahead does)
            for r in ranks:
                r.side.wait_event(r.emitted)
                r.count(r.side, ranks)
            _exchange(torch, ranks, lambda r: r.side)
            for r in ranks:
                r.side.wait_event(r.trace_done[(r.n - 1) % 2])  # the last reader of the emit's buffer
                r.emit(r.side)
                r.emit_ready = True
        # assemble frame i on its own stream (rank 0's receive), while the next frame renders
        rgb = torch.empty(H * W * 3, dtype=torch.float32, device=dev)
        argb = torch.empty(H * W, dtype=torch.int32, device=dev)
        with torch.cuda.stream(asm):
            for r in ranks:
                asm.wait_event(r.trace_done[r.n % 2])
                if partition == "bands":
                    a, b = r.y0 * W, r.y1 * W
                    argb[a:b].copy_(r.argb[k][a:b])
                    rgb[3 * a:3 * b].copy_(r.img[k][3 * a:3 * b])
                else:
                    argb.view(H, W).index_copy_(0, ys[r.rank], r.argb[k].view(r.rows, W))
                    rgb.view(H, W * 3).index_copy_(0, ys[r.rank], r.img[k].view(r.rows, W * 3))
            asm_done[k].record(asm)
        frames.append((rgb, argb))
    torch.cuda.synchronize()
    for r in ranks:
        r.rr.close()
    # the same frames on one GPU, one after the other
    one = Renderer(sphere_seed=SEED)
    one.set_scene(scene)
    f1 = make_frame(cam, W, H, D, 1)
    rgb1 = torch.empty(H * W * 3, dtype=torch.float32, device=dev)
    argb1 = torch.empty(H * W, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    equal = []
    for i in range(FRAMES):
        one.render_frame(f1, rgb1.data_ptr(), argb1.data_ptr(), 0, s.cuda_stream)
        torch.cuda.synchronize()
        equal.append(bool(torch.equal(frames[i][0], rgb1)) and bool(torch.equal(frames[i][1], argb1)))
    one.close()
    return equal, frames


@pytest.mark.parametrize("world,size,tile_order", [(2, (1920, 1080), 3), (4, (1920, 1080), 3), (8, (7680, 4320), None)])
def test_bands_steady_state_equals_single_gpu(world, size, tile_order):
    W, H = size
    start = equal_bounds(H, world)
    # re-cut as the balancer does: uneven, multiples of 8 rows, one band 8 rows high
    cut = [0] + [min(H - 8 * (world - r), max(8 * r, (H * r // world + (-1) ** r * 8 * (r + 3)) // 8 * 8))
                 for r in range(1, world)] + [H]
    if world > 2:
        cut[2] = cut[1] + 8
    assert all(cut[r] < cut[r + 1] for r in range(world)) and cut != start, cut
    equal, frames = _run("bands", world, W, H, 8, tile_order, bounds=start, recut=cut)
    assert equal == [True] * FRAMES, equal
    if (W, H) == (7680, 4320):
        c = manifest()["cases"]["hash_synth16_7680x4320_d8"]
        assert sha(frames[0][1].cpu().numpy().view(np.uint32)) == c["sha_argb"]
        assert sha(frames[0][0].cpu().numpy()) == c["sha_f32"]


@pytest.mark.parametrize("world,size,tile_order", [(3, (1920, 1080), 3), (4, (7680, 4320), None)])
def test_strips_steady_state_equals_single_gpu(world, size, tile_order):
    W, H = size
    equal, frames = _run("strips", world, W, H, 8, tile_order)
    assert equal == [True] * FRAMES, equal
    if (W, H) == (7680, 4320):
        c = manifest()["cases"]["hash_synth16_7680x4320_d8"]
        assert sha(frames[0][1].cpu().numpy().view(np.uint32)) == c["sha_argb"]
        assert sha(frames[0][0].cpu().numpy()) == c["sha_f32"]


def test_emitted_frame_must_match_its_emit():
    """rfx_render_frame_emitted refuses a frame whose band differs from the emitted one (RFX_ERR_STATE), and traces
    it after rfx_frame_rng_discard + a fresh emit."""
    import torch
    from reflaxman_amd.render import Renderer, build_scene, make_frame
    L = _lib.load()
    scene, cam = build_scene(scenes.get_scene("synth16"))
    W, H = 256, 144
    rr = Renderer(sphere_seed=SEED)
    rr.set_scene(scene)
    f = make_frame(cam, W, H, 8, 1, row_block=0, rank=0, nranks=2, pixel_begin=0, pixel_end=64 * W)
    bps = C.c_uint64()
    _lib.check(L.rfx_frame_rng_blocks(rr._h, C.byref(f), 2, C.byref(bps)))
    cnt = torch.zeros(2 * bps.value, dtype=torch.int32, device="cuda")
    img = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    for sl in range(2):
        _lib.check(L.rfx_frame_rng_count(rr._h, C.byref(f), sl, 2, C.c_void_p(cnt.data_ptr()), None))
    _lib.check(L.rfx_frame_rng_emit(rr._h, C.byref(f), 2, C.c_void_p(cnt.data_ptr()), None, None))
    f.pixel_end = 72 * W  # the band grew after the emit
    rc = L.rfx_render_frame_emitted(rr._h, C.byref(f), C.c_void_p(img.data_ptr()), None, None, None)
    assert rc == -3, rc
    s = C.c_uint32()
    assert L.rfx_frame_rng_pending(rr._h, C.byref(s)) == 1 and s.value == SEED
    _lib.check(L.rfx_frame_rng_discard(rr._h))
    assert L.rfx_frame_rng_pending(rr._h, C.byref(s)) == 0 and s.value == SEED
    _lib.check(L.rfx_frame_rng_emit(rr._h, C.byref(f), 2, C.c_void_p(cnt.data_ptr()), None, None))
    _lib.check(L.rfx_render_frame_emitted(rr._h, C.byref(f), C.c_void_p(img.data_ptr()), None, None, None))
    rr.synchronize()
    rr.close()
