"""The multi-GPU orchestration (reflaxman_amd/dist.py) with world_size 2 over gloo on CPU.

The renderer is replaced by a CPU stand-in with the same three entry points
(blocks_per_slice / rng_count / render_counted) so the collectives -- the
count all-gather and the ARGB strip gather + un-interleave -- run for real.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from reflaxman_amd import dist as rdist
from reflaxman_amd import _lib


class FakeOps:
    """Slice counts of the n-th count call = slice * 1000 + 100 * n + block (so a frame that traced with another
    frame's counts shows); strip pixels = (frame row << 12) | x."""

    def __init__(self, W, H, rb, rank, world, bps=5):
        self.W, self.H, self.rb, self.rank, self.world, self.bps = W, H, rb, rank, world, bps
        self.seen_counts = None
        self.frame = 0
        self.ncount = 0
        self.band = None  # (y0, y1): band partition (whole-frame buffers, absolute rows)

    def set_rows(self, y0, y1):
        self.band = (y0, y1)

    def blocks_per_slice(self, nslices):
        return self.bps

    def rng_count(self, slice_, nslices, d_counts, stream=0):
        t = torch.from_numpy(__import__("numpy").ctypeslib.as_array(
            (__import__("ctypes").c_int32 * (nslices * self.bps)).from_address(d_counts)))
        for b in range(self.bps):
            t[slice_ * self.bps + b] = slice_ * 1000 + 100 * self.ncount + b
        self.ncount += 1

    def render_counted(self, nslices, d_counts, d_img, d_argb, d_counters=0, emitted_event=0):
        import ctypes
        import numpy as np
        cnt = np.ctypeslib.as_array((ctypes.c_int32 * (nslices * self.bps)).from_address(d_counts)).copy()
        self.seen_counts = cnt
        if self.band:  # whole-frame buffers, the band's rows written in place
            rows = self.H
            ys = [(y, y) for y in range(*self.band)]
        else:
            rows = rdist.strip_rows(self.H, self.rb, self.rank, self.world)
            ys = [(i, rdist.strip_row_to_y(i, self.rb, self.rank, self.world)) for i in range(rows)]
        argb = np.ctypeslib.as_array((ctypes.c_int32 * (rows * self.W)).from_address(d_argb)) if rows else None
        rgb = np.ctypeslib.as_array((ctypes.c_float * (rows * self.W * 3)).from_address(d_img)) if rows else None
        for i, y in ys:
            argb[i * self.W:(i + 1) * self.W] = (self.frame << 24) | (y << 12) | np.arange(self.W)
            rgb[i * self.W * 3:(i + 1) * self.W * 3] = rgb_pattern(self.frame, y, self.W)
        self.frame += 1


def rgb_pattern(frame, y, W):
    import numpy as np
    return (frame * 100000 + y * 100 + np.arange(3 * W) % 3 + 10 * (np.arange(3 * W) // 3)).astype(np.float32)


def _worker(rank, world, port, W, H, rb, pipeline, q, gather_rgb=False, count_ahead=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = FakeOps(W, H, rb, rank, world)
        sf = rdist.StripFrame(ops, W, H, rb, rank, world, torch.device("cpu"), pipeline=pipeline,
                              gather_rgb=gather_rgb, count_ahead=count_ahead)
        assert sf.pipeline == pipeline and sf.count_ahead == count_ahead
        ok_counts = ok_frame = True
        for frame in range(4):  # four frames: both buffer sets of the pipeline, each reused
            if frame == 2:
                sf.drop_lookahead()  # the counts of a look-ahead are discarded: frame 2 counts afresh
            out = sf.step()
            n = frame + 1 if count_ahead and frame >= 2 else frame  # the count call whose counts frame uses
            expect = [s * 1000 + 100 * n + b for s in range(world) for b in range(ops.bps)]
            ok_counts &= ops.seen_counts.tolist() == expect
            if rank == 0:
                ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
                ok_frame &= bool(torch.equal(out, ((frame << 24) | (ys << 12) | xs).to(torch.int32)))
                if gather_rgb:
                    import numpy as np
                    want = np.stack([rgb_pattern(frame, y, W) for y in range(H)]).reshape(H, W, 3)
                    ok_frame &= bool(np.array_equal(sf.rgb_full.numpy(), want))
            else:
                ok_frame &= out is None
        q.put((rank, ok_counts, ok_frame))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("pipeline,gather_rgb,count_ahead", [(False, False, False), (True, False, False),
                                                              (False, True, False), (True, True, False),
                                                              (False, False, True), (True, True, True)])
@pytest.mark.parametrize("W,H,rb", [(16, 37, 4), (8, 64, 8), (5, 3, 8)])
def test_strip_frame_world2_gloo(W, H, rb, pipeline, gather_rgb, count_ahead):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, rb, pipeline, q, gather_rgb, count_ahead))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True, True), (1, True, True)], res


def test_strip_helpers_match_library():
    L = _lib.load()
    for H in (1, 7, 123, 2160, 4320, 6109):
        for world in (1, 2, 3, 4, 8):
            for rb in (1, 8, 16):
                for r in range(world):
                    assert rdist.strip_rows(H, rb, r, world) == L.rfx_strip_rows(H, rb, r, world)
                    n = rdist.strip_rows(H, rb, r, world)
                    for i in (0, n // 2, n - 1) if n else ():
                        assert rdist.strip_row_to_y(i, rb, r, world) == L.rfx_strip_row_to_y(i, rb, r, world)


def _band_worker(rank, world, port, W, H, pipeline, q, gather_rgb, count_ahead, toggle=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np
        ops = FakeOps(W, H, 0, rank, world)
        sf = rdist.BandFrame(ops, W, H, rank, world, torch.device("cpu"), pipeline=pipeline, gather_rgb=gather_rgb,
                             count_ahead=count_ahead, grain=2)
        ok_frame = True
        bounds = []
        for frame in range(5):
            if frame == 2:
                # re-cut the bands from fake per-rank times (rank r's rows cost r + 1 each): the frames stay whole
                nb = sf.balance(rounds=2, timer=lambda step: (step(), sf.rows * (sf.rank + 1))[1])
                bounds.append(nb)
            if toggle and frame == 3:  # bench.py's second timing: the f32 plane sent too, from the next frame on
                sf.set_gather_rgb(not gather_rgb)
                gather_rgb = not gather_rgb
            out = sf.step()
            fno = ops.frame - 1
            if rank == 0:
                ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
                ok_frame &= bool(torch.equal(out, ((fno << 24) | (ys << 12) | xs).to(torch.int32)))
                if gather_rgb:
                    want = np.stack([rgb_pattern(fno, y, W) for y in range(H)]).reshape(H, W, 3)
                    ok_frame &= bool(np.array_equal(sf.rgb_full.numpy(), want))
            else:
                ok_frame &= out is None
        q.put((rank, ok_frame, bounds[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipeline,gather_rgb,count_ahead,toggle", [(False, False, False, False),
                                                                     (True, True, True, False),
                                                                     (True, False, True, True),
                                                                     (False, True, False, True)])
@pytest.mark.parametrize("world,W,H", [(2, 16, 37), (3, 8, 64)])
def test_band_frame_gloo(world, W, H, pipeline, gather_rgb, count_ahead, toggle):
    """Bands over gloo: whole frames on rank 0, re-balanced mid-run; with `toggle`, the f32 RGB plane's transfer is
    switched on (or off) after frame 3 (BandFrame.set_gather_rgb, bench.py's with_rgb_gather timing)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, W, H, pipeline, q, gather_rgb, count_ahead, toggle))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert [r[1] for r in res] == [True] * world, res
    b = res[0][2]
    assert all(r[2] == b for r in res)  # every rank cut the same bands
    assert b[0] == 0 and b[-1] == H and all(b[i] < b[i + 1] for i in range(world))
    assert b[1] - b[0] > b[world] - b[world - 1]  # the cheap rank 0 took more rows than the dearest


def test_balanced_bounds():
    # uniform cost: equal bands; a band twice as dear per row: cut where the cumulative cost halves
    assert rdist.balanced_bounds([0, 50, 100], [1.0, 1.0], 100, 1) == [0, 50, 100]
    assert rdist.balanced_bounds([0, 50, 100], [1.0, 3.0], 100, 1) == [0, 67, 100]
    b = rdist.balanced_bounds(rdist.equal_bounds(4320, 8), [1, 1, 1, 1, 2, 2, 2, 2], 4320)
    assert b[0] == 0 and b[-1] == 4320 and all(x % 8 == 0 for x in b) and b == sorted(set(b))
    # degenerate inputs keep valid bands
    assert rdist.balanced_bounds([0, 8, 16, 24], [0.0, 1.0, 1e9], 24, 8) == [0, 8, 16, 24]


class FakePassOps(FakeOps):
    """A stand-in whose random stream is a counter: slice counts encode the counting rank's stream state, a band
    emit checks that every slice of the all-gathered counts came from the same state and advances the state by the
    span's rows, and band pixels are (frame << 24) | (y << 12) | x."""

    def __init__(self, W, H, rank, world, bps=3):
        super().__init__(W, H, 0, rank, world, bps)
        self.state, self.jitter, self.span, self.fno = 7, 0, None, 0
        self.consistent = True
        self.passes_traced = 0

    def set_span(self, y0, y1):
        self.span = (y0, y1)

    def rng_state(self):
        return self.state, self.jitter

    def set_rng_state(self, sphere, jitter):
        self.state, self.jitter = sphere, jitter

    def rng_count(self, slice_, nslices, d_counts, stream=0):
        import ctypes
        import numpy as np
        t = np.ctypeslib.as_array((ctypes.c_int32 * (nslices * self.bps)).from_address(d_counts))
        for b in range(self.bps):
            t[slice_ * self.bps + b] = (self.state * 10 + slice_) * 100 + b

    def render_counted(self, nslices, d_counts, d_img, d_argb, d_counters=0, emitted_event=0):
        import ctypes
        import numpy as np
        cnt = np.ctypeslib.as_array((ctypes.c_int32 * (nslices * self.bps)).from_address(d_counts)).copy()
        want = [(self.state * 10 + s) * 100 + b for s in range(nslices) for b in range(self.bps)]
        self.consistent &= cnt.tolist() == want
        y0, y1 = self.band
        assert self.span[0] <= y0 < y1 <= self.span[1]
        argb = np.ctypeslib.as_array((ctypes.c_int32 * (self.H * self.W)).from_address(d_argb))
        for y in range(y0, y1):
            argb[y * self.W:(y + 1) * self.W] = (self.fno << 24) | (y << 12) | np.arange(self.W)
        self.state += self.span[1] - self.span[0]
        self.jitter += 1
        self.passes_traced += 1


def _pass_worker(rank, world, port, W, H, ss, launch_traces, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = FakePassOps(W, H, rank, world)
        sf = rdist.BandFrame(ops, W, H, rank, world, torch.device("cpu"), pipeline=False, ss=ss,
                             launch_traces=launch_traces)
        assert sf.passes and not sf.count_ahead and not sf.emit_ahead
        ok = True
        for frame in range(3):
            ops.fno = frame
            out = sf.step()
            if rank == 0:
                ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
                ok &= bool(torch.equal(out, ((frame << 24) | (ys << 12) | xs).to(torch.int32)))
            else:
                ok &= out is None
        q.put((rank, ok, ops.consistent, ops.state, ops.jitter, ops.passes_traced, len(sf.passes)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,ss,launch_traces", [
    (2, 8, 10, 2, 8 * 4 * 3 // 2),   # passes of 3 rows (the last of 1): a rank sits out the last pass
    (3, 8, 10, 2, 8 * 4 * 2 // 3),   # passes of 2 rows: every pass leaves one of 3 ranks out
    (3, 6, 13, 3, 6 * 9 * 4 // 3),   # passes of 4 rows, the last of 1
    (2, 5, 8, 4, 5 * 16 * 2),        # passes of 4 rows, 2 per rank: no rank sits out, no handover
])
def test_band_frame_row_span_passes_gloo(world, W, H, ss, launch_traces):
    """The RCCL path's frames of more traces than one pass (SSAA screenshots): row-span passes with the count exchange
    per pass, the stream continued across passes and frames, ranks that sit a pass out brought up to rank 0's stream
    state, every band on rank 0 (reflaxman_amd/dist.py BandFrame._step_passes)."""
    plan = rdist.pass_plan(W, H, ss, world, launch_traces)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pass_worker, args=(r, world, port, W, H, ss, launch_traces, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(r[1] and r[2] for r in res), res  # whole frames on rank 0; every pass saw one stream state
    assert {r[3] for r in res} == {7 + 3 * H}    # every rank ends where the serial stream does (3 frames x H rows)
    assert len({r[4] for r in res}) == 1         # and with the same jitter state
    assert res[0][5] == 3 * len(plan)            # rank 0 traced every pass


def test_pass_plan_matches_the_group_rule():
    """dist.pass_plan cuts frames the way rfx_group_render_frame does (rfx_group.cpp: at most min(N x launch limit, 2^31)
    traces per pass, whole rows), every pass within 2^31 traces; pass_bands gives min(N, rows) equal bands."""
    assert rdist.pass_plan(3840, 2160, 1, 8) is None          # C3/C4-sized one-sample frames take one pass
    assert rdist.pass_plan(7680, 4320, 1, 2) is None
    for W, H, ss, N in [(1920, 1080, 128, 1), (1920, 1080, 128, 2), (1920, 1080, 128, 8), (800, 600, 128, 4),
                        (7680, 4320, 256, 8), (1280, 720, 64, 2), (7680, 4320, 16, 8)]:
        plan = rdist.pass_plan(W, H, ss, N)
        assert plan, (W, H, ss, N)
        cap = min(N * rdist.LAUNCH_TRACES, rdist.MAX_PASS_TRACES)
        assert plan[0][0] == 0 and plan[-1][1] == H and all(a[1] == b[0] for a, b in zip(plan, plan[1:]))
        assert all((y1 - y0) * W * ss * ss <= cap for y0, y1 in plan)
        assert all(y1 - y0 == plan[0][1] for y0, y1 in plan[:-1])  # equal passes, the last one shorter
        for y0, y1 in plan:
            bd = rdist.pass_bands(y0, y1, N)
            assert bd[0] == y0 and bd[-1] == y1 and len(bd) - 1 == min(N, y1 - y0)
            assert all(b > a for a, b in zip(bd, bd[1:]))
            for r in range(N):
                a, b = rdist.pass_rows(bd, r, y1)
                assert y0 <= a < b <= y1
    # 7680 x 256^2 samples: 4 rows a pass, so 4 of 8 ranks sit every pass out
    assert rdist.pass_plan(7680, 4320, 256, 8)[0] == (0, 4)
    # 1280x720 at 64x64 (3.8e9 traces, between 2^31 and 2^32): passes, no longer refused (round-5 advice)
    assert len(rdist.pass_plan(1280, 720, 64, 2)) == 2
