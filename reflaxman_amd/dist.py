"""Multi-GPU frames: row bands (or block-cyclic strips), one RCCL exchange in the RNG pre-pass, frame assembly on
rank 0.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Per
frame, rank r:

1. counts the accepted LCG triples of its 1/N slice of the random stream
   (``rfx_frame_rng_count``) into its slice of a device array;
2. all-gathers that array -- the only exchange the path needs, N x ~1K uint32;
3. scans it, emits the randDirs of *its* rows and traces them
   (``rfx_render_frame_counted``, or ``rfx_frame_rng_emit`` + ``rfx_render_frame_emitted``
   when steps 1-3a run a frame ahead on a side stream) -- pre-pass and trace work are both 1/N;
4. BandFrame: sends its band to rank 0, received in place in the frame (RCCL p2p);
   StripFrame: gathers its ARGB8 strip to rank 0, which un-interleaves the strips
   with one device ``index_copy_`` (rfx_strip_row_to_y).

The assembled frame equals the 1-GPU frame bit-exactly (tests/test_gpu_parity.py
emulates the ranks in one process; tests/test_dist_gloo.py runs this module's
collectives with world_size 2 and 3 over gloo on CPU; tests/test_gpu_multirank.py
runs bench.py with gloo ranks on one GPU and the look-aheads over RCCL).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib


class RfxStripOps:
    """The renderer side of a rank's strip frame (librfx.so C-ABI)."""

    def __init__(self, renderer, frame: _lib.Frame, stream_ptr: int):
        if not stream_ptr:
            # NULL would select the renderer's own non-blocking stream, unordered with the collectives
            raise ValueError("RfxStripOps needs the (non-default) torch stream the collectives run on")
        self.r = renderer
        self.frame = frame
        self.stream = stream_ptr
        self.L = _lib.load()

    def rng_emit(self, nslices: int, d_counts: int, stream: int = 0, emitted_event: int = 0):
        """Emit-ahead: the next frame's randDirs from the all-gathered counts, on `stream` (rfx_frame_rng_emit)."""
        _lib.check(self.L.rfx_frame_rng_emit(self.r._h, C.byref(self.frame), nslices, C.c_void_p(d_counts),
                                             C.c_void_p(stream or self.stream), C.c_void_p(emitted_event or None)),
                   "frame_rng_emit")

    def render_emitted(self, d_img: int, d_argb: int, d_counters: int = 0):
        """Emit-ahead: trace the emitted frame on the ops' stream (rfx_render_frame_emitted)."""
        _lib.check(self.L.rfx_render_frame_emitted(self.r._h, C.byref(self.frame), C.c_void_p(d_img),
                                                   C.c_void_p(d_argb or None), C.c_void_p(d_counters or None),
                                                   C.c_void_p(self.stream or None)), "render_frame_emitted")

    def rng_discard(self):
        _lib.check(self.L.rfx_frame_rng_discard(self.r._h), "frame_rng_discard")

    def rng_pending(self) -> int:
        """The sphere-stream state the next traced frame starts from (rfx_frame_rng_pending; synchronises)."""
        s = C.c_uint32()
        _lib.check(self.L.rfx_frame_rng_pending(self.r._h, C.byref(s)), "frame_rng_pending")
        return s.value

    def set_rows(self, y0: int, y1: int):
        """Band partition: this rank traces rows [y0, y1) (rfx.h: row_block 0, pixel span of whole rows)."""
        self.frame.row_block = 0
        self.frame.pixel_begin, self.frame.pixel_end = y0 * self.frame.width, y1 * self.frame.width

    def set_span(self, y0: int, y1: int):
        """The rows [y0, y1) the random stream of the next band frames runs over (rfx.h span_begin / span_end; 0, 0:
        the whole frame)."""
        self.frame.span_begin, self.frame.span_end = y0 * self.frame.width, y1 * self.frame.width

    def rng_state(self):
        """(sphere stream state, jitter stream state) of the renderer (synchronises its stream)."""
        return self.r.get_rng()

    def set_rng_state(self, sphere: int, jitter: int):
        self.r.set_rng(sphere, jitter)

    def blocks_per_slice(self, nslices: int) -> int:
        bps = C.c_uint64()
        _lib.check(self.L.rfx_frame_rng_blocks(self.r._h, C.byref(self.frame), nslices, C.byref(bps)), "rng_blocks")
        return bps.value

    def rng_count(self, slice_: int, nslices: int, d_counts: int, stream: int = 0):
        """Count the accepted triples of slice `slice_` of the NEXT frame's stream (from the state the last emit
        left), on `stream` (default: the ops' stream)."""
        _lib.check(self.L.rfx_frame_rng_count(self.r._h, C.byref(self.frame), slice_, nslices, C.c_void_p(d_counts),
                                              C.c_void_p(stream or self.stream)), "rng_count")

    def render_counted(self, nslices: int, d_counts: int, d_img: int, d_argb: int, d_counters: int = 0,
                       emitted_event: int = 0):
        """Scan the all-gathered counts, emit this rank's randDirs (then record `emitted_event`, a hipEvent_t,
        if given) and trace its strips."""
        _lib.check(self.L.rfx_render_frame_counted_ev(self.r._h, C.byref(self.frame), nslices, C.c_void_p(d_counts),
                                                      C.c_void_p(d_img), C.c_void_p(d_argb or None),
                                                      C.c_void_p(d_counters or None), C.c_void_p(self.stream or None),
                                                      C.c_void_p(emitted_event or None)),
                   "render_frame_counted")


class _Done:
    """An exchange that already completed (gloo on CPU)."""

    def wait(self):
        pass


class _EventWork:
    """A completed-on-device step as a work object: wait() orders the current stream after it."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def strip_rows(H: int, row_block: int, rank: int, world: int) -> int:
    """Rows of rank `rank` under block-cyclic strips (== rfx_strip_rows)."""
    if world <= 1:
        return H
    full, rem = divmod(H, row_block)
    rows = (full // world) * row_block + (row_block if rank < full % world else 0)
    if rem and full % world == rank:
        rows += rem
    return rows


def strip_row_to_y(i: int, row_block: int, rank: int, world: int) -> int:
    """Frame row of strip row i (== rfx_strip_row_to_y)."""
    if world <= 1:
        return i
    return (i // row_block * world + rank) * row_block + i % row_block


class _CountedFrame:
    """The per-frame RNG exchange of a partitioned frame (strips or bands): every rank counts its slice of the
    frame's random stream, the slice counts are all-gathered, and the emit scans them (rfx.h
    rfx_frame_rng_count / rfx_render_frame_counted).

    count_ahead (default: on for the nccl backend): frame i+1's RNG count and its all-gather (their own
    communicator, on a side stream) start as soon as frame i's randDirs are emitted -- the next frame's
    stream state is then on the device -- and run while frame i traces, so the exchange step leaves the
    per-frame critical path (count, all-gather, emit, trace becomes emit, trace).  The renderer's random
    stream must not advance between steps by any other call (drop_lookahead() first, on every rank).

    emit_ahead (default: with count_ahead on a device): frame i+1's emit too runs on the side stream, into the
    renderer's second randDir buffer, while frame i traces (rfx_frame_rng_emit / rfx_render_frame_emitted): the
    critical path becomes the trace alone.  The emit waits for the trace before frame i, the last reader of the
    buffer it overwrites.
    """

    def _init_counts(self, ops, rank: int, world: int, device: torch.device, count_ahead: Optional[bool],
                     emit_ahead: Optional[bool] = None):
        self.ops, self.rank, self.world, self.device = ops, rank, world, device
        self.bps = ops.blocks_per_slice(world)
        self.counts = torch.zeros(world * self.bps, dtype=torch.int32, device=device)
        cuda = device.type == "cuda"
        if count_ahead is None:
            # on for RCCL, and for gloo ranks sharing one GPU (the one-box rehearsal runs the same stream and
            # buffer choreography, its all-gathers staged through host memory on the side stream)
            count_ahead = world > 1 and (dist.get_backend() == "nccl" or self._host_staged())
        # (asked for explicitly it also runs at world 1: the device-side ordering test, tests/test_gpu_multirank.py)
        self.count_ahead = bool(count_ahead)
        self.count_group = dist.new_group(list(range(world))) if self.count_ahead else None
        self.count_stream = torch.cuda.Stream(device=device) if self.count_ahead and cuda else None
        self.emitted = torch.cuda.Event() if self.count_ahead and cuda else None
        if self.emitted is not None:
            self.emitted.record(torch.cuda.current_stream(device))  # torch creates the hipEvent_t at its first record
        self.ahead = None  # the next frame's count all-gather in flight (its work object), once one is
        if emit_ahead is None:
            emit_ahead = self.count_ahead
        self.emit_ahead = bool(emit_ahead) and self.count_ahead and cuda and hasattr(ops, "rng_emit")
        self.emit_ready = False  # emit-ahead: the next frame's randDirs are emitted (self.emitted marks when)
        self.trace_done = [torch.cuda.Event(), torch.cuda.Event()] if self.emit_ahead else []
        for e in self.trace_done:
            e.record(torch.cuda.current_stream(device))
        self._n = 0  # frames rendered (emit-ahead bookkeeping)
        self._emit_events: Optional[list] = None  # time_emits(): (start, end) events around each side-stream emit

    def _frame_counts(self):
        """This frame's all-gathered slice counts in self.counts, ordered before the emit on this stream."""
        if self.emit_ahead and self.emit_ready:
            return  # counted, all-gathered and emitted on the side stream
        if self.ahead is not None:
            # counted and all-gathered while the last frame traced: order this stream after them
            self.ahead.wait()
        else:
            self.ops.rng_count(self.rank, self.world, self.counts.data_ptr())
            if self.world > 1:
                self._all_gather_counts()
        self.ahead = None

    def _render(self, img: torch.Tensor, argb: torch.Tensor, d_counters: int, events: Optional[list] = None):
        """This frame's emit (unless emitted ahead) and trace, and the next frame's look-ahead.  events: a (start,
        end) pair of timing events to record around the trace."""
        if not self.emit_ahead:
            if events:
                events[0].record()
            self.ops.render_counted(self.world, self.counts.data_ptr(), img.data_ptr(), argb.data_ptr(), d_counters,
                                    self.emitted.cuda_event if self.emitted is not None else 0)
            if events:
                events[1].record()
            if self.count_ahead:
                self._count_next()
            return
        main = torch.cuda.current_stream(self.device)
        if not self.emit_ready:  # nothing emitted ahead: this frame's counts are in self.counts
            self.ops.rng_emit(self.world, self.counts.data_ptr(), stream=main.cuda_stream,
                              emitted_event=self.emitted.cuda_event)
        else:
            main.wait_event(self.emitted)
        self.emit_ready = False
        if events:
            events[0].record()
        self.ops.render_emitted(img.data_ptr(), argb.data_ptr(), d_counters)
        if events:
            events[1].record()
        self._n += 1
        self.trace_done[self._n % 2].record(main)
        # the next frame: count its slice, all-gather, and emit it -- all on the side stream
        with torch.cuda.stream(self.count_stream):
            self.count_stream.wait_event(self.emitted)  # the stream state past this frame
            self.ops.rng_count(self.rank, self.world, self.counts.data_ptr(), stream=self.count_stream.cuda_stream)
            w = self._all_gather_counts(group=self.count_group, async_op=True)
            if w is not None:
                w.wait()  # the side stream waits for the all-gather
            self.count_stream.wait_event(self.trace_done[(self._n - 1) % 2])  # the last reader of the emit's buffer
            ev = None
            if self._emit_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(self.count_stream)
                self._emit_events.append(ev)
            self.ops.rng_emit(self.world, self.counts.data_ptr(), stream=self.count_stream.cuda_stream,
                              emitted_event=self.emitted.cuda_event)
            if ev is not None:
                ev[1].record(self.count_stream)
        self.emit_ready = True

    def time_emits(self, enable: bool) -> Optional[float]:
        """Time the look-ahead emits on the side stream (HIP events there): enable, render, then disable to read the
        average ms per emit (synchronises; None without emit-ahead or emits)."""
        if enable:
            self._emit_events = [] if self.emit_ahead else None
            return None
        ev, self._emit_events = self._emit_events, None
        if not ev:
            return None
        torch.cuda.synchronize(self.device)
        return sum(s.elapsed_time(e) for s, e in ev) / len(ev)

    def _count_next(self):
        """Count the next frame's slice and start its all-gather, ordered after this frame's emit only."""
        if self.count_stream is None:  # CPU (gloo orchestration tests): the ops are synchronous
            self.ops.rng_count(self.rank, self.world, self.counts.data_ptr())
            self.ahead = self._all_gather_counts(group=self.count_group, async_op=True) or _Done()
            return
        with torch.cuda.stream(self.count_stream):
            self.count_stream.wait_event(self.emitted)
            self.ops.rng_count(self.rank, self.world, self.counts.data_ptr(), stream=self.count_stream.cuda_stream)
            self.ahead = self._all_gather_counts(group=self.count_group, async_op=True)
        if self.ahead is None:  # completed on the side stream: order the next emit after it
            ev = torch.cuda.Event()
            ev.record(self.count_stream)
            self.ahead = _EventWork(ev)

    def drop_lookahead(self):
        """Complete and discard the next frame's counts (and emitted randDirs, restoring the stream state) -- call
        on every rank before anything else advances the renderer's random stream; the next step counts afresh."""
        if self.ahead is not None:
            self.ahead.wait()
        if self.count_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.count_stream)
        if self.emit_ready:
            self.ops.rng_discard()
            self.emit_ready = False
        self.ahead = None

    def _host_staged(self) -> bool:
        # gloo on device tensors (a multi-rank rehearsal on one GPU): stage the collectives through host memory
        return self.device.type == "cuda" and dist.get_backend() != "nccl"

    def _all_gather_counts(self, group=None, async_op: bool = False, bps: Optional[int] = None):
        """All-gather the ranks' slices of bps blocks (default self.bps) in the first world * bps words of counts."""
        bps = bps or self.bps
        counts = self.counts[:self.world * bps]
        mine = counts[self.rank * bps:(self.rank + 1) * bps]
        if dist.get_backend() == "nccl":
            return dist.all_gather_into_tensor(counts, mine.clone(), group=group, async_op=async_op)
        if self._host_staged():
            # gloo ranks on one GPU: through host memory on the current stream (the side stream of a look-ahead:
            # .cpu() waits for the count there, the copy back is ordered before the emit); completes here
            h = counts.cpu()
            dist.all_gather(list(h.split(bps)), h[self.rank * bps:(self.rank + 1) * bps].clone(), group=group)
            counts.copy_(h, non_blocking=False)
            return None
        if async_op:  # gloo on CPU (the orchestration tests): the exchange completes here
            dist.all_gather(list(counts.split(bps)), mine.clone(), group=group)
            return None
        else:
            dist.all_gather(list(counts.split(bps)), mine.clone())


class StripFrame(_CountedFrame):
    """Rank `rank`'s part of a W x H frame rendered by `world` ranks; rank 0 ends with the ARGB8 frame and,
    with gather_rgb, the float RGB frame too (the reference's std::vector<Color> image, Render.h:10, that
    Render::imagePixel reads, Render.cpp:103-114).

    pipeline (default: on for the nccl backend): the strip gathers of frame i run on their own communicator
    (a second process group, so their RCCL stream does not serialise with the next frame's count
    all-gather) while frame i+1 renders; strip and gather buffers are double-buffered, and rank 0
    un-interleaves on a side stream.  A frame's assembled image is complete once the device is
    synchronised (every step's work, gathers included, is on the device's streams).  count_ahead: see
    _CountedFrame.
    """

    def __init__(self, ops, W: int, H: int, row_block: int, rank: int, world: int, device: torch.device,
                 gather_to_root: bool = True, pipeline: Optional[bool] = None, gather_rgb: bool = False,
                 count_ahead: Optional[bool] = None, emit_ahead: Optional[bool] = None):
        self.W, self.H, self.rb = W, H, row_block
        self._init_counts(ops, rank, world, device, count_ahead, emit_ahead)
        self.gather_to_root = gather_to_root
        self.gather_rgb = bool(gather_rgb) and gather_to_root and world > 1
        self.rows = strip_rows(H, row_block, rank, world)
        self.max_rows = max(strip_rows(H, row_block, r, world) for r in range(world))
        if pipeline is None:
            pipeline = world > 1 and gather_to_root and dist.get_backend() == "nccl"
        self.pipeline = bool(pipeline) and world > 1 and gather_to_root and not self._host_staged()
        nbuf = 2 if self.pipeline else 1
        # per-rank strip buffers (every rank the same size for the gather): ARGB8, float RGB
        self.argb_bufs = [torch.zeros(self.max_rows * W, dtype=torch.int32, device=device) for _ in range(nbuf)]
        self.img_bufs = [torch.zeros(max(self.max_rows, 1) * W * 3, dtype=torch.float32, device=device)
                         for _ in range(nbuf if self.gather_rgb else 1)]
        self.argb, self.img = self.argb_bufs[0], self.img_bufs[0]
        # what rank 0 gathers: (strip buffers, values per frame row, dtype)
        self.planes = [(self.argb_bufs, W, torch.int32)]
        if self.gather_rgb:
            self.planes.append((self.img_bufs, 3 * W, torch.float32))
        self.fulls: List[List[torch.Tensor]] = []         # [plane][k]: H x per_row frame on rank 0
        self.gather_lists: List[List[List[torch.Tensor]]] = []  # [plane][k][rank]
        self.row_index: List[torch.Tensor] = []
        if gather_to_root and rank == 0:
            for bufs, per_row, dt in self.planes:
                self.fulls.append([torch.zeros(H * per_row, dtype=dt, device=device) for _ in range(nbuf)])
                self.gather_lists.append([[torch.empty_like(bufs[0]) for _ in range(world)] for _ in range(nbuf)])
            for r in range(world):
                n = strip_rows(H, row_block, r, world)
                self.row_index.append(torch.tensor([strip_row_to_y(i, row_block, r, world) for i in range(n)],
                                                   dtype=torch.int64, device=device))
        self.full: Optional[torch.Tensor] = self.fulls[0][0] if self.fulls else None
        self.rgb_full: Optional[torch.Tensor] = self.fulls[1][0] if self.gather_rgb and self.fulls else None
        self.group = dist.new_group(list(range(world))) if self.pipeline else None
        cuda = device.type == "cuda"
        self.side = torch.cuda.Stream(device=device) if self.pipeline and cuda and rank == 0 else None
        self.works: List[list] = [[] for _ in range(nbuf)]
        self.done: List[Optional[torch.cuda.Event]] = [None] * nbuf
        self.frame = 0

    def _gather_strips(self, k: int):
        for pi, (bufs, _, _) in enumerate(self.planes):
            lst = self.gather_lists[pi][k] if self.rank == 0 else None
            if not self._host_staged():
                dist.gather(bufs[k], lst, dst=0)
                continue
            hl = [torch.empty(bufs[k].shape, dtype=bufs[k].dtype) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(bufs[k].cpu(), hl, dst=0)
            if self.rank == 0:
                for d, h in zip(lst, hl):
                    d.copy_(h)

    def _assemble(self, k: int) -> torch.Tensor:
        out = []
        for pi, (_, per_row, _) in enumerate(self.planes):
            fv = self.fulls[pi][k].view(self.H, per_row)
            for r in range(self.world):
                n = self.row_index[r].numel()
                if n:
                    fv.index_copy_(0, self.row_index[r], self.gather_lists[pi][k][r][: n * per_row].view(n, per_row))
            out.append(fv)
        self.full = out[0]
        if self.gather_rgb:
            self.rgb_full = out[1].view(self.H, self.W, 3)
        return out[0]

    def step(self, d_counters: int = 0) -> Optional[torch.Tensor]:
        """Render this rank's strips of one frame; rank 0 returns the (H, W) int32 ARGB frame (with
        pipeline: complete once the device is synchronised; with gather_rgb also in self.rgb_full)."""
        k = self.frame % len(self.argb_bufs)
        self.frame += 1
        cuda = self.device.type == "cuda"
        if self.pipeline:
            # buffer set k was last used two frames ago: its gathers and (rank 0) un-interleave must be done
            for w in self.works[k]:
                w.wait()
            self.works[k] = []
            if cuda and self.done[k] is not None:
                torch.cuda.current_stream(self.device).wait_event(self.done[k])
        argb = self.argb_bufs[k]
        img = self.img_bufs[k % len(self.img_bufs)]
        self.argb, self.img = argb, img
        self._frame_counts()
        self._render(img, argb, d_counters)
        if self.world == 1 or not self.gather_to_root:
            return argb[: self.rows * self.W].view(self.rows, self.W) if self.world == 1 else None
        if not self.pipeline:
            self._gather_strips(k)
            return self._assemble(k) if self.rank == 0 else None
        for pi, (bufs, _, _) in enumerate(self.planes):
            self.works[k].append(dist.gather(bufs[k], self.gather_lists[pi][k] if self.rank == 0 else None, dst=0,
                                             group=self.group, async_op=True))
        if self.rank != 0:
            return None
        if not cuda:
            for w in self.works[k]:
                w.wait()
            self.works[k] = []
            return self._assemble(k)
        with torch.cuda.stream(self.side):
            for w in self.works[k]:
                w.wait()  # the side stream waits for the gathers
            fv = self._assemble(k)
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.done[k] = ev
        return fv


def equal_bounds(H: int, world: int, grain: int = 8) -> List[int]:
    """Band bounds (world + 1 rows, 0 .. H) of about H / world rows each, on multiples of `grain`."""
    b = [0] + [min(H, max(0, int(round(H * r / world / grain)) * grain)) for r in range(1, world)] + [H]
    return _fix_bounds(b, H, grain)


def _fix_bounds(b: List[int], H: int, grain: int) -> List[int]:
    """Strictly increasing bounds, each band at least `grain` rows where the frame allows it."""
    world = len(b) - 1
    g = grain if H >= grain * world else 1
    out = [0]
    for r in range(1, world):
        out.append(min(max(b[r], out[-1] + g), H - g * (world - r)))
    out.append(H)
    return out


def balanced_bounds(bounds: List[int], times: List[float], H: int, grain: int = 8) -> List[int]:
    """New band bounds from each band's measured time per frame: the cost density of band r (time / rows) is taken
    as uniform over its rows, and the frame's cumulative cost is cut into `world` equal parts on multiples of
    `grain`.  Deterministic in its inputs, so ranks that all-gathered the same times agree on the result."""
    world = len(bounds) - 1
    rows = [bounds[r + 1] - bounds[r] for r in range(world)]
    known = [t / n for t, n in zip(times, rows) if n > 0 and t > 0]
    mean = sum(known) / len(known) if known else 1.0
    dens = [(t / n if n > 0 and t > 0 else mean) for t, n in zip(times, rows)]
    total = sum(d * n for d, n in zip(dens, rows))
    out = [0]
    r, acc = 0, 0.0  # acc: cost of the rows before band r's start
    for k in range(1, world):
        target = total * k / world
        while r < world - 1 and acc + dens[r] * rows[r] < target:
            acc += dens[r] * rows[r]
            r += 1
        y = bounds[r] + (target - acc) / dens[r]
        out.append(int(round(y / grain)) * grain)
    out.append(H)
    return _fix_bounds(out, H, grain)


LAUNCH_TRACES = 1 << 30  # rfx_host.cpp RFX_LAUNCH_TRACES: the library's default launch limit
MAX_PASS_TRACES = 1 << 31  # rfx_host.cpp kMaxLaunchTraces: a band's span (its scan offsets are 32-bit)


def pass_plan(W: int, H: int, ss: int, world: int, launch_traces: int = LAUNCH_TRACES) -> Optional[List[tuple]]:
    """The row spans [y0, y1) a band frame of W x H pixels at ss x ss samples runs as, or None when one pass over the
    whole frame takes it: at most min(world x launch_traces, 2^31) traces per pass (rfx_group.cpp does the same)."""
    spp = max(1, ss) ** 2
    cap = min(world * launch_traces, MAX_PASS_TRACES)
    if W * H * spp <= cap:
        return None
    per = cap // (W * spp)  # rows per pass
    if per == 0:
        raise ValueError(f"one row of {W} x {spp} samples exceeds {cap} traces")
    return [(y, min(H, y + per)) for y in range(0, H, per)]


def pass_bands(y0: int, y1: int, world: int) -> List[int]:
    """Equal bands of the span [y0, y1) for ranks 0 .. m - 1, m = min(world, rows): m + 1 bounds."""
    m = min(world, y1 - y0)
    return [y0 + ((y1 - y0) * i) // m for i in range(m + 1)]


def pass_rows(bd: List[int], rank: int, y1: Optional[int]):
    """Rank `rank`'s rows of a pass with bands bd; a rank without a band gets the span's last row when y1 is given (its
    count of the span's stream needs a valid band frame; it traces nothing), else the empty range."""
    if rank < len(bd) - 1:
        return bd[rank], bd[rank + 1]
    return (y1 - 1, y1) if y1 is not None else (0, 0)


class BandFrame(_CountedFrame):
    """Rank `rank`'s band of a W x H frame rendered by `world` ranks: contiguous rows [bounds[rank],
    bounds[rank + 1]), traced into whole-frame buffers (rfx.h band partition), so that rank 0 receives every band
    straight into its rows of the frame -- its own band is rendered there in place -- with no strip
    un-interleave: rank 0's work beyond the other ranks' is the RCCL receive alone.  Bands are load-balanced from
    measured per-rank frame times (balance(): a few rounds before timing starts), which also shrinks rank 0's
    band by what the receive costs it.  Rank 0 ends with the ARGB8 frame (and with gather_rgb the float RGB frame,
    the reference's image that Render::imagePixel reads, Render.cpp:103-114).

    pipeline (default: on for the nccl backend): frame i's band sends / receives run on their own communicator
    while frame i + 1 renders into the other of two buffer sets.  count_ahead: see _CountedFrame.
    """

    def __init__(self, ops, W: int, H: int, rank: int, world: int, device: torch.device, gather_to_root: bool = True,
                 pipeline: Optional[bool] = None, gather_rgb: bool = False, count_ahead: Optional[bool] = None,
                 bounds: Optional[List[int]] = None, grain: int = 8, emit_ahead: Optional[bool] = None, ss: int = 1,
                 launch_traces: int = LAUNCH_TRACES):
        self.W, self.H, self.grain = W, H, grain
        # a frame of more traces than one pass takes (world x launch_traces, and at most 2^31 for the band scan's
        # offsets: SSAA screenshots reach 2.2e12) runs as passes over row spans (pass_plan)
        self.passes = pass_plan(W, H, ss, world, launch_traces)
        if self.passes:
            count_ahead = emit_ahead = False  # one pass's count exchange is negligible beside its trace
            y0, y1 = self.passes[0]          # the largest pass: the count buffer is sized for it
            ops.set_span(y0, y1)
            bd = pass_bands(y0, y1, world)
            ops.set_rows(*pass_rows(bd, rank, y1))
        else:
            b0 = bounds or equal_bounds(H, world, grain)
            ops.set_rows(b0[rank], b0[rank + 1])  # a band frame from here on (the RNG layout below reads it)
        self._init_counts(ops, rank, world, device, count_ahead, emit_ahead)
        self.gather_to_root = gather_to_root and world > 1
        self.gather_rgb = bool(gather_rgb) and self.gather_to_root
        if pipeline is None:
            pipeline = world > 1 and gather_to_root and dist.get_backend() == "nccl"
        self.pipeline = bool(pipeline) and self.gather_to_root and not self._host_staged()
        nbuf = 2 if self.pipeline else 1
        # whole-frame buffers: ARGB8 and float RGB (rank 0's are the assembled frames)
        self.argb_bufs = [torch.zeros(H * W, dtype=torch.int32, device=device) for _ in range(nbuf)]
        self.img_bufs = [torch.zeros(H * W * 3, dtype=torch.float32, device=device)
                         for _ in range(nbuf if self.gather_rgb else 1)]
        self.argb, self.img = self.argb_bufs[0], self.img_bufs[0]
        self.group = dist.new_group(list(range(world))) if self.pipeline else None
        self.works: List[list] = [[] for _ in range(nbuf)]
        self.frame = 0
        self._events: Optional[list] = None  # (start, end) HIP events around each frame's render while balancing
        if self.passes:
            self.bounds = equal_bounds(H, world, grain) if H >= world else list(range(world)) + [H]
            self.y0, self.y1 = self.bounds[rank], self.bounds[rank + 1]
            self.rows = sum(max(0, b[1] - b[0]) for b in (pass_rows(pass_bands(a, e, world), rank, None)
                                                           for a, e in self.passes))
        else:
            self.set_bounds(b0)
        self.full: Optional[torch.Tensor] = self.argb.view(H, W) if rank == 0 else None
        self.rgb_full: Optional[torch.Tensor] = self.img.view(H, W, 3) if rank == 0 and self.gather_rgb else None

    def set_bounds(self, bounds: List[int]):
        """Band bounds for the next frames (the same list on every rank)."""
        if self.passes:
            raise ValueError("BandFrame: a frame rendered in row-span passes takes equal bands per pass")
        assert len(bounds) == self.world + 1 and bounds[0] == 0 and bounds[-1] == self.H, bounds
        assert all(bounds[r] < bounds[r + 1] for r in range(self.world)), bounds
        if getattr(self, "emit_ready", False) and list(bounds) != self.bounds:
            self.drop_lookahead()  # the frame emitted ahead holds the old band's randDirs only
        self.bounds = list(bounds)
        self.y0, self.y1 = bounds[self.rank], bounds[self.rank + 1]
        self.rows = self.y1 - self.y0
        self.ops.set_rows(self.y0, self.y1)

    def set_gather_rgb(self, on: bool):
        """Send the f32 RGB plane to rank 0 as well (on) or the ARGB8 plane only (off) from the next frame on; waits
        for the transfers in flight (bench.py times the bands both ways).  Every rank must call it alike."""
        on = bool(on) and self.gather_to_root
        if on == self.gather_rgb:
            return
        for ws in self.works:
            for w in ws:
                w.wait()
        self.works = [[] for _ in self.works]
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        nbuf = len(self.argb_bufs)
        if on and len(self.img_bufs) < nbuf:
            self.img_bufs += [torch.zeros_like(self.img_bufs[0]) for _ in range(nbuf - len(self.img_bufs))]
        self.gather_rgb = on
        if not on:
            self.rgb_full = None

    def _sends(self, k: int, bounds: Optional[List[int]] = None):
        """(tensor, peer, is_send) of frame buffer set k: every band to rank 0 (bounds: the bands of ranks
        0 .. len(bounds) - 2, default the frame's; ranks beyond them send nothing)."""
        W, ops = self.W, []
        bounds = self.bounds if bounds is None else bounds
        n = len(bounds) - 1
        planes = [(self.argb_bufs[k], 1)]
        if self.gather_rgb:
            planes.append((self.img_bufs[k], 3))
        for buf, per in planes:
            if self.rank == 0:
                for r in range(1, n):
                    ops.append((buf[bounds[r] * W * per:bounds[r + 1] * W * per], r, False))
            elif self.rank < n:
                ops.append((buf[bounds[self.rank] * W * per:bounds[self.rank + 1] * W * per], 0, True))
        return ops

    def _exchange(self, k: int, bounds: Optional[List[int]] = None):
        todo = self._sends(k, bounds)
        if self._host_staged():  # gloo on device tensors (one-GPU rehearsal): through host memory, in order
            for t, peer, send in todo:
                if send:
                    dist.send(t.cpu(), peer)
                else:
                    h = torch.empty(t.shape, dtype=t.dtype)
                    dist.recv(h, peer)
                    t.copy_(h)
            return []
        if dist.get_backend() == "nccl":
            p2p = [dist.P2POp(dist.isend if send else dist.irecv, t, peer, group=self.group) for t, peer, send in todo]
            return dist.batch_isend_irecv(p2p) if p2p else []
        return [dist.isend(t, peer, group=self.group) if send else dist.irecv(t, peer, group=self.group)
                for t, peer, send in todo]

    def step(self, d_counters: int = 0) -> Optional[torch.Tensor]:
        """Render this rank's band of one frame; rank 0 returns the (H, W) int32 ARGB frame (with pipeline:
        complete once the device is synchronised; with gather_rgb also in self.rgb_full)."""
        k = self.frame % len(self.argb_bufs)
        self.frame += 1
        for w in self.works[k]:  # buffer set k's sends / receives of two frames ago
            w.wait()
        self.works[k] = []
        argb = self.argb_bufs[k]
        img = self.img_bufs[k % len(self.img_bufs)]
        self.argb, self.img = argb, img
        if self.passes:
            return self._step_passes(k, img, argb, d_counters)
        self._frame_counts()
        ev = None
        if self._events is not None:
            ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
            self._events.append(ev)
        self._render(img, argb, d_counters, ev)
        if self.world == 1 or not self.gather_to_root:
            return argb.view(self.H, self.W) if self.world == 1 else None
        works = self._exchange(k)
        if self.pipeline and self.device.type == "cuda":
            self.works[k] = works
        else:
            for w in works:
                w.wait()
        if self.rank != 0:
            return None
        self.full = argb.view(self.H, self.W)
        if self.gather_rgb:
            self.rgb_full = img.view(self.H, self.W, 3)
        return self.full

    def _step_passes(self, k: int, img: torch.Tensor, argb: torch.Tensor, d_counters: int) -> Optional[torch.Tensor]:
        """One frame as passes over row spans (Render.cpp:136-215's cursor walks the same rows in order).  Per pass:
        the span's rows are cut into equal bands of ranks 0 .. m - 1 (m = min(world, rows)); every rank counts its
        1/world slice of the span's random stream and the counts are all-gathered; ranks with a band emit its
        randDirs and trace it (the stream continues from pass to pass on every rank); the bands go to rank 0.  A pass
        of fewer rows than ranks leaves ranks m .. world - 1 behind rank 0's stream: rank 0's state is broadcast to
        them before the next pass counts."""
        for y0, y1 in self.passes:
            bd = pass_bands(y0, y1, self.world)
            m = len(bd) - 1
            self.ops.set_span(y0, y1)
            self.ops.set_rows(*pass_rows(bd, self.rank, y1))
            bps = self.ops.blocks_per_slice(self.world)
            self.ops.rng_count(self.rank, self.world, self.counts.data_ptr())
            if self.world > 1:
                self._all_gather_counts(bps=bps)
            if self.rank < m:
                self.ops.render_counted(self.world, self.counts.data_ptr(), img.data_ptr(), argb.data_ptr(),
                                        d_counters)
            if m < self.world:
                self._hand_over_rng_state()
            if self.gather_to_root:
                works = self._exchange(k, bd)
                if self.pipeline and self.device.type == "cuda":
                    self.works[k] += works
                else:
                    for w in works:
                        w.wait()
        if self.world == 1 or not self.gather_to_root:
            return argb.view(self.H, self.W) if self.world == 1 else None
        if self.rank != 0:
            return None
        self.full = argb.view(self.H, self.W)
        if self.gather_rgb:
            self.rgb_full = img.view(self.H, self.W, 3)
        return self.full

    def _hand_over_rng_state(self):
        """Rank 0's random-stream states to every rank (the ranks that sat a pass out are behind it)."""
        st = torch.tensor(list(self.ops.rng_state()) if self.rank == 0 else [0, 0], dtype=torch.int64)
        if dist.get_backend() == "nccl":
            st = st.to(self.device)
        dist.broadcast(st, 0)
        sphere, jitter = (int(v) for v in st.tolist())
        if self.rank != 0:
            self.ops.set_rng_state(sphere, jitter)

    def balance(self, rounds: int = 3, frames: int = 8, timer=None) -> List[int]:
        """Re-cut the bands `rounds` times from each rank's measured render time over `frames` frames (HIP events
        on the render stream, or `timer(step)` -> seconds per frame); returns the final bounds."""
        if self.passes:
            return self.bounds  # equal bands per pass: nothing to balance
        for _ in range(rounds):
            t = timer(self.step) if timer else self._time_render(frames)
            times = torch.tensor([t], dtype=torch.float64)
            if dist.get_backend() == "nccl":
                times = times.to(self.device)
            allt = [torch.zeros_like(times) for _ in range(self.world)]
            dist.all_gather(allt, times)
            self.set_bounds(balanced_bounds(self.bounds, [float(x.item()) for x in allt], self.H, self.grain))
        return self.bounds

    def _time_render(self, frames: int) -> float:
        """Seconds per frame of this rank's emit + trace: HIP events around the render on its stream (after the
        wait for the counts, so other ranks' progress is not counted; what concurrent sends / receives take from
        the render on this device is)."""
        self._events = []
        for _ in range(frames):
            self.step()
        torch.cuda.synchronize(self.device)
        ev, self._events = self._events, None
        return sum(s.elapsed_time(e) for s, e in ev) * 1e-3 / max(len(ev), 1)
