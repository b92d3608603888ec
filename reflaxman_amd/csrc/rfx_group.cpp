// Multi-GPU frames from one process (include/rfx.h rfx_group_*): the frame of Render::renderNext
// (Render.cpp:136-215) cut into row bands, one per device of the group, for C/C++ callers that have no
// torch.distributed -- the drop-in Render (include/reflaxman/dropin/Render.h) among them.
//
// Per frame, on each member's stream:
//   1. the member's random stream is set to member 0's (the caller may have rendered on member 0 alone);
//   2. the member counts the accepted LCG triples of its 1/n slice of the frame's random stream and pushes its
//      slice of counts to every other member (hipMemcpyPeerAsync over xGMI): the one exchange step of the
//      partitioned pre-pass, n x ~1K words;
//   3. once every slice has arrived, it emits the randDirs of its band and traces the band
//      (rfx_render_frame_counted_ev with the band partition of rfx_frame);
//   4. members 1..n-1 copy their band rows into the caller's frame on member 0's device (peer copies), and the
//      caller's stream waits for them.
// The bands start equal (multiples of 8 rows) and are re-cut from the measured per-member trace times every
// kBalanceEvery frames (the frame's cumulative cost cut into n equal parts, as reflaxman_amd/dist.py
// balanced_bounds), reading only events that have already completed: no frame waits for a measurement.
// The assembled frame equals the single-GPU frame bit for bit (tests/test_gpu_group.py).
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "rfx_internal.h"

namespace {
constexpr int kBalanceEvery = 8;
constexpr uint32_t kGrain = 8;

int hip_fail(hipError_t e, const char *what)
{
  return rfx_detail_fail(RFX_ERR_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}
#define GCHECK(expr)                                  \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)
#define RCHECK(expr)             \
  do {                           \
    int rc_ = (expr);            \
    if (rc_ != RFX_OK) return rc_; \
  } while (0)

// strictly increasing bounds, each band at least `grain` rows where the frame allows it (dist.py _fix_bounds)
std::vector<uint32_t> fix_bounds(std::vector<double> b, uint32_t H, uint32_t grain)
{
  const size_t n = b.size() - 1;
  const uint32_t g = H >= grain * n ? grain : 1;
  std::vector<uint32_t> out(n + 1);
  out[0] = 0;
  for (size_t r = 1; r < n; ++r)
  {
    double y = std::max(b[r], (double)out[r - 1] + g);
    y = std::min(y, (double)H - (double)g * (n - r));
    out[r] = (uint32_t)y;
  }
  out[n] = H;
  return out;
}

std::vector<uint32_t> equal_bounds(uint32_t H, size_t n)
{
  std::vector<double> b(n + 1);
  for (size_t r = 0; r <= n; ++r) b[r] = r == n ? H : std::round((double)H * r / n / kGrain) * kGrain;
  return fix_bounds(b, H, kGrain);
}

// cut the frame's cumulative cost (band r's density time / rows, uniform over its rows) into n equal parts
std::vector<uint32_t> balanced_bounds(const std::vector<uint32_t> &bounds, const std::vector<double> &t, uint32_t H)
{
  const size_t n = bounds.size() - 1;
  std::vector<double> rows(n), dens(n);
  double known = 0.0;
  int nk = 0;
  for (size_t r = 0; r < n; ++r)
  {
    rows[r] = bounds[r + 1] - bounds[r];
    if (rows[r] > 0 && t[r] > 0) { known += t[r] / rows[r]; ++nk; }
  }
  const double mean = nk ? known / nk : 1.0;
  double total = 0.0;
  for (size_t r = 0; r < n; ++r)
  {
    dens[r] = rows[r] > 0 && t[r] > 0 ? t[r] / rows[r] : mean;
    total += dens[r] * rows[r];
  }
  std::vector<double> out(n + 1);
  out[0] = 0;
  size_t r = 0;
  double acc = 0.0;
  for (size_t k = 1; k < n; ++k)
  {
    const double target = total * k / n;
    while (r < n - 1 && acc + dens[r] * rows[r] < target) { acc += dens[r] * rows[r]; ++r; }
    out[k] = std::round((bounds[r] + (target - acc) / dens[r]) / kGrain) * kGrain;
  }
  out[n] = H;
  return fix_bounds(out, H, kGrain);
}
}  // namespace

struct rfx_group {
  std::vector<int> dev;
  std::vector<rfx_renderer *> r;
  std::vector<hipStream_t> own;                  // per member: the stream its counts, emits and traces run on
  std::vector<hipStream_t> cp;                   // per member: the stream its band copies to the caller's frame run on
  std::vector<uint32_t *> cnt[2];                // per member: n x bps count words, double-buffered by frame parity
  uint64_t cnt_words = 0, bps = 0;
  std::vector<float *> rgb[2];                   // per member: whole-frame scratch (its band rows written), double-
  std::vector<uint32_t *> argb[2];               // buffered by pass parity: pass k traces while pass k - 1's copy runs
  size_t px_cap = 0;
  float *rgb0 = nullptr;                         // a one-member frame's floats when the caller wants ARGB8 only
  size_t rgb0_cap = 0;
  std::vector<hipEvent_t> ev_start, ev_cnt, ev_emit[2], ev_t1, ev_copied[2];
  std::vector<uint64_t> seq;                     // members' random-stream state counters after the group's last pass
  bool seq_ok = false;
  std::vector<uint32_t> bounds;
  bool fixed = false;
  uint32_t W = 0, H = 0;
  uint64_t frames = 0;
  std::vector<double> acc;                       // balancing: summed trace ms per member
  int acc_frames = 0;
  bool timing_pending = false;
  int timing_parity = 0;
  size_t n() const { return r.size(); }
};

static void destroy(rfx_group *g)
{
  for (size_t i = 0; i < g->dev.size(); ++i)
  {
    (void)hipSetDevice(g->dev[i]);
    if (i < g->own.size() && g->own[i]) (void)hipStreamSynchronize(g->own[i]);
    if (i < g->cp.size() && g->cp[i]) (void)hipStreamSynchronize(g->cp[i]);
  }
  for (size_t i = 0; i < g->dev.size(); ++i)
  {
    (void)hipSetDevice(g->dev[i]);
    for (int b = 0; b < 2; ++b)
    {
      if (i < g->cnt[b].size()) (void)hipFree(g->cnt[b][i]);
      if (i < g->rgb[b].size()) (void)hipFree(g->rgb[b][i]);
      if (i < g->argb[b].size()) (void)hipFree(g->argb[b][i]);
    }
    for (std::vector<hipEvent_t> *v : {&g->ev_start, &g->ev_cnt, &g->ev_emit[0], &g->ev_emit[1], &g->ev_t1,
                                       &g->ev_copied[0], &g->ev_copied[1]})
      if (i < v->size() && (*v)[i]) (void)hipEventDestroy((*v)[i]);
    if (i < g->own.size() && g->own[i]) (void)hipStreamDestroy(g->own[i]);
    if (i < g->cp.size() && g->cp[i]) (void)hipStreamDestroy(g->cp[i]);
  }
  if (g->rgb0)
  {
    (void)hipSetDevice(g->dev[0]);
    (void)hipFree(g->rgb0);
  }
  for (rfx_renderer *r : g->r) rfx_renderer_destroy(r);
  delete g;
}

extern "C" void rfx_group_destroy(rfx_group *g)
{
  if (g) destroy(g);
}

static int create(rfx_group *g, const int *devices, int n)
{
  for (int i = 0; i < n; ++i)
  {
    rfx_renderer *r = nullptr;
    RCHECK(rfx_renderer_create(&r, devices[i]));
    g->r.push_back(r);
    g->dev.push_back(devices[i]);
  }
  // peer access between distinct devices (band and count copies over xGMI)
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
    {
      if (g->dev[i] == g->dev[j]) continue;
      int can = 0;
      GCHECK(hipDeviceCanAccessPeer(&can, g->dev[i], g->dev[j]));
      if (!can) continue;  // hipMemcpyPeerAsync still works, staged by the runtime
      GCHECK(hipSetDevice(g->dev[i]));
      const hipError_t e = hipDeviceEnablePeerAccess(g->dev[j], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hip_fail(e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();
    }
  for (int i = 0; i < n; ++i)
  {
    GCHECK(hipSetDevice(g->dev[i]));
    hipStream_t s = nullptr, c = nullptr;
    GCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g->own.push_back(s);
    GCHECK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    g->cp.push_back(c);
    hipEvent_t e[7];
    for (hipEvent_t &x : e) GCHECK(hipEventCreate(&x));
    g->ev_start.push_back(e[0]);
    g->ev_cnt.push_back(e[1]);
    g->ev_emit[0].push_back(e[2]);
    g->ev_emit[1].push_back(e[3]);
    g->ev_t1.push_back(e[4]);
    g->ev_copied[0].push_back(e[5]);
    g->ev_copied[1].push_back(e[6]);
    // the double-buffer waits of the first two passes find recorded events
    for (int k = 2; k < 7; ++k)
      if (k != 4) GCHECK(hipEventRecord(e[k], s));
    for (int b = 0; b < 2; ++b)
    {
      g->cnt[b].push_back(nullptr);
      g->rgb[b].push_back(nullptr);
      g->argb[b].push_back(nullptr);
    }
  }
  g->acc.assign(n, 0.0);
  g->seq.assign(n, 0);
  return RFX_OK;
}

extern "C" int rfx_group_create(rfx_group **out, const int *devices, int n)
{
  if (!out || !devices || n <= 0 || n > 64) return rfx_detail_fail(RFX_ERR_ARG, "group_create: 1..64 devices");
  *out = nullptr;
  rfx_group *g = new rfx_group();
  const int rc = create(g, devices, n);
  if (rc != RFX_OK)
  {
    destroy(g);
    return rc;
  }
  *out = g;
  return RFX_OK;
}

extern "C" int rfx_group_size(const rfx_group *g) { return g ? (int)g->n() : 0; }

extern "C" rfx_renderer *rfx_group_renderer(rfx_group *g, int i)
{
  return g && i >= 0 && (size_t)i < g->n() ? g->r[i] : nullptr;
}

extern "C" int rfx_group_set_scene(rfx_group *g, const rfx_scene *s)
{
  if (!g || !s) return rfx_detail_fail(RFX_ERR_ARG, "group_set_scene: bad args");
  for (rfx_renderer *r : g->r) RCHECK(rfx_renderer_set_scene(r, s));
  return RFX_OK;
}

extern "C" int rfx_group_set_bands(rfx_group *g, uint32_t height, const uint32_t *bounds)
{
  if (!g) return rfx_detail_fail(RFX_ERR_ARG, "group_set_bands: null group");
  if (!bounds)
  {
    g->fixed = false;
    g->bounds.clear();
    return RFX_OK;
  }
  const size_t n = g->n();
  if (bounds[0] != 0 || bounds[n] != height) return rfx_detail_fail(RFX_ERR_ARG, "group_set_bands: 0 .. height");
  for (size_t i = 0; i < n; ++i)
    if (bounds[i] >= bounds[i + 1]) return rfx_detail_fail(RFX_ERR_ARG, "group_set_bands: bands must be non-empty");
  g->bounds.assign(bounds, bounds + n + 1);
  g->fixed = true;
  g->H = height;
  return RFX_OK;
}

extern "C" int rfx_group_get_bands(const rfx_group *g, uint32_t *bounds)
{
  if (!g || !bounds) return rfx_detail_fail(RFX_ERR_ARG, "group_get_bands: bad args");
  if (g->bounds.empty()) return rfx_detail_fail(RFX_ERR_STATE, "group_get_bands: no frame rendered yet");
  std::copy(g->bounds.begin(), g->bounds.end(), bounds);
  return RFX_OK;
}

// the last frame's per-member trace times, once all are complete (never waits): every kBalanceEvery frames re-cut
static int collect_times(rfx_group *g)
{
  if (!g->timing_pending || g->fixed) return RFX_OK;
  const size_t n = g->n();
  for (size_t i = 0; i < n; ++i)
  {
    GCHECK(hipSetDevice(g->dev[i]));
    if (hipEventQuery(g->ev_t1[i]) != hipSuccess) return RFX_OK;  // not yet: try after the next frame
  }
  g->timing_pending = false;
  for (size_t i = 0; i < n; ++i)
  {
    float ms = 0.0f;
    GCHECK(hipSetDevice(g->dev[i]));
    GCHECK(hipEventElapsedTime(&ms, g->ev_emit[g->timing_parity][i], g->ev_t1[i]));
    g->acc[i] += ms;
  }
  if (++g->acc_frames >= kBalanceEvery)
  {
    g->bounds = balanced_bounds(g->bounds, g->acc, g->H);
    g->acc.assign(n, 0.0);
    g->acc_frames = 0;
  }
  return RFX_OK;
}

static int ensure_buffers(rfx_group *g, const rfx_frame &f0, size_t m)
{
  const size_t n = g->n();
  uint64_t bps = 0;
  RCHECK(rfx_frame_rng_blocks(g->r[0], &f0, (uint32_t)m, &bps));
  g->bps = bps;
  if (bps * m > g->cnt_words)
  {
    for (size_t i = 0; i < n; ++i)
    {
      GCHECK(hipSetDevice(g->dev[i]));
      GCHECK(hipDeviceSynchronize());  // frames still in flight read the old arrays
      for (int b = 0; b < 2; ++b)
      {
        (void)hipFree(g->cnt[b][i]);
        g->cnt[b][i] = nullptr;
        GCHECK(hipMalloc(&g->cnt[b][i], bps * m * sizeof(uint32_t)));
      }
    }
    g->cnt_words = bps * m;
  }
  const size_t px = (size_t)f0.width * f0.height;
  if (px > g->px_cap)
  {
    for (size_t i = 0; i < n; ++i)
    {
      GCHECK(hipSetDevice(g->dev[i]));
      GCHECK(hipDeviceSynchronize());  // traces and copies still in flight use the old scratch
      for (int b = 0; b < 2; ++b)
      {
        (void)hipFree(g->rgb[b][i]); (void)hipFree(g->argb[b][i]);
        g->rgb[b][i] = nullptr; g->argb[b][i] = nullptr;
        GCHECK(hipMalloc(&g->rgb[b][i], px * 3 * sizeof(float)));
        GCHECK(hipMalloc(&g->argb[b][i], px * sizeof(uint32_t)));
      }
    }
    g->px_cap = px;
  }
  return RFX_OK;
}

// One pass of the group over the rows [y0, y1) of the frame: members 0..m-1 take the bands bd[i] .. bd[i + 1] (whole rows
// within [y0, y1)), the random stream runs over the pass's rows (rfx_frame span_begin / span_end).  A frame is one pass
// over all rows, or -- 2^31 traces or more -- consecutive passes of row spans (the stream continues from pass to pass on
// every member, as Render.cpp:136-215's cursor does).
//
// Each member counts, emits and traces on its own stream into its own scratch frame (double-buffered by pass parity), and
// copies its band rows into the caller's frame on a copy stream: so member i's copy of pass k overlaps its trace of pass
// k + 1.  Only the copies wait for the caller's stream (its work before the call may still read or write the frame); the
// traces wait for it only when a member's random stream may differ from member 0's (a frame rendered on member 0 alone,
// a rewind, set_rng: the stream-state counters moved) or the frame accumulates onto the caller's pixels.
static int group_pass(rfx_group *g, const rfx_frame *f, uint32_t y0, uint32_t y1, const std::vector<uint32_t> &bd,
                      float *d_rgb, uint32_t *d_argb, hipStream_t s0)
{
  const size_t m = bd.size() - 1;
  const uint32_t W = f->width;
  std::vector<rfx_frame> fr(m, *f);
  for (size_t i = 0; i < m; ++i)
  {
    fr[i].row_block = 0;
    fr[i].rank = (uint32_t)i;
    fr[i].nranks = (uint32_t)m;
    fr[i].pixel_begin = (uint64_t)bd[i] * W;
    fr[i].pixel_end = (uint64_t)bd[i + 1] * W;
    fr[i].span_begin = (uint64_t)y0 * W;
    fr[i].span_end = (uint64_t)y1 * W;
  }
  RCHECK(ensure_buffers(g, fr[0], m));
  const int b = (int)(g->frames & 1);
  const bool accumulate = f->additive_counter > 1;
  const std::vector<hipStream_t> &st = g->own;
  // 0. the caller's work on its stream before this pass
  GCHECK(hipSetDevice(g->dev[0]));
  GCHECK(hipEventRecord(g->ev_start[0], s0));
  bool handoff = !g->seq_ok;
  for (size_t i = 0; i < g->n(); ++i) handoff = handoff || rfx_detail_state_seq(g->r[i]) != g->seq[i];
  const uint32_t jitter = rfx_detail_jitter(g->r[0]);
  for (size_t i = 0; i < m; ++i)
  {
    GCHECK(hipSetDevice(g->dev[i]));
    if (handoff || accumulate) GCHECK(hipStreamWaitEvent(st[i], g->ev_start[0], 0));
    // member 0's stream state is the group's: handed to the others when theirs may differ
    if (handoff && i)
      GCHECK(hipMemcpyPeerAsync(rfx_detail_seed_word(g->r[i]), g->dev[i], rfx_detail_seed_word(g->r[0]), g->dev[0],
                                sizeof(uint32_t), st[i]));
    rfx_detail_set_jitter(g->r[i], jitter);
    GCHECK(hipStreamWaitEvent(st[i], g->ev_copied[b][i], 0));  // the copy of two passes ago has read scratch b
  }
  // 1. each member counts its slice of the pass's random stream and pushes it to every other member
  const size_t sl = g->bps * sizeof(uint32_t);
  for (size_t i = 0; i < m; ++i)
  {
    RCHECK(rfx_frame_rng_count(g->r[i], &fr[i], (uint32_t)i, (uint32_t)m, g->cnt[b][i], st[i]));
    GCHECK(hipSetDevice(g->dev[i]));
    for (size_t j = 0; j < m; ++j)
    {
      if (j == i) continue;
      GCHECK(hipStreamWaitEvent(st[i], g->ev_emit[b][j], 0));  // j's emit of two passes ago read this array
      GCHECK(hipMemcpyPeerAsync(g->cnt[b][j] + i * g->bps, g->dev[j], g->cnt[b][i] + i * g->bps, g->dev[i], sl, st[i]));
    }
    GCHECK(hipEventRecord(g->ev_cnt[i], st[i]));
  }
  // 2. every slice arrived: emit the band's randDirs and trace the band into scratch; 3. the band rows to the caller's
  // frame on the member's copy stream
  for (size_t i = 0; i < m; ++i)
  {
    GCHECK(hipSetDevice(g->dev[i]));
    for (size_t j = 0; j < m; ++j)
      if (j != i) GCHECK(hipStreamWaitEvent(st[i], g->ev_cnt[j], 0));
    const uint64_t r0 = bd[i], rows = bd[i + 1] - r0;
    float *img = g->rgb[b][i];
    uint32_t *a = g->argb[b][i];
    if (accumulate)  // the accumulated rows this member adds to (Render.cpp:191-194)
      GCHECK(hipMemcpyPeerAsync(img + r0 * W * 3, g->dev[i], d_rgb + r0 * W * 3, g->dev[0], rows * W * 12, st[i]));
    const uint32_t j0 = rfx_detail_jitter(g->r[i]);
    RCHECK(rfx_render_frame_counted_ev(g->r[i], &fr[i], (uint32_t)m, g->cnt[b][i], img, d_argb ? a : nullptr, nullptr,
                                       st[i], g->ev_emit[b][i]));
    rfx_detail_set_rewindable(g->r[i], j0);
    GCHECK(hipSetDevice(g->dev[i]));
    GCHECK(hipEventRecord(g->ev_t1[i], st[i]));
    GCHECK(hipStreamWaitEvent(g->cp[i], g->ev_t1[i], 0));
    GCHECK(hipStreamWaitEvent(g->cp[i], g->ev_start[0], 0));  // the caller's frame is free to be written
    if (d_rgb)
      GCHECK(hipMemcpyPeerAsync(d_rgb + r0 * W * 3, g->dev[0], img + r0 * W * 3, g->dev[i], rows * W * 12, g->cp[i]));
    if (d_argb)
      GCHECK(hipMemcpyPeerAsync(d_argb + r0 * W, g->dev[0], a + r0 * W, g->dev[i], rows * W * 4, g->cp[i]));
    GCHECK(hipEventRecord(g->ev_copied[b][i], g->cp[i]));
  }
  GCHECK(hipSetDevice(g->dev[0]));
  for (size_t i = 0; i < m; ++i) GCHECK(hipStreamWaitEvent(s0, g->ev_copied[b][i], 0));
  ++g->frames;
  for (size_t i = 0; i < g->n(); ++i) g->seq[i] = rfx_detail_state_seq(g->r[i]);
  // members m..n-1 sat this pass out (a span of fewer rows than members): their streams stayed behind member 0's, so
  // the next pass hands member 0's state over again
  g->seq_ok = m == g->n();
  return RFX_OK;
}

extern "C" int rfx_group_render_frame(rfx_group *g, const rfx_frame *f, float *d_rgb, uint32_t *d_argb, void *stream)
{
  if (!g || !f || (!d_rgb && !d_argb)) return rfx_detail_fail(RFX_ERR_ARG, "group_render_frame: bad args");
  const size_t n = g->n();
  const uint32_t W = f->width, H = f->height;
  const uint64_t npx = (uint64_t)W * H;
  // ARGB8-only frames (a display that never reads the float image): only the 4-B/px plane crosses to member 0
  const bool argb_only = d_rgb == nullptr;
  if (argb_only && f->additive_counter > 1)
    return rfx_detail_fail(RFX_ERR_ARG, "group_render_frame: an accumulating frame needs the float frame (d_rgb)");
  if (f->sample_num <= 0 || f->sample_num > 256 || (f->nranks > 1) ||
      !((f->pixel_begin == 0 && f->pixel_end == 0) || (f->pixel_begin == 0 && f->pixel_end == npx)))
    return rfx_detail_fail(RFX_ERR_ARG, "group_render_frame: a whole frame with sample_num > 0 (no partition fields)");
  hipStream_t s0 = stream ? (hipStream_t)stream : rfx_detail_stream(g->r[0]);
  if (n == 1 || H < n)  // one member renders the frame (and splits a large one itself)
  {
    if (argb_only && npx > g->rgb0_cap)
    {
      GCHECK(hipSetDevice(g->dev[0]));
      GCHECK(hipDeviceSynchronize());  // any earlier frame on any stream may still write the old buffer
      (void)hipFree(g->rgb0);
      g->rgb0 = nullptr;
      g->rgb0_cap = 0;
      GCHECK(hipMalloc(&g->rgb0, npx * 3 * sizeof(float)));
      g->rgb0_cap = npx;
    }
    g->seq_ok = false;
    return rfx_render_frame(g->r[0], f, argb_only ? g->rgb0 : d_rgb, d_argb, nullptr, s0);
  }
  // a frame of more traces than one pass takes -- every member's band at most its launch limit, the pass under the band
  // scan's 2^31 -- runs as passes over consecutive row spans, each cut into equal bands (no balancing)
  const uint64_t spp = (uint64_t)f->sample_num * (uint64_t)f->sample_num;
  const uint64_t cap = std::min<uint64_t>((uint64_t)n * rfx_detail_launch_traces(g->r[0]), 1ull << 31);
  if (npx * spp > cap)
  {
    const uint64_t per = cap / ((uint64_t)W * spp);  // rows per pass
    if (!per) return rfx_detail_fail(RFX_ERR_ARG, "group_render_frame: one row exceeds 2^31 traces");
    GCHECK(hipSetDevice(g->dev[0]));
    const uint32_t jitter0 = rfx_detail_jitter(g->r[0]);
    // the frame's start state for a rewind, saved on member 0's stream after the caller's work (the first pass hands
    // member 0's state over when it differs)
    GCHECK(hipEventRecord(g->ev_start[0], s0));
    GCHECK(hipStreamWaitEvent(g->own[0], g->ev_start[0], 0));
    RCHECK(rfx_detail_save_start(g->r[0], g->own[0]));
    for (uint64_t y = 0; y < H; y += per)
    {
      const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)std::min<uint64_t>(H, y + per);
      const size_t m = std::min<size_t>(n, y1 - y0);
      std::vector<uint32_t> bd(m + 1);
      for (size_t i = 0; i <= m; ++i) bd[i] = y0 + (uint32_t)(((uint64_t)(y1 - y0) * i) / m);
      RCHECK(group_pass(g, f, y0, y1, bd, d_rgb, d_argb, s0));
    }
    g->timing_pending = false;  // the bands of a split frame are not the frame's bands
    rfx_detail_set_rewindable_saved(g->r[0], jitter0, s0);
    return RFX_OK;
  }
  if (W != g->W || H != g->H || g->bounds.size() != n + 1)
  {
    if (g->fixed && H != g->H) return rfx_detail_fail(RFX_ERR_ARG, "group_render_frame: fixed bands of another height");
    if (!g->fixed) g->bounds = equal_bounds(H, n);
    g->W = W;
    g->H = H;
    g->acc.assign(n, 0.0);
    g->acc_frames = 0;
    g->timing_pending = false;
  }
  RCHECK(collect_times(g));
  const int parity = (int)(g->frames & 1);
  RCHECK(group_pass(g, f, 0, H, g->bounds, d_rgb, d_argb, s0));
  g->timing_parity = parity;
  g->timing_pending = true;
  return RFX_OK;
}
