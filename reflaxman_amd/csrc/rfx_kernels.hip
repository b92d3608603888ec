// gfx950 kernels of librfx.so besides the trace kernel families (rfx_trace.h, rfx_trace_*.hip):
//   rng_count / rng_emit : the reference's serial LCG stream (trace_math.h:34-39, Vector3.cpp:176-188) as a
//       parallel pre-pass;
//   lpt_hist / lpt_scan / lpt_scatter : the longest-tile-first schedule of the trace launch;
//   qs_hist / qs_scan / qs_scatter : the regroup queue's bucket order (ray regrouping of large scenes);
//   kat_* : the trace kernel's primitive code on known-answer inputs (rfx.h rfx_kat_*);
// and the library-internal launchers.
#include "rfx_trace.h"

#pragma clang fp contract(off)

namespace rfx {

// ------------------------------------------------------------- LPT tile order
// The tile costs of a frame (clock cycles per tile) become the next launch's tile order, most
// expensive first: a counting sort on a log-scale key (exponent and 3 mantissa bits: buckets ~9% wide) over
// kLptGroups workgroups -- per-group LDS histograms, one scan of (bucket, group) offsets, a scatter.  The
// order within a bucket is whatever the LDS atomics give: any permutation renders the same pixels, only
// the schedule changes.
constexpr int kLptThreads = 1024, kLptBuckets = 256, kLptGroups = 64;

__device__ __forceinline__ uint32_t lpt_key(const uint32_t *cost, uint32_t i)
{
  const uint32_t c = max(cost[i], 1u);  // clock cycles from the workgroup's start to a wave's end (mod 2^32)
  const uint32_t e = 31u - (uint32_t)__clz(c);
  const uint32_t m = e >= 3u ? (c >> (e - 3u)) & 7u : (c << (3u - e)) & 7u;
  return (uint32_t)(kLptBuckets - 1) - min(e * 8u + m, (uint32_t)(kLptBuckets - 1));  // descending cost
}

// histogram of group g's tiles [g chunk, (g + 1) chunk) into hist[g][bucket]
__global__ __launch_bounds__(kLptThreads) void lpt_hist(const uint32_t *cost, uint32_t n, uint32_t chunk, uint32_t *hist)
{
  __shared__ uint32_t h[kLptBuckets];
  for (uint32_t b = threadIdx.x; b < kLptBuckets; b += kLptThreads) h[b] = 0;
  __syncthreads();
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kLptThreads) atomicAdd(&h[lpt_key(cost, i)], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kLptBuckets; b += kLptThreads) hist[blockIdx.x * kLptBuckets + b] = h[b];
}

// hist[g][b] <- first slot of group g's tiles of bucket b (buckets in order, groups in order within one).  The bucket
// totals' exclusive scan runs across the lanes (wave shuffles, then the four waves' totals), not in one thread: a
// serial pass over 256 LDS words held the sort's critical path (18 us of the tile sort's 28, rocprofv3).
__global__ __launch_bounds__(kLptBuckets) void lpt_scan(uint32_t *hist)
{
  __shared__ uint32_t wtot[kLptBuckets / 64];
  const uint32_t b = threadIdx.x, lane = b & 63u;
  uint32_t v[kLptGroups];  // all loads first (independent), then the running sum in registers
#pragma unroll
  for (int g = 0; g < kLptGroups; ++g) v[g] = hist[g * kLptBuckets + b];
  uint32_t run = 0;
#pragma unroll
  for (int g = 0; g < kLptGroups; ++g) { const uint32_t c = v[g]; v[g] = run; run += c; }
  uint32_t inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
  {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += t;
  }
  if (lane == 63u) wtot[b >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - run;
  for (uint32_t w = 0; w < (b >> 6); ++w) base += wtot[w];
#pragma unroll
  for (int g = 0; g < kLptGroups; ++g) hist[g * kLptBuckets + b] = v[g] + base;
}

__global__ __launch_bounds__(kLptThreads) void lpt_scatter(const uint32_t *cost, uint32_t n, uint32_t chunk,
                                                            const uint32_t *hist, uint32_t *order)
{
  __shared__ uint32_t off[kLptBuckets];
  for (uint32_t b = threadIdx.x; b < kLptBuckets; b += kLptThreads) off[b] = hist[blockIdx.x * kLptBuckets + b];
  __syncthreads();
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kLptThreads) order[atomicAdd(&off[lpt_key(cost, i)], 1u)] = i;
}

uint32_t trace_tiles(const FrameParams &P);

// bytes of scratch launch_tile_order needs
size_t tile_order_scratch() { return (size_t)kLptGroups * kLptBuckets * sizeof(uint32_t); }

hipError_t launch_tile_order(const uint32_t *cost, uint32_t n, uint32_t *order, uint32_t *scratch, hipStream_t st)
{
  const uint32_t chunk = (n + kLptGroups - 1) / kLptGroups;
  hipLaunchKernelGGL(lpt_hist, dim3(kLptGroups), dim3(kLptThreads), 0, st, cost, n, chunk, scratch);
  hipLaunchKernelGGL(lpt_scan, dim3(1), dim3(kLptBuckets), 0, st, scratch);
  hipLaunchKernelGGL(lpt_scatter, dim3(kLptGroups), dim3(kLptThreads), 0, st, cost, n, chunk, scratch, order);
  return hipGetLastError();
}

// ------------------------------------------------------------- regroup queue sort
// The parked traces of a frame (QRay queue, count on the device) listed bucket by bucket (rfx_trace.h queue_key:
// direction octant, origin cell), so that the bounce kernel's packed waves take traces that walk similar BVH paths.
// A counting sort over kQsGroups workgroups: per-group LDS histograms added into a global one, one scan, then each
// group reserves its range of every bucket with one atomic and ranks its entries in LDS.  The order within a bucket
// is whatever the atomics give: it changes which wave resumes a trace, never a value.
constexpr int kQsThreads = 1024, kQsGroups = 256;

__global__ __launch_bounds__(kQsThreads) void qs_hist(const uint32_t *count, const uint32_t *key, uint32_t *hist)
{
  __shared__ uint32_t h[kQueueBuckets];
  for (uint32_t b = threadIdx.x; b < kQueueBuckets; b += kQsThreads) h[b] = 0;
  __syncthreads();
  const uint32_t n = *count, chunk = (n + kQsGroups - 1) / kQsGroups;
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kQsThreads) atomicAdd(&h[key[i]], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kQueueBuckets; b += kQsThreads)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// hist <- exclusive prefix sums (the first slot of each bucket); 4 buckets per thread
__global__ __launch_bounds__(kQsThreads) void qs_scan(uint32_t *hist)
{
  static_assert(kQueueBuckets == 4 * kQsThreads, "qs_scan: 4 buckets per thread");
  __shared__ uint32_t s[kQsThreads];
  const uint32_t t = threadIdx.x;
  const uint4 v = reinterpret_cast<const uint4 *>(hist)[t];
  const uint32_t sum = v.x + v.y + v.z + v.w;
  s[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < kQsThreads; off <<= 1)
  {
    const uint32_t x = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  const uint32_t e = s[t] - sum;
  reinterpret_cast<uint4 *>(hist)[t] = make_uint4(e, e + v.x, e + v.x + v.y, e + v.x + v.y + v.z);
}

__global__ __launch_bounds__(kQsThreads) void qs_scatter(const uint32_t *count, const uint32_t *key, uint32_t *cursor,
                                                         uint32_t *order)
{
  __shared__ uint32_t h[kQueueBuckets];
  for (uint32_t b = threadIdx.x; b < kQueueBuckets; b += kQsThreads) h[b] = 0;
  __syncthreads();
  const uint32_t n = *count, chunk = (n + kQsGroups - 1) / kQsGroups;
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kQsThreads) atomicAdd(&h[key[i]], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kQueueBuckets; b += kQsThreads)
    if (h[b]) h[b] = atomicAdd(&cursor[b], h[b]);  // this group's first slot of bucket b
  __syncthreads();
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kQsThreads) order[atomicAdd(&h[key[i]], 1u)] = i;
}

// hist: kQueueBuckets zeroed words (the frame's queue counter memset clears them)
hipError_t launch_queue_sort(const uint32_t *count, const uint32_t *key, uint32_t *hist, uint32_t *order, hipStream_t st)
{
  hipLaunchKernelGGL(qs_hist, dim3(kQsGroups), dim3(kQsThreads), 0, st, count, key, hist);
  hipLaunchKernelGGL(qs_scan, dim3(1), dim3(kQsThreads), 0, st, hist);
  hipLaunchKernelGGL(qs_scatter, dim3(kQsGroups), dim3(kQsThreads), 0, st, count, key, hist, order);
  return hipGetLastError();
}

// ------------------------------------------------------------- RNG pre-pass
// Triple j of the stream (0-based) is LCG draws 3j+1..3j+3 after the frame's starting state.  Thread t
// of the pre-pass owns triples [16t, 16t + 16); its starting state is the frame state jumped 48t draws,
// composed from two host-made tables of affine LCG maps (A, C): 48*256*b draws for its block b and
// 48*tid draws for its place in the block -- two multiply-adds instead of a 27-step binary power.
constexpr int kTriplesPerThread = 16;
constexpr int kRngBlock = 256;
constexpr uint64_t kTriplesPerBlock = (uint64_t)kTriplesPerThread * kRngBlock;

__device__ __forceinline__ uint32_t thread_state(uint32_t s, const uint32_t *jump, uint64_t b, uint32_t tid)
{
  const uint32_t *bj = jump + 2 * (kRngBlock + b), *tj = jump + 2 * tid;
  return tj[0] * (bj[0] * s + bj[1]) + tj[1];
}

// A thread's 16-triple run as two chains of 8 triples each (the second starts 24 draws later: one affine
// jump), so two independent LCG dependency chains interleave -- the same states, half the serial latency.
constexpr int kHalfRun = kTriplesPerThread / 2;
struct LcgJump { uint32_t a, c; };
constexpr LcgJump lcg_jump_const(int draws)
{
  uint32_t a = 1u, c = 0u;
  for (int i = 0; i < draws; ++i) { a = 214013u * a; c = 214013u * c + 2531011u; }
  return LcgJump{a, c};
}
constexpr LcgJump kHalfJump = lcg_jump_const(3 * kHalfRun);
struct TripleJumps { LcgJump m[kTriplesPerThread]; };
constexpr TripleJumps triple_jumps()
{
  TripleJumps t{};
  for (int j = 0; j < kTriplesPerThread; ++j) t.m[j] = lcg_jump_const(3 * j);
  return t;
}
constexpr TripleJumps kTripleJump = triple_jumps();  // (A, C) of 3j draws, j < 16: triple j's state from the thread's

// Vector3.cpp:182-185's accept test of one triple of draws k1..k3: !(x*x + y*y + z*z > 1) in float, x = k / 16383.5 - 1.
__device__ __forceinline__ bool float_accept(uint32_t s1, uint32_t s2, uint32_t s3)
{
  const float x = rand_component_dev(lcg_out(s1)), y = rand_component_dev(lcg_out(s2)),
              z = rand_component_dev(lcg_out(s3));
  return !(x * x + y * y + z * z > 1.f);                                        // Vector3.cpp:185
}

// The same test in integers: x is within 2^-23 of v / 32767, v = 2k - 32767, so the float test agrees with
// N = v1^2 + v2^2 + v3^2 <= 32767^2 except on a thin shell around the sphere.  tests/native/sphere_shell.c checks all
// 2^45 triples: every accepted triple has N <= 32767^2 + 298 and every rejected one N >= 32767^2 - 174, so outside
// |N - 32767^2| <= kSphereShell the integer answer is the float one.  A thread with a triple inside the shell (about 3
// threads in 10^5) redoes its 16 in float.  Per draw: a bit-field extract and two 24-bit multiply-adds, not eight
// operations.
#ifndef RFX_RNG_INT_ACCEPT
#define RFX_RNG_INT_ACCEPT 1
#endif
constexpr uint32_t kSphereN = 32767u * 32767u;
constexpr uint32_t kSphereShell = 1024u;

// N of draws k1..k3 from the k alone: N = 4 (k1^2 + k2^2 + k3^2) - 4 * 32767 (k1 + k2 + k3) + 3 * 32767^2, evaluated
// mod 2^32 (N < 2^32), every product a 24-bit one.  The squares are v_mad_u32_u24 in inline asm: written in C (k * k or
// __umul24), this compiler (ROCm 7.2, clang 22) folds two of them into v_perm + v_dot4_u32_u8 over one byte of each k
// only, dropping bits 8..14 (tests/test_sphere_shell.py checks the built code object for that instruction).
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c)
{
  uint32_t d;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

__device__ __forceinline__ uint32_t sphere_n(uint32_t k1, uint32_t k2, uint32_t k3)
{
  const uint32_t q = mad_u24(k3, k3, mad_u24(k2, k2, mad_u24(k1, k1, 0u))), t = k1 + k2 + k3;
  return 4u * q - 131068u * t + 3u * kSphereN;
}

// one triple from state s (advanced past it): its accept flag into bit j of acc, and (integer test) bit j of und when
// it lies inside the shell
__device__ __forceinline__ void triple(uint32_t &s, int j, uint32_t &acc, uint32_t &und)
{
  const uint32_t s1 = lcg_step(s), s2 = lcg_step(s1), s3 = lcg_step(s2);
  s = s3;
#if RFX_RNG_INT_ACCEPT
  const uint32_t n = sphere_n(lcg_out(s1), lcg_out(s2), lcg_out(s3));
  acc |= (n < kSphereN ? 1u : 0u) << j;
  und |= (n - (kSphereN - kSphereShell) <= 2u * kSphereShell ? 1u : 0u) << j;
#else
  acc |= (float_accept(s1, s2, s3) ? 1u : 0u) << j;
#endif
}

// the 16 accept flags of the thread whose first triple starts at state s0 (bit j: triple j); st (optional): the state
// before each triple
template <bool kStates>
__device__ __forceinline__ uint32_t thread_flags(uint32_t s0, uint32_t *st)
{
  uint32_t s = s0, s2 = kHalfJump.a * s0 + kHalfJump.c, acc = 0, und = 0;
#pragma unroll
  for (int j = 0; j < kHalfRun; ++j)
  {
    if (kStates)
    {
      st[j] = s;
      st[j + kHalfRun] = s2;
    }
    triple(s, j, acc, und);
    triple(s2, j + kHalfRun, acc, und);
  }
  if (__builtin_expect(und != 0u, 0))
  {
    // a triple on the shell: the thread's 16 in float, one chain (rare enough that its latency does not matter)
    acc = 0u;
    s = s0;
#pragma nounroll
    for (int j = 0; j < kTriplesPerThread; ++j)
    {
      const uint32_t s1 = lcg_step(s), s2b = lcg_step(s1), s3 = lcg_step(s2b);
      s = s3;
      acc |= (float_accept(s1, s2b, s3) ? 1u : 0u) << j;
    }
  }
  return acc;
}

// accepted-triple count of blocks [blk0, blk0 + gridDim.x): one slice of the stream (multi-GPU: one per rank)
// masks (optional, one device): each thread's 16 accept flags, so that rng_emit regenerates only the LCG states
__global__ __launch_bounds__(kRngBlock) void rng_count(const uint32_t *seed, const uint32_t *jump, uint32_t *blk_cnt,
                                                       uint64_t blk0, uint16_t *masks)
{
  const uint64_t b = blk0 + blockIdx.x;
  const uint32_t acc = thread_flags<false>(thread_state(*seed, jump, b, threadIdx.x), nullptr);
  uint32_t c = (uint32_t)__popc(acc);
  if (masks) masks[b * kRngBlock + threadIdx.x] = (uint16_t)acc;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  __shared__ uint32_t wsum[kRngBlock / 64];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0)
  {
    uint32_t tot = 0;
    for (int w = 0; w < kRngBlock / 64; ++w) tot += wsum[w];
    blk_cnt[b] = tot;
  }
}

// Which traces a rank needs randDirs for: trace i -> pixel i / ss2 -> row -> strip (row / row_block)
// -> owner strip % nranks (rfx_strip_row_to_y); nranks <= 1: the traces [lo, hi) (a band of rows, or every trace).
struct EmitFilter {
  uint64_t ss2;       // traces per pixel (ss^2), 1 in block mode
  uint64_t W;         // pixels per row of the trace index space
  uint32_t row_block, rank, nranks;
  uint64_t lo, hi;    // nranks <= 1: trace range written
};

__device__ __forceinline__ bool owned(uint64_t idx, const EmitFilter &f)
{
  if (f.nranks <= 1) return idx >= f.lo && idx < f.hi;
  return ((idx / f.ss2 / f.W / f.row_block) % f.nranks) == f.rank;
}

// Scatter of the accepted triples: block b's accepted triples are the contiguous trace range
// [off_b, off_b + blk_cnt[b]), off_b the sum of the counts before b.  Each thread regenerates its 16
// triples, keeping for each the LCG state before its three draws; the block scans the accept counts,
// places the accepted triples' states in LDS at their block-local rank, and writes the range out with
// coalesced 4-byte stores.  Trace i then re-derives its randDir from that state (rd_from_state): three
// LCG steps and three exact conversions.
constexpr int kScanThreads = 1024;

// The inputs of block b's emit: its accept count, the thread's first LCG state and (one device) its 16 accept flags.
// Loaded together -- rng_emit issues them with the prefix sum's loads, so the block waits on memory once.
struct EmitIn {
  uint32_t cnt, s0, mask;
};
__device__ __forceinline__ EmitIn emit_in(uint32_t b, const uint32_t *seed, const uint32_t *jump, const uint32_t *blk_cnt,
                                          const uint16_t *masks)
{
  EmitIn e;
  e.cnt = blk_cnt[b];
  e.s0 = thread_state(*seed, jump, b, threadIdx.x);
  e.mask = masks ? (uint32_t)masks[(uint64_t)b * kRngBlock + threadIdx.x] : 0u;
  return e;
}

// One block of the emit: block b's accepted triples are the traces [off, off + in.cnt).  Every thread of the workgroup
// calls it with the same off and b's inputs (emit_in).  have_masks: in.mask holds the thread's accept flags (rng_count's), so only the LCG
// states are regenerated.
__device__ __forceinline__ void emit_block(uint64_t off, const EmitIn &in, bool have_masks, uint64_t need,
                                           uint32_t *rd_state, uint32_t *next_seed, const EmitFilter &flt,
                                           uint32_t *sst, uint32_t *wsum)
{
  if (off >= need) return;
  const uint32_t cnt = (uint32_t)min((uint64_t)in.cnt, need - off);  // triples this block emits
  const uint64_t last = off + cnt - 1;
  // block-uniform skip: a block whose accepted indices all belong to other ranks' strips (and do not
  // include the frame's last trace, whose stream state every rank carries forward) writes nothing
  if (flt.nranks <= 1 && last != need - 1 && (last < flt.lo || off >= flt.hi)) return;  // outside the band
  if (flt.nranks > 1 && last != need - 1)
  {
    const uint64_t s_lo = off / flt.ss2 / flt.W / flt.row_block, s_hi = last / flt.ss2 / flt.W / flt.row_block;
    bool any = false;
    for (uint64_t st = s_lo; st <= s_hi && !any; ++st) any = (st % flt.nranks) == flt.rank;
    if (!any) return;
  }
  uint32_t st[kTriplesPerThread];
  uint32_t acc;
  if (have_masks)
  {
    acc = in.mask;
    // each triple's state straight from the thread's: one affine jump of 3j draws (a multiply-add), not 3j steps
#pragma unroll
    for (int j = 0; j < kTriplesPerThread; ++j) st[j] = kTripleJump.m[j].a * in.s0 + kTripleJump.m[j].c;
  }
  else
    acc = thread_flags<true>(in.s0, st);
  const uint32_t c = (uint32_t)__popc(acc);
  // exclusive scan of c across the workgroup
  const uint32_t lane = threadIdx.x & 63;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
  {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += v;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) wbase += wsum[w];
  uint32_t li = wbase + (inc - c);                                               // block-local rank
  // trace need - 1's block-local rank when this block holds it (the stream state after its triple is the next frame's)
  const uint32_t fin = last == need - 1 ? cnt - 1 : ~0u;
#pragma unroll
  for (int j = 0; j < kTriplesPerThread; ++j)
    if ((acc >> j) & 1u)
    {
      if (li == fin) *next_seed = lcg_step(lcg_step(lcg_step(st[j])));
      if (li < cnt) sst[li] = st[j];
      ++li;
    }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cnt; i += kRngBlock)
  {
    const uint64_t idx = off + i;
    if (owned(idx, flt)) rd_state[idx] = sst[i];
  }
}

__global__ __launch_bounds__(kRngBlock) void rng_emit(const uint32_t *seed, const uint32_t *jump, const uint32_t *blk_cnt,
                                                      const uint16_t *masks, uint64_t need, uint32_t *rd_state,
                                                      uint32_t *next_seed, int *err, EmitFilter flt)
{
  __shared__ uint32_t sst[kTriplesPerBlock];
  __shared__ uint32_t wsum[kRngBlock / 64];
  __shared__ uint32_t wpart[kRngBlock / 64];
  // the block's own inputs first: their loads are in flight with the prefix sum's
  const EmitIn in = emit_in(blockIdx.x, seed, jump, blk_cnt, masks);
  // this block's first trace: the accept counts of the blocks before it, summed by the block (the count
  // array is a few KB and L2-resident, so no separate scan pass)
  uint32_t part = 0;
  if (((uintptr_t)blk_cnt & 15u) == 0)
  {
    // 16-byte loads, up to four per thread in flight before any is summed: one round trip to L2 per 4096 counts
    const uint4 *v4 = reinterpret_cast<const uint4 *>(blk_cnt);
    const uint32_t nvec = blockIdx.x >> 2;
    for (uint32_t k0 = 0; k0 < nvec; k0 += 4 * kRngBlock)
    {
      uint4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
      {
        const uint32_t k = k0 + (uint32_t)u * kRngBlock + threadIdx.x;
        a[u] = k < nvec ? v4[k] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) part += a[u].x + a[u].y + a[u].z + a[u].w;
    }
    if (threadIdx.x < (blockIdx.x & 3u)) part += blk_cnt[(nvec << 2) + threadIdx.x];
  }
  else
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += kRngBlock) part += blk_cnt[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = part;
  __syncthreads();
  uint64_t off = 0;  // (a launch has fewer than 2^32 traces, so each wave's partial fits 32 bits)
#pragma unroll
  for (int w = 0; w < kRngBlock / 64; ++w) off += wpart[w];
  // the last block flags a stream too short for the frame (host: RFX_ERR_RNG)
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0 && off + in.cnt < need) *err = 1;
  emit_block(off, in, masks != nullptr, need, rd_state, next_seed, flt, sst, wsum);
}

// Band emit (multi-GPU band partition): only the blocks holding the band's traces [flt.lo, flt.hi), and the block of
// the frame's last trace (every rank carries the stream state past it), run -- a rank of N emits about 1/N of the
// blocks instead of launching all of them.  One workgroup scans the counts into offsets and finds those blocks
// (range: first, last, final); the emit's workgroups then loop over them.
// One workgroup, tiles of kScanTile counts staged in LDS with coalesced loads (the counts are L2-resident, so
// per-thread serial loads would leave it latency-bound): each thread scans 16 contiguous counts from LDS, the 1024
// partial sums are scanned with wave shuffles, and the offsets leave with coalesced stores.  Offsets fit 32 bits
// (a frame has fewer than 2^32 traces).
constexpr uint32_t kScanTile = 16 * kScanThreads;
__global__ __launch_bounds__(kScanThreads) void rng_band_range(const uint32_t *blk_cnt, uint64_t nblk, uint64_t need,
                                                               uint64_t lo, uint64_t hi, uint64_t *off, uint32_t *range,
                                                               int *err)
{
  __shared__ uint32_t t[kScanTile];
  __shared__ uint32_t wsum[kScanThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  if (tid == 0) { range[0] = 0; range[1] = 0; range[2] = 0; }
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nblk; base += kScanTile)
  {
    const uint32_t n = (uint32_t)min((uint64_t)kScanTile, nblk - base);
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
    {
      const uint32_t i = k * kScanThreads + tid;
      t[i] = i < n ? blk_cnt[base + i] : 0u;
    }
    __syncthreads();
    uint32_t c[16], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) { c[k] = t[16 * tid + k]; sum += c[k]; }
    // exclusive scan of the 1024 thread sums: within each wave by shuffles, then over the 16 wave totals
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
    {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += v;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (uint32_t w = 0; w < kScanThreads / 64; ++w)
    {
      wb += w < wv ? wsum[w] : 0u;
      tot += wsum[w];
    }
    uint64_t run = carry + wb + (inc - sum);
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
    {
      // block base + 16 tid + k holds traces [run, run + c): the band's first / last block and the frame's final one
      const uint64_t b = base + 16 * tid + k, e = run + c[k];
      if (c[k] && run <= lo && lo < e) range[0] = (uint32_t)b;
      if (c[k] && run <= hi - 1 && hi - 1 < e) range[1] = (uint32_t)b;
      if (c[k] && run <= need - 1 && need - 1 < e) range[2] = (uint32_t)b;
      t[16 * tid + k] = (uint32_t)run;
      run = e;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
    {
      const uint32_t i = k * kScanThreads + tid;
      if (i < n) off[base + i] = t[i];
    }
    carry += tot;
    __syncthreads();
  }
  if (tid == 0 && carry < need) *err = 1;  // stream too short for the frame
}

// The same scan over many workgroups (launches of many blocks: a split frame's 2^30-trace spans have 524K).  One
// workgroup scanning 524K counts runs for milliseconds beside the other stream's trace, which holds the chip's issue
// slots; two kernels of one workgroup per tile of kScanTileCounts counts do it in parallel:
//   rng_tile_sums: each tile's total (coalesced 16-byte loads, a workgroup reduction);
//   rng_tile_scan: each tile's prefix (the totals of the tiles before it, at most a few hundred words), then the tile's
//   exclusive scan, the offsets, and the band's / the frame's range blocks found in the tile.
constexpr uint32_t kScanTileCounts = 4096, kTileSumThreads = 256;
__global__ __launch_bounds__(kTileSumThreads) void rng_tile_sums(const uint32_t *blk_cnt, uint64_t nblk,
                                                                 uint32_t *tile_sum, uint32_t *range)
{
  __shared__ uint32_t wsum[kTileSumThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTileCounts;
  const uint32_t n = (uint32_t)min((uint64_t)kScanTileCounts, nblk - base);
  uint32_t sum = 0;
  if (n == kScanTileCounts && ((uintptr_t)(blk_cnt + base) & 15u) == 0)
  {
    const uint4 *v = reinterpret_cast<const uint4 *>(blk_cnt + base);
#pragma unroll
    for (uint32_t k = 0; k < kScanTileCounts / 4 / kTileSumThreads; ++k)
    {
      const uint4 a = v[k * kTileSumThreads + threadIdx.x];
      sum += a.x + a.y + a.z + a.w;
    }
  }
  else
    for (uint32_t i = threadIdx.x; i < n; i += kTileSumThreads) sum += blk_cnt[base + i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0)
  {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kTileSumThreads / 64; ++w) t += wsum[w];
    tile_sum[blockIdx.x] = t;
    if (blockIdx.x == 0) { range[0] = 0; range[1] = 0; range[2] = 0; }  // rng_tile_scan runs after every tile sum
  }
}

__global__ __launch_bounds__(kScanThreads) void rng_tile_scan(const uint32_t *blk_cnt, uint64_t nblk, uint64_t need,
                                                              uint64_t lo, uint64_t hi, const uint32_t *tile_sum,
                                                              uint64_t *off, uint32_t *range, int *err)
{
  __shared__ uint32_t wsum[kScanThreads / 64];
  __shared__ uint64_t s_pre;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  // this tile's prefix: the totals of the tiles before it
  unsigned long long pre = 0;
  for (uint32_t t = tid; t < blockIdx.x; t += kScanThreads) pre += tile_sum[t];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (tid == 0) s_pre = 0;
  __syncthreads();
  if (lane == 0 && pre) atomicAdd((unsigned long long *)&s_pre, pre);
  __syncthreads();
  // four counts per thread: one 16-byte load where the tile is whole and aligned
  const uint64_t base = (uint64_t)blockIdx.x * kScanTileCounts;
  const uint64_t b0 = base + 4u * tid;
  uint32_t c[4];
  if (b0 + 3 < nblk && ((uintptr_t)(blk_cnt + b0) & 15u) == 0)
  {
    const uint4 a = *reinterpret_cast<const uint4 *>(blk_cnt + b0);
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
  }
  else
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) c[k] = b0 + k < nblk ? blk_cnt[b0 + k] : 0u;
  const uint32_t sum = c[0] + c[1] + c[2] + c[3];
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
  {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += v;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (uint32_t w = 0; w < kScanThreads / 64; ++w)
  {
    wb += w < wv ? wsum[w] : 0u;
    tot += wsum[w];
  }
  uint64_t run = s_pre + wb + (inc - sum);
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
  {
    const uint64_t b = b0 + k, e = run + c[k];
    if (b < nblk)
    {
      // block b holds traces [run, e): the band's first / last block and the frame's final one (one block each)
      if (c[k] && run <= lo && lo < e) range[0] = (uint32_t)b;
      if (c[k] && run <= hi - 1 && hi - 1 < e) range[1] = (uint32_t)b;
      if (c[k] && run <= need - 1 && need - 1 < e) range[2] = (uint32_t)b;
      off[b] = run;
    }
    run = e;
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0 && s_pre + tot < need) *err = 1;  // stream too short for the frame
}

__global__ __launch_bounds__(kRngBlock) void rng_emit_band(const uint32_t *seed, const uint32_t *jump,
                                                           const uint32_t *blk_cnt, const uint16_t *masks,
                                                           const uint64_t *off, const uint32_t *range, uint64_t nblk,
                                                           uint64_t need, uint32_t *rd_state, uint32_t *next_seed,
                                                           EmitFilter flt)
{
  __shared__ uint32_t sst[kTriplesPerBlock];
  __shared__ uint32_t wsum[kRngBlock / 64];
  const uint32_t first = range[0], last = range[1], fin = range[2];
  const uint32_t n = last - first + 1 + (fin > last || fin < first ? 1u : 0u);  // the band's blocks, then the final one
  for (uint32_t j = blockIdx.x; j < n; j += gridDim.x)
  {
    const uint32_t b = j <= last - first ? first + j : fin;
    if (b >= nblk) break;  // (a stream too short for the frame leaves the range unset: the error flag is raised)
    emit_block(off[b], emit_in(b, seed, jump, blk_cnt, masks), masks != nullptr, need, rd_state, next_seed, flt, sst,
               wsum);
    __syncthreads();  // sst / wsum are reused by the next block
  }
}

// One-pass pre-pass (one device, no partition): count, scan and scatter in one launch.  Each workgroup generates its
// 16 triples per thread once (states and accept flags), publishes its accept count, then finds its offset by decoupled
// look-back over the published words of the blocks before it -- 64 at a time, one per lane of the first wave -- until
// one holds an inclusive prefix; it publishes its own inclusive prefix and scatters as emit_block does.  A status word
// is epoch << 36 | flag << 34 | value (flag 1: the block's count, 2: its inclusive prefix); a word of another launch's
// epoch reads as not yet published, so the array is never cleared (the host clears it when the epoch wraps).
// Block order: an ordered ticket, not blockIdx.x.  The hardware's workgroup dispatch order is not specified
// (MI355X_MICROARCH.md: placement-independent protocols only), and with the ticket a block only ever waits on blocks that
// took smaller tickets -- blocks already running, each waiting only on smaller tickets again -- so the look-back always
// finishes, in any dispatch order and beside any other kernel (rocPRIM's ordered_block_id does the same).  The ticket
// word counts up across launches and is never reset: the host passes the count of tickets its earlier launches took
// (base), so no launch races another's reset.  The waits stay bounded as a guard against a broken invariant, never as a
// path a correct launch takes: past kLookbackSpins polls the block recomputes its offset from the random stream itself
// (below), so even then the frame's randDirs are exact and no later call is left to report a wrong frame.
// RFX_RNG_TICKET=0 keeps the blockIdx.x order (timing builds only: it relies on in-order dispatch).
#ifndef RFX_RNG_TICKET
#define RFX_RNG_TICKET 1
#endif
#ifndef RFX_LOOKBACK_SLEEP
#define RFX_LOOKBACK_SLEEP 1  // s_sleep between polls of a not yet published status word (units of 64 cycles)
#endif
constexpr uint64_t kStatAgg = 1ull << 34, kStatPre = 2ull << 34, kStatVal = (1ull << 34) - 1;
#ifndef RFX_LOOKBACK_SPINS
#define RFX_LOOKBACK_SPINS (1u << 22)  // 0: every wait gives up at once (a timing build that exercises the fallback)
#endif
constexpr uint32_t kLookbackSpins = RFX_LOOKBACK_SPINS;

// Relaxed device-scope accesses: a status word carries its own value, and no other data is handed over through it, so
// no fence is needed (release / acquire at device scope would write back and invalidate the XCDs' L2s on every access).
__device__ __forceinline__ unsigned long long status_load(const unsigned long long *p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void status_store(unsigned long long *p, unsigned long long v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kRngBlock) void rng_fused(const uint32_t *seed, const uint32_t *jump, uint32_t nblk,
                                                       uint64_t need, uint32_t *rd_state, uint32_t *next_seed, int *err,
                                                       unsigned long long *status, unsigned long long *ticket,
                                                       unsigned long long base, uint32_t epoch)
{
  __shared__ uint32_t sst[kTriplesPerBlock];
  __shared__ uint32_t wsum[kRngBlock / 64];
  __shared__ uint64_t s_off;
  uint32_t b = blockIdx.x;
#if RFX_RNG_TICKET
  __shared__ uint32_t s_b;
  if (threadIdx.x == 0) s_b = (uint32_t)(atomicAdd(ticket, 1ull) - base);
  __syncthreads();
  b = s_b;
#endif
  // the block's triples, generated once: the state before each and its accept flag (rng_count / emit_block)
  uint32_t st[kTriplesPerThread];
  const uint32_t acc = thread_flags<true>(thread_state(*seed, jump, b, threadIdx.x), st);
  const uint32_t c = (uint32_t)__popc(acc);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
  {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += v;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = inc;
  __shared__ uint32_t s_gaveup;
  if (threadIdx.x == 0) s_gaveup = 0;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
  for (uint32_t w = 0; w < kRngBlock / 64; ++w)
  {
    if (w < (threadIdx.x >> 6)) wbase += wsum[w];
    tot += wsum[w];
  }
  const unsigned long long tag = (unsigned long long)epoch << 36;
  if (threadIdx.x < 64)
  {
    uint64_t excl = 0;
    if (b == 0)
    {
      if (lane == 0) status_store(&status[0], tag | kStatPre | tot);
    }
    else
    {
      if (lane == 0) status_store(&status[b], tag | kStatAgg | tot);
      int64_t j = (int64_t)b - 1 - (int64_t)lane;  // this lane's predecessor in the window
      uint32_t spins = 0;
      bool gaveup = false;
      for (;;)
      {
        const unsigned long long w = j >= 0 ? status_load(&status[j]) : (tag | kStatPre);
        const bool ready = (w >> 36) == (unsigned long long)epoch && (w & (3ull << 34)) != 0;
        const uint64_t pre = __ballot(ready && (w & (3ull << 34)) == kStatPre);
        const uint32_t first = pre ? (uint32_t)__builtin_ctzll(pre) : 64u;  // nearest predecessor with a prefix
        const uint64_t upto = first >= 63 ? ~0ull : (2ull << first) - 1ull;
        if (__ballot(!ready) & upto)
        {
          if (++spins > kLookbackSpins)
          {
            gaveup = true;
            break;
          }
          __builtin_amdgcn_s_sleep(RFX_LOOKBACK_SLEEP);
          continue;
        }
        uint64_t v = lane <= first ? (uint64_t)(w & kStatVal) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (first < 64) break;
        j -= 64;
      }
      if (gaveup)
      {
        if (lane == 0) s_gaveup = 1;
      }
      else if (lane == 0)
        status_store(&status[b], tag | kStatPre | ((excl + tot) & kStatVal));
    }
    if (lane == 0) s_off = excl;
  }
  __syncthreads();
  if (s_gaveup)
  {
    // The look-back outwaited its bound (only a broken invariant gets here): the offset is recomputed from the random
    // stream itself -- the accept counts of blocks 0 .. b - 1, regenerated by this workgroup -- so the frame's randDirs
    // stay exact whatever the other blocks do.  Bit 4 of the error word records that it happened (not an error: the
    // frame is exact; rfx_synchronize fails only on bits 1 and 2).
    uint32_t part = 0;
    for (uint32_t pb = 0; pb < b; ++pb)
    {
      part += (uint32_t)__popc(thread_flags<false>(thread_state(*seed, jump, pb, threadIdx.x), nullptr));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (threadIdx.x == 0) s_off = 0;
    __syncthreads();
    if (lane == 0) atomicAdd((unsigned long long *)&s_off, (unsigned long long)part);
    __syncthreads();
    if (threadIdx.x == 0)
    {
      status_store(&status[b], tag | kStatPre | ((s_off + tot) & kStatVal));
      atomicOr(err, 4);
    }
  }
  const uint64_t off = s_off;
  if (b == nblk - 1 && threadIdx.x == 0 && off + tot < need) *err = 1;  // stream too short for the frame
  if (off >= need) return;
  const uint32_t cnt = (uint32_t)min((uint64_t)tot, need - off);
  uint32_t li = wbase + (inc - c);                                               // block-local rank
  const uint32_t fin = off + cnt == need ? cnt - 1 : ~0u;  // trace need - 1's block-local rank, if this block holds it
#pragma unroll
  for (int j = 0; j < kTriplesPerThread; ++j)
    if ((acc >> j) & 1u)
    {
      if (li == fin) *next_seed = lcg_step(lcg_step(lcg_step(st[j])));
      if (li < cnt) sst[li] = st[j];
      ++li;
    }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cnt; i += kRngBlock) rd_state[off + i] = sst[i];
}

// ------------------------------------------------------------- device known-answer kernels
// Thread i runs the trace kernel's own device code on one case (rfx.h rfx_kat_*), so the reference's
// known answers (tests/golden/kat_*.npz, outputs of the unmodified Sphere / Triangle / Plane / Skybox /
// Texture / Color / powf code) pin every device primitive, edge cases no rendered frame reaches included.
constexpr uint32_t kKatThreads = 256;

__device__ __forceinline__ void stage_lut(float *lut)
{
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = (float)i / 255.0f;  // Color.cpp:11-13
}

// rays: n x 6 (origin, direction); objs: n object indices of S; out: n x 15 -- hit, drop, normal, reflected
// ray, distance, material colour (the texel of a textured triangle), any-hit: the refharness kat_* layout.
// The closest-hit derivation is the bounce loop's: the test up to t (and |ray t|^2), then the winner's
// drop = origin + ray t, normal, reflect(ray t, normal) and distance sqrt(|ray t|^2).
__global__ __launch_bounds__(kKatThreads) void kat_objects(DevScene S, const float *rays, const int32_t *objs, uint32_t n,
                                                          float *out)
{
  __shared__ float lut[256];
  stage_lut(lut);
  __syncthreads();
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  if (i >= n) return;
  Cnt cnt;
  const float *q = rays + 6 * (size_t)i;
  const v3 o = mk(q[0], q[1], q[2]), ray = mk(q[3], q[4], q[5]);
  const int32_t loc = S.obj_loc[objs[i]];
  const int kind = loc >> 28, idx = loc & 0x0FFFFFFF;
  const RayConst k = ray_const(ray);
  bool hit = false, any = false, pre_bad = false;
  float t = 0.0f, sq = 0.0f, t2, sq2, u = 0.0f, v = 0.0f, u2, v2;
  v3 norm = mk(0.0f, 0.0f, 0.0f), drop = o;
  col c = mkc(0.0f, 0.0f, 0.0f);
  if (kind == 0)
  {
    const SphereGeo g = S.sph_geo[idx];
    SpherePair p;
    p.cx[0] = g.cx; p.cy[0] = g.cy; p.cz[0] = g.cz; p.r2[0] = g.sq_radius;
    p.cx[1] = 0.0f; p.cy[1] = 0.0f; p.cz[1] = 0.0f; p.r2[1] = -INFINITY;  // the padding of an odd count
    f2 b, d;
    pair_bd(p, o, k, b, d);
    hit = pair_may_hit(b, d) && sphere_tail<false, false>(b.x, d.x, ray, k, t, sq, cnt);
    any = pair_may_hit(b, d) && sphere_tail<false, true>(b.x, d.x, ray, k, t2, sq2, cnt);
    if (hit)
    {
      drop = add(o, mul(ray, t));
      norm = sub(drop, mk(g.cx, g.cy, g.cz));
      const MatRec m = S.sph_mat[idx];
      c = mkc(m.r, m.g, m.b);
    }
  }
  else if (kind == 1)
  {
    hit = tri_hit<false, false>(S.tri_geo[idx], o, ray, t, u, v, sq, cnt, k);
    any = tri_hit<false, true>(S.tri_geo[idx], o, ray, t2, u2, v2, sq2, cnt, k);
    // the large-scene shadow form (reject before the divide) must decide alike: a disagreement reads as NaN
    if (tri_hit<false, true, true>(S.tri_geo[idx], o, ray, t2, u2, v2, sq2, cnt, k) != any) pre_bad = true;
    if (hit)
    {
      drop = add(o, mul(ray, t));
      const TriShade sh = S.tri_shade[idx];
      norm = mk(sh.nx, sh.ny, sh.nz);
      const MatRec m = S.tri_mat[idx];
      c = sh.tex >= 0 ? tri_texel<false>(S, sh, u, v, lut, cnt) : mkc(m.r, m.g, m.b);
    }
  }
  else
  {
    const PlaneGeo g = S.pln_geo[idx];
    hit = plane_hit<false, false>(g, o, ray, t, sq, cnt, k);
    any = plane_hit<false, true>(g, o, ray, t2, sq2, cnt, k);
    if (hit)
    {
      drop = add(o, mul(ray, t));
      norm = mk(g.nx, g.ny, g.nz);
      const MatRec m = S.pln_mat[idx];
      c = mkc(m.r, m.g, m.b);
    }
  }
  float *w = out + 15 * (size_t)i;
  for (int j = 0; j < 15; ++j) w[j] = 0.0f;
  w[0] = hit ? 1.0f : 0.0f;
  if (hit)
  {
    const v3 rf = reflect(mul(ray, t), norm);
    w[1] = drop.x; w[2] = drop.y; w[3] = drop.z;
    w[4] = norm.x; w[5] = norm.y; w[6] = norm.z;
    w[7] = rf.x; w[8] = rf.y; w[9] = rf.z;
    w[10] = sqrt_rn(sq);
    w[11] = c.r; w[12] = c.g; w[13] = c.b;
  }
  w[14] = pre_bad ? __builtin_nanf("") : any ? 1.0f : 0.0f;
}

// tex >= 0: Texture::getTexelColor(u, v) of texture tex (in: n x 2); tex < 0: Skybox::getTexelColor(ray)
// (in: n x 3).  out: n x 3.
__global__ __launch_bounds__(kKatThreads) void kat_texels(DevScene S, int tex, const float *in, uint32_t n, float *out)
{
  __shared__ float lut[256];
  stage_lut(lut);
  __syncthreads();
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  if (i >= n) return;
  Cnt cnt;
  const col c = tex >= 0 ? texel_uv<false>(S, tex, in[2 * (size_t)i], in[2 * (size_t)i + 1], lut, cnt)
                         : skybox_texel<false>(S, mk(in[3 * (size_t)i], in[3 * (size_t)i + 1], in[3 * (size_t)i + 2]), lut, cnt);
  out[3 * (size_t)i] = c.r; out[3 * (size_t)i + 1] = c.g; out[3 * (size_t)i + 2] = c.b;
}

// pow(x, y) as the bounce loop evaluates it (Scene.cpp:175,196): xy n x 2 -> out n
__global__ __launch_bounds__(kKatThreads) void kat_powf(const float *xy, uint32_t n, float *out)
{
  stage_powf_tables();
  __syncthreads();
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  if (i < n)
  {
    const float x = xy[2 * (size_t)i], y = xy[2 * (size_t)i + 1];
    out[i] = y == 3.0f ? powf3_dev(x) : powf_dev(x, y);  // Scene.cpp:196 runs the cube form, :175 the general one
  }
}

// powf3_dev(x) against powf_dev(x, 3) for the float bit patterns first .. first + n - 1 (every float in [0, 1] is
// 0 .. 0x3f800000): counts[0] += mismatches, counts[1] += lanes that took glibc's algorithm
__global__ __launch_bounds__(kKatThreads) void kat_powf_cube(uint32_t first, uint32_t n, unsigned long long *counts)
{
  stage_powf_tables();
  __syncthreads();
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  bool bad = false, slow = false;
  if (i < n)
  {
    const float x = __uint_as_float(first + i);
    float p;
    slow = !powf_cube_fast(x, p);
    bad = __float_as_uint(powf3_dev(x)) != __float_as_uint(powf_dev(x, 3.0f));
  }
  const uint64_t mb = __ballot(bad), ms = __ballot(slow);
  if ((threadIdx.x & 63u) == 0 && (mb | ms))
  {
    atomicAdd(&counts[0], (unsigned long long)__popcll(mb));
    atomicAdd(&counts[1], (unsigned long long)__popcll(ms));
  }
}

// rfx_math.h's division fast paths (div_rn, normalized's shared reciprocal, div_fast_unit) against IEEE '/' on operand
// pairs drawn from a hash
// of the pair index (first + i): raw bit patterns (every class: zeros, denormals, infinities, NaNs), divisors on both
// edges of [2^-40, 2^100] (a few ulps either side), quotients on both edges of [2^-60, 2^60], zero and denormal
// numerators, powers of two.  counts[0] += quotients whose bits differ from '/' (two NaNs compare equal), counts[1] +=
// quotients that took the fast path, counts[2] += quotients checked.
__device__ __forceinline__ uint32_t kat_mix(uint64_t x)
{
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float kat_float(uint32_t sign, int32_t e, uint32_t mant)  // +-2^e (1 + mant 2^-23), e normal
{
  return __uint_as_float((sign & 1u) << 31 | (uint32_t)(e + 127) << 23 | (mant & 0x7FFFFFu));
}
__device__ __forceinline__ bool kat_same(float x, float y)
{
  return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}
__global__ __launch_bounds__(kKatThreads) void kat_div(uint64_t first, uint32_t n, unsigned long long *counts)
{
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  uint32_t bad = 0, fast = 0, seen = 0;
  if (i < n)
  {
    const uint64_t k = first + i;
    const uint32_t h0 = kat_mix(k), h1 = kat_mix(k ^ 0x9E3779B97F4A7C15ull), h2 = kat_mix(k * 3 + 1);
    float a, b;
    switch (h0 & 7u)
    {
      case 0: a = __uint_as_float(h1); b = __uint_as_float(h2); break;
      case 1:  // divisor over [2^-45, 2^105], quotient exponent over [-66, 66]: both edges of both bounds
      {
        b = kat_float(h1 >> 31, (int32_t)(h1 % 151u) - 45, h2);
        a = b * kat_float(h2 >> 31, (int32_t)((h0 >> 3) % 133u) - 66, h1 >> 5);
        break;
      }
      case 2:  // divisor within 3 ulps of 2^-40 / 2^100, quotient near 2^-60 / 2^60 / 1
      {
        const float edge = (h1 & 1u) ? 0x1p100f : 0x1p-40f;
        b = __uint_as_float(__float_as_uint(edge) + (int32_t)((h1 >> 1) % 7u) - 3) * ((h1 & 2u) ? -1.0f : 1.0f);
        const int32_t qe = (h2 % 3u == 0) ? -60 : (h2 % 3u == 1) ? 60 : 0;
        a = b * kat_float(h2 >> 31, qe + (int32_t)((h2 >> 2) % 5u) - 2, h0 >> 3);
        break;
      }
      case 3:  // zero, denormal and tiny numerators
      {
        const uint32_t m = h1 % 3u;
        a = m == 0 ? ((h1 & 8u) ? -0.0f : 0.0f) : m == 1 ? __uint_as_float((h1 & 0x807FFFFFu)) : kat_float(h1 >> 31, -126 + (int32_t)(h2 % 40u), h2);
        b = kat_float(h2 >> 31, (int32_t)(h0 % 141u) - 40, h1 >> 3);
        break;
      }
      case 4: b = kat_float(h1 >> 31, (int32_t)((h1 >> 1) % 3u) - 1, h2); a = kat_float(h2 >> 31, (int32_t)(h0 % 253u) - 126, h1 >> 4); break;
      case 5: a = kat_float(h1 >> 31, (int32_t)(h0 % 253u) - 126, h2); b = kat_float(h2 >> 31, (int32_t)(h1 % 253u) - 126, h0); break;
      case 6: b = kat_float(h1 >> 31, (int32_t)(h0 % 141u) - 40, h2); a = b * __uint_as_float(0x3f800000u + (h2 & 0xFu) - 8u); break;
      default: b = kat_float(h1 >> 31, (int32_t)(h0 % 253u) - 126, 0u); a = kat_float(h2 >> 31, (int32_t)(h1 % 253u) - 126, h2 >> 1); break;
    }
    const float q = div_rn(a, b);
    bool ok;
    (void)div_fast(a, div_prep(b), ok);
    // the normalize form (one reciprocal of the length, one range compare per component) on (a, a2, a3)
    const float a2 = __uint_as_float(__float_as_uint(a) ^ (h2 & 0x807F0000u)), a3 = b * -0.5f;
    const v3 v = mk(a, a2, a3), nv = normalized(v);
    const float l = len(v);
    const bool sv = l > kVerySmall;  // Vector3.cpp:63-72 divides only then
    const float rx = sv ? v.x / l : v.x, ry = sv ? v.y / l : v.y, rz = sv ? v.z / l : v.z;
    // the skybox form: a component over the largest one (|p| <= den, den = |b| + VERY_SMALL_NUMBER)
    const float den = fabsf(b) + kVerySmall, p = fabsf(a) <= den ? a : copysignf(den, a) * 0.75f;
    bool okp;
    float pd = div_fast_unit(p, den, rcp_refined(den), okp);
    const bool unit_ok = den <= 0x1p64f;  // div_fast_unit's precondition (the skybox's den is at most 1 + 2^-63)
    if (!okp) pd = p / den;
    bad = (kat_same(q, a / b) ? 0u : 1u) + (kat_same(nv.x, rx) ? 0u : 1u) + (kat_same(nv.y, ry) ? 0u : 1u) +
          (kat_same(nv.z, rz) ? 0u : 1u) + (!unit_ok || kat_same(pd, p / den) ? 0u : 1u);
    fast = ok ? 1u : 0u;
    seen = 5;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
  {
    bad += __shfl_xor(bad, o, 64);
    fast += __shfl_xor(fast, o, 64);
    seen += __shfl_xor(seen, o, 64);
  }
  if ((threadIdx.x & 63u) == 0 && seen)
  {
    if (bad) atomicAdd(&counts[0], (unsigned long long)bad);
    atomicAdd(&counts[1], (unsigned long long)fast);
    atomicAdd(&counts[2], (unsigned long long)seen);
  }
}

// The kernel-argument layout the bounce loops read through the kernarg segment pointer (rfx_trace.h launder_scene,
// kernarg_params): the laundered DevScene and FrameParams against the by-value arguments, word by word.  out[0] / out[1]:
// words of the DevScene / FrameParams that differ (0 expected), out[2]: 1 when the build reads the record laundered.
// kat_kernarg_swapped takes the arguments the other way round -- what a kernel with a swapped signature would read --
// so the test can show the check catches it.
template <bool SWAPPED>
__device__ __forceinline__ void kernarg_compare(const DevScene &S, const FrameParams &P, uint32_t *out)
{
  const uint32_t *ps = (const uint32_t *)&P, *qs = (const uint32_t *)&kernarg_params();
  uint32_t bad_p = 0, bad_s = 0;
  for (size_t i = 0; i < sizeof(FrameParams) / 4; ++i) bad_p += ps[i] != qs[i] ? 1u : 0u;
#ifdef RFX_LAUNDER_SCENE
  const uint32_t *a = (const uint32_t *)&S, *b = (const uint32_t *)&launder_scene<true>(S);
  for (size_t i = 0; i < sizeof(DevScene) / 4; ++i) bad_s += a[i] != b[i] ? 1u : 0u;
  out[2] = 1;
#else
  out[2] = 0;
#endif
  out[0] = bad_s;
  out[1] = bad_p;
}
__global__ void kat_kernarg(DevScene S, FrameParams P, uint32_t *out)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) kernarg_compare<false>(S, P, out);
}
__global__ void kat_kernarg_swapped(FrameParams P, DevScene S, uint32_t *out)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) kernarg_compare<true>(S, P, out);
}

// Color::argb (Color.cpp:114-117) as the epilogue evaluates it: rgb n x 3 -> out n
__global__ __launch_bounds__(kKatThreads) void kat_argb(const float *rgb, uint32_t n, uint32_t *out)
{
  const uint32_t i = blockIdx.x * kKatThreads + threadIdx.x;
  if (i < n) out[i] = argb(mkc(rgb[3 * (size_t)i], rgb[3 * (size_t)i + 1], rgb[3 * (size_t)i + 2]));
}

}  // namespace rfx



// ------------------------------------------------------------- launchers (library-internal)
namespace rfx {

uint64_t rng_blocks_for(uint64_t traces)
{
  // >= 2x the expected 1.91 triples per trace, plus slack; the scan flags a short stream
  const uint64_t triples = 2 * traces + 65536;
  return (triples + kTriplesPerBlock - 1) / kTriplesPerBlock;
}

// the jump table rng_count / rng_emit expect: (A, C) of 3*16*tid draws for tid < 256, then of
// 3*16*256*b draws for b < nblk (affine LCG maps s -> A s + C, trace_math.h:36)
void rng_jump_table(uint64_t nblk, uint32_t *out)
{
  uint32_t a1 = 1u, c1 = 0u;  // one thread's 48 draws
  for (int i = 0; i < 3 * kTriplesPerThread; ++i) { c1 = 214013u * c1 + 2531011u; a1 = 214013u * a1; }
  uint32_t A = 1u, C = 0u;
  for (int t = 0; t < kRngBlock; ++t)
  {
    out[2 * t] = A; out[2 * t + 1] = C;
    C = a1 * C + c1; A = a1 * A;            // compose one more thread stride
  }
  const uint32_t ab = A, cb = C;            // one block's 48 * 256 draws
  A = 1u; C = 0u;
  for (uint64_t b = 0; b < nblk; ++b)
  {
    out[2 * (kRngBlock + b)] = A; out[2 * (kRngBlock + b) + 1] = C;
    C = ab * C + cb; A = ab * A;
  }
}

// first half of the pre-pass: accept counts of blocks [blk0, blk0 + nblk_slice)
hipError_t launch_rng_count(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_blk_cnt, uint64_t blk0,
                            uint64_t nblk_slice, uint16_t *d_masks, hipStream_t st)
{
  if (nblk_slice)
    hipLaunchKernelGGL(rng_count, dim3((uint32_t)nblk_slice), dim3(kRngBlock), 0, st, d_seed, d_jump, d_blk_cnt, blk0,
                       d_masks);
  return hipGetLastError();
}

// second half: scan all nblk counts, scatter the randDirs this rank needs, carry the stream state
hipError_t launch_rng_finish(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed,
                             const uint32_t *d_blk_cnt, const uint16_t *d_masks, uint64_t nblk, uint64_t traces,
                             uint32_t *d_rd_state, int *d_err, uint64_t ss2, uint64_t W, uint32_t row_block,
                             uint32_t rank, uint32_t nranks, hipStream_t st)
{
  const EmitFilter flt{ss2 ? ss2 : 1, W ? W : 1, row_block ? row_block : 1, rank, nranks ? nranks : 1, 0, UINT64_MAX};
  hipLaunchKernelGGL(rng_emit, dim3((uint32_t)nblk), dim3(kRngBlock), 0, st, d_seed, d_jump, d_blk_cnt, d_masks,
                     traces, d_rd_state, d_next_seed, d_err, flt);
  return hipGetLastError();
}

// the band partition's emit: traces [lo, hi) (and the frame's last trace's stream state); scratch: nblk offsets,
// 3 range words and one word per tile of kScanTileCounts blocks (d_tile_sum; null: the one-workgroup scan).  Also the one-device emit of launches with many blocks (lo = 0, hi = traces, the count kernel's
// accept flags in d_masks): rng_emit's per-block prefix sums cost O(nblk^2) reads, this scan O(nblk).
#ifndef RFX_SCAN_TILES
#define RFX_SCAN_TILES 2  // launches of at least this many tiles of kScanTileCounts blocks scan in many workgroups (0: never)
#endif
hipError_t launch_rng_finish_band(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed,
                                  const uint32_t *d_blk_cnt, const uint16_t *d_masks, uint64_t nblk, uint64_t traces,
                                  uint32_t *d_rd_state, int *d_err, uint64_t lo, uint64_t hi, uint64_t *d_off,
                                  uint32_t *d_range, uint32_t *d_tile_sum, hipStream_t st)
{
  const EmitFilter flt{1, 1, 1, 0, 1, lo, hi};
  const uint64_t ntiles = (nblk + kScanTileCounts - 1) / kScanTileCounts;
  if (RFX_SCAN_TILES && ntiles >= RFX_SCAN_TILES && d_tile_sum)
  {
    hipLaunchKernelGGL(rng_tile_sums, dim3((uint32_t)ntiles), dim3(kTileSumThreads), 0, st, d_blk_cnt, nblk, d_tile_sum,
                       d_range);
    hipLaunchKernelGGL(rng_tile_scan, dim3((uint32_t)ntiles), dim3(kScanThreads), 0, st, d_blk_cnt, nblk, traces, lo, hi,
                       (const uint32_t *)d_tile_sum, d_off, d_range, d_err);
  }
  else
    hipLaunchKernelGGL(rng_band_range, dim3(1), dim3(kScanThreads), 0, st, d_blk_cnt, nblk, traces, lo, hi, d_off,
                       d_range, d_err);
  // about (hi - lo) / (accept rate pi/6 x 4096) blocks hold the band; the workgroups loop over however many there are
  const uint64_t est = (hi - lo) / 2048 + 4;
  hipLaunchKernelGGL(rng_emit_band, dim3((uint32_t)std::min<uint64_t>(est, nblk)), dim3(kRngBlock), 0, st, d_seed, d_jump,
                     d_blk_cnt, d_masks, (const uint64_t *)d_off, (const uint32_t *)d_range, nblk, traces, d_rd_state,
                     d_next_seed, flt);
  return hipGetLastError();
}

// the one-pass pre-pass of a one-device launch (rng_fused); status: nblk words, ticket: one word, both zeroed once at
// allocation; base: the tickets earlier launches took; epoch: this launch's tag, distinct from every earlier launch's on
// the same status array since it was last cleared (never 0)
hipError_t launch_rng_fused(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed, uint64_t nblk,
                            uint64_t traces, uint32_t *d_rd_state, int *d_err, unsigned long long *d_status,
                            unsigned long long *d_ticket, unsigned long long base, uint32_t epoch, hipStream_t st)
{
  hipLaunchKernelGGL(rng_fused, dim3((uint32_t)nblk), dim3(kRngBlock), 0, st, d_seed, d_jump, (uint32_t)nblk, traces,
                     d_rd_state, d_next_seed, d_err, d_status, d_ticket, base, epoch);
  return hipGetLastError();
}

static void launch_mode_cfg(bool stats, int mode, int cfg, dim3 grid, const DevScene &S, const FrameParams &P,
                            hipStream_t st)
{
  if (mode == kModeBlock) (stats ? launch_trace_block_stats : launch_trace_block_fast)(cfg, grid, S, P, st);
  else if (mode == kModePlain)
  {
    if (stats) launch_trace_plain_stats(cfg, grid, S, P, st);
    else if (P.park_after > 0) launch_trace_plain_park(cfg, grid, S, P, st);
    else launch_trace_plain_fast(cfg, grid, S, P, st);
  }
  else if (mode == kModeSsaaLanes) (stats ? launch_trace_lanes_stats : launch_trace_lanes_fast)(cfg, grid, S, P, st);
  else if (mode == kModeSsaaChunks) (stats ? launch_trace_chunks_stats : launch_trace_chunks_fast)(cfg, grid, S, P, st);
  else (stats ? launch_trace_ssaa_stats : launch_trace_ssaa_fast)(cfg, grid, S, P, st);
}

static dim3 kat_grid(uint32_t n) { return dim3((n + kKatThreads - 1) / kKatThreads); }

hipError_t launch_kat_kernarg(const DevScene &S, const FrameParams &P, int swapped, uint32_t *out, hipStream_t st)
{
  if (swapped) hipLaunchKernelGGL(kat_kernarg_swapped, dim3(1), dim3(64), 0, st, P, S, out);
  else hipLaunchKernelGGL(kat_kernarg, dim3(1), dim3(64), 0, st, S, P, out);
  return hipGetLastError();
}

hipError_t launch_kat(int what, const DevScene &S, int tex, const void *in, const int32_t *objs, uint32_t n, void *out,
                      hipStream_t st)
{
  if (!n) return hipSuccess;
  switch (what)
  {
    case 0: hipLaunchKernelGGL(kat_objects, kat_grid(n), dim3(kKatThreads), 0, st, S, (const float *)in, objs, n, (float *)out); break;
    case 1: hipLaunchKernelGGL(kat_texels, kat_grid(n), dim3(kKatThreads), 0, st, S, tex, (const float *)in, n, (float *)out); break;
    case 2: hipLaunchKernelGGL(kat_powf, kat_grid(n), dim3(kKatThreads), 0, st, (const float *)in, n, (float *)out); break;
    default: hipLaunchKernelGGL(kat_argb, kat_grid(n), dim3(kKatThreads), 0, st, (const float *)in, n, (uint32_t *)out); break;
  }
  return hipGetLastError();
}

hipError_t launch_kat_div(uint64_t first, uint32_t n, unsigned long long *counts, hipStream_t st)
{
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(kat_div, kat_grid(n), dim3(kKatThreads), 0, st, first, n, counts);
  return hipGetLastError();
}

hipError_t launch_kat_powf_cube(uint32_t first, uint32_t n, unsigned long long *counts, hipStream_t st)
{
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(kat_powf_cube, kat_grid(n), dim3(kKatThreads), 0, st, first, n, counts);
  return hipGetLastError();
}

#ifndef RFX_NOCULL_MAX_TILES
#define RFX_NOCULL_MAX_TILES 0
#endif

// the mode of a trace launch (rfx_trace.h TraceMode)
static int trace_mode(const FrameParams &P)
{
  if (P.ss < 0) return kModeBlock;
  if (P.ss == 1 && !P.additive && !P.accumulate) return kModePlain;
  if (!RFX_SSAA_LANES || !ss_lane_block(P.ss)) return kModeSsaa;
  return P.ss > 8 ? kModeSsaaChunks : kModeSsaaLanes;
}

static dim3 trace_grid(const FrameParams &P)
{
  const int mode = trace_mode(P);
  if (mode == kModeSsaaLanes || mode == kModeSsaaChunks)  // waves of bw x bw pixels (their samples in the lanes), two
  {                                                       // side by side
    const uint32_t bw = ss_lane_block(P.ss);
    return dim3((P.W + kTileWavesX * bw - 1) / (kTileWavesX * bw), (P.grid_rows + kTileWavesY * bw - 1) / (kTileWavesY * bw));
  }
  const uint32_t cols = P.ss < 0 ? (P.W + (uint32_t)(-P.ss) - 1) / (uint32_t)(-P.ss) : P.W;
  return dim3((cols + kTileW - 1) / kTileW, (P.grid_rows + kTileH - 1) / kTileH);
}

// workgroups (tiles) of the frame's trace launch
uint32_t trace_tiles(const FrameParams &P)
{
  const dim3 g = trace_grid(P);
  return kWgWaves * g.x * g.y;
}

// the frame runs kModeSsaaLanes (its per-view masks are prim_cull_kernel<., true>'s)
bool trace_lanes(const FrameParams &P)
{
  return trace_mode(P) == kModeSsaaLanes;
}

// the frame runs kModeSsaaChunks (one pixel per wave; its per-view masks are prim_cull_kernel<., true>'s closest-hit
// masks over the pixel's sample rectangle)
bool trace_chunks(const FrameParams &P)
{
  return trace_mode(P) == kModeSsaaChunks;
}

// the per-view masks of a small scene's plain or SSAA frame (prim_cull_kernel, kPrimStride words per wave tile), or
// a large scene's chunk lists (prim_cull_large_kernel, kPrimLargeStride words)
hipError_t launch_prim_cull(const DevScene &S, const FrameParams &P, uint64_t *masks, hipStream_t st)
{
  const dim3 grid = trace_grid(P);
  if (!(S.n_sph <= 32 && S.n_tri <= 32))  // large scenes: the primary bundles' chunk lists
    hipLaunchKernelGGL(prim_cull_large_kernel<0>, grid, dim3(kWgThreads), 0, st, S, P, masks);
  else if (trace_lanes(P) || trace_chunks(P))
  {
    if (S.n_pln > 0)
      hipLaunchKernelGGL((prim_cull_kernel<true, true>), grid, dim3(kWgThreads), 0, st, S, P, masks);
    else
      hipLaunchKernelGGL((prim_cull_kernel<false, true>), grid, dim3(kWgThreads), 0, st, S, P, masks);
  }
  else if (S.n_pln > 0)
    hipLaunchKernelGGL(prim_cull_kernel<true>, grid, dim3(kWgThreads), 0, st, S, P, masks);
  else
    hipLaunchKernelGGL(prim_cull_kernel<false>, grid, dim3(kWgThreads), 0, st, S, P, masks);
  return hipGetLastError();
}

hipError_t launch_trace(const DevScene &S, const FrameParams &P, bool stats, hipStream_t st)
{
  const dim3 grid = trace_grid(P);
  FrameParams Pt = P;
  Pt.tiles_x = kTileWavesX * grid.x;  // wave tiles per row (the schedule's unit)
  const int mode = trace_mode(P);
  // the stats build counts the reference's every test, so it never culls.  RFX_NOCULL_MAX_TILES (experiment): small
  // scenes in frames of at most that many wave tiles -- all waves resident at once, the launch as long as its slowest
  // tile -- skip the bundle cull, trading tests for the cull's serial latency
  const bool cull = !stats && !(RFX_NOCULL_MAX_TILES > 0 && S.n_sph <= 32 && S.n_tri <= 32 &&
                                trace_tiles(P) <= (uint32_t)RFX_NOCULL_MAX_TILES);
  const int cfg = (S.n_light > 32 ? kCfgManyLights : 0) | (cull ? kCfgCull : 0) |
                  (S.n_sph <= 32 && S.n_tri <= 32 ? kCfgSmall : 0) | (S.n_pln > 0 ? kCfgPlanes : 0) |
                  (S.n_light == 1 && !stats && RFX_ONE_LIGHT ? kCfgOneLight : 0);
  launch_mode_cfg(stats, mode, cfg, grid, S, Pt, st);
  return hipGetLastError();
}

}  // namespace rfx
