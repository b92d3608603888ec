// rfx_trace.h -- device code of ReflaxMan's per-pixel trace loop for gfx950, shared by the kernel TUs
// (rfx_kernels.hip: RNG pre-pass, tile schedule, known-answer kernels; rfx_trace_<mode>_<stats>.hip: one
// trace_kernel family each, compiled in parallel).
//
//   rng_count / rng_emit : the reference's serial LCG stream
//       (trace_math.h:34-39, Vector3.cpp:176-188) as a parallel pre-pass:
//       LCG jump-ahead per thread, accept flags, block scan, scatter of the
//       i-th accepted triple to trace i.
//   trace_kernel<STATS, BLOCK> : Render::renderNext (Render.cpp:136-215) +
//       Scene::trace (Scene.cpp:73-236), one lane per trace, 8x8-pixel wave
//       tiles, the bounce "recursion" as the reference's own iterative loop.
//       Scene arrays are walked in wave-uniform order (scalar loads);
//       closest hit keeps only (dist, object, t, u, v) per candidate and
//       re-derives drop/normal/reflection/texel for the winner with the same
//       expressions; the shadow any-hit loop exits per lane on the first
//       occluder and per wave once every lane has (exec-mask early out).
//
// Numerics: compiled with -ffp-contract=off, IEEE div/sqrt, f32 denormals on,
// so every operation rounds exactly as the reference's x86-64 build does.
// Work the reference does but whose result cannot matter is skipped only
// where the skip is provably exact (each site says why).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <type_traits>

#include "rfx_math.h"
#include "rfx_powf.h"
#include "rfx_types.h"

#pragma clang fp contract(off)

namespace rfx {

struct Cnt { uint32_t c[C_COUNT]; };

#define RFX_CNT(k)                   \
  do {                               \
    if constexpr (STATS) cnt.c[k]++; \
  } while (0)

// Diagnostic build only (RFX_DEBUG_PROF, tools/regionprof.py): wave clock cycles spent per region of
// the bounce segment, summed by each region's first active lane into a device-global table.
#ifdef RFX_DEBUG_PROF
enum ProfRegion { P_SPH = 0, P_TRI, P_WIN, P_LIGHT, P_SHADOW, P_MAT, P_SKY, P_SEG, P_COUNT };
static __device__ unsigned long long g_prof[2 * P_COUNT];  // cycles, then wave executions (per TU)
__shared__ unsigned long long s_prof[2 * P_COUNT];  // per workgroup, flushed to g_prof at kernel end
#define RFX_PROF_BEGIN(k) const uint64_t prof_t0_##k = __builtin_amdgcn_s_memtime()
#define RFX_PROF_END(k)                                                                   \
  do {                                                                                    \
    const uint64_t dt_ = __builtin_amdgcn_s_memtime() - prof_t0_##k;                     \
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)__ballot(1)) - 1))           \
    {                                                                                     \
      atomicAdd(&s_prof[k], (unsigned long long)dt_);                                     \
      atomicAdd(&s_prof[P_COUNT + k], 1ull);                                              \
    }                                                                                     \
  } while (0)
// cull statistics (diagnostic build): per bundle kind (0 closest hit, 1 shadow): bundles, usable bundles,
// live lanes, kept sphere pairs, kept triangles, valid pairs, valid triangles
static __device__ unsigned long long g_cull[32];
// large scenes (kind 2 closest hit, 3 shadow): bundles, usable bundles, live lanes, kept chunks, kept spheres,
// pair tests run
#define RFX_CULL_STAT_LARGE(kind, ok, live_mask, chunks, spheres, pairs)                            \
  do {                                                                                              \
    if ((threadIdx.x & 63u) == 0u)                                                                  \
    {                                                                                               \
      atomicAdd(&g_cull[8 * (kind) + 0], 1ull);                                                     \
      atomicAdd(&g_cull[8 * (kind) + 1], (ok) ? 1ull : 0ull);                                       \
      atomicAdd(&g_cull[8 * (kind) + 2], (unsigned long long)__popcll(live_mask));                 \
      atomicAdd(&g_cull[8 * (kind) + 3], (unsigned long long)(chunks));                            \
      atomicAdd(&g_cull[8 * (kind) + 4], (unsigned long long)(spheres));                           \
      atomicAdd(&g_cull[8 * (kind) + 5], (unsigned long long)(pairs));                             \
    }                                                                                               \
  } while (0)
#define RFX_CULL_STAT(kind, ok, live_mask, om, valid)                                                 \
  do {                                                                                              \
    if ((threadIdx.x & 63u) == 0u)                                                                  \
    {                                                                                               \
      atomicAdd(&g_cull[8 * (kind) + 0], 1ull);                                                     \
      atomicAdd(&g_cull[8 * (kind) + 1], (ok) ? 1ull : 0ull);                                       \
      atomicAdd(&g_cull[8 * (kind) + 2], (unsigned long long)__popcll(live_mask));                 \
      atomicAdd(&g_cull[8 * (kind) + 3], (unsigned long long)__popc(small_pairs(om)));             \
      atomicAdd(&g_cull[8 * (kind) + 4], (unsigned long long)__popcll(small_tris(om)));            \
      atomicAdd(&g_cull[8 * (kind) + 5], (unsigned long long)__popc(small_pairs(valid)));          \
      atomicAdd(&g_cull[8 * (kind) + 6], (unsigned long long)__popcll(small_tris(valid)));         \
    }                                                                                               \
  } while (0)
#define RFX_PROF_INIT()                                          \
  do {                                                           \
    if (threadIdx.x < 2 * P_COUNT) s_prof[threadIdx.x] = 0ull;   \
  } while (0)
#define RFX_PROF_FLUSH()                                                            \
  do {                                                                              \
    __syncthreads();                                                                \
    if (threadIdx.x < 2 * P_COUNT) atomicAdd(&g_prof[threadIdx.x], s_prof[threadIdx.x]); \
  } while (0)
#else
#define RFX_PROF_INIT() \
  do {                  \
  } while (0)
#define RFX_PROF_FLUSH() \
  do {                   \
  } while (0)
#define RFX_PROF_BEGIN(k) \
  do {                    \
  } while (0)
#define RFX_PROF_END(k) \
  do {                  \
  } while (0)
#define RFX_CULL_STAT(kind, ok, live_mask, om, valid) \
  do {                                                \
  } while (0)
#define RFX_CULL_STAT_LARGE(kind, ok, live_mask, chunks, spheres, pairs) \
  do {                                                                   \
  } while (0)
#endif

// Color(ARGB) (Color.cpp:9-14) through a 256-entry LDS table of float(k) / 255.0f:
// the table holds exactly the quotients the reference computes per channel.
__device__ __forceinline__ col from_argb_lut(uint32_t c, const float *lut)
{
  return mkc(lut[(c >> 16) & 0xFFu], lut[(c >> 8) & 0xFFu], lut[c & 0xFFu]);
}

// glibc powf's tables (rfx_powf.h) copied to LDS by each workgroup: the lookups index them per lane,
// and LDS answers such gathers in ~100 cycles where the constant/global path takes several hundred.
__shared__ double s_powf_log[16][2];
__shared__ uint64_t s_powf_exp[32];
__shared__ double s_powf_add[2][4];

__device__ __forceinline__ void stage_powf_tables()
{
  const uint32_t t = threadIdx.x;
  if (t < 32)
  {
    s_powf_exp[t] = kExp2fTab[t];
    s_powf_log[t >> 1][t & 1u] = kPowfLog2Tab[t >> 1][t & 1u];
    if (t < 8) s_powf_add[t >> 2][t & 3u] = kPowfAdd[t >> 2][t & 3u];
  }
}

__device__ __forceinline__ float powf_dev(float x, float y)
{
  return powf_glibc_t(x, y, s_powf_log, s_powf_exp, s_powf_add);
}

// powf(x, 3) for x in [0, 1] (the Fresnel term): the double cube where it provably rounds like glibc, glibc's
// algorithm for the few lanes where it may not (rfx_powf.h powf_cube_fast)
__device__ __forceinline__ float powf3_dev(float x)
{
  float p;
  if (!powf_cube_fast(x, p)) p = powf_dev(x, 3.0f);
  return p;
}

// Small scenes (<= 32 spheres, <= 32 triangles): the per-object records the hit lanes gather by their
// own object index (winner geometry and material, the cull lane table) staged in LDS per workgroup.
__shared__ SphereGeo s_sph_geo[32];
__shared__ MatRec s_sph_mat[32];
__shared__ int32_t s_sph_info[64];
__shared__ TriShade s_tri_shade[32];
__shared__ MatRec s_tri_mat[32];
__shared__ CullRec s_cull[64];

template <bool SMALL>
struct Tabs {
  const DevScene &S;
  __device__ __forceinline__ SphereGeo sph_geo(int i) const { return S.sph_geo[i]; }
  __device__ __forceinline__ MatRec sph_mat(int i) const { return S.sph_mat[i]; }
  __device__ __forceinline__ int32_t sph_info(int k) const { return S.sph_info[k]; }
  __device__ __forceinline__ TriShade tri_shade(int i) const { return S.tri_shade[i]; }
  __device__ __forceinline__ MatRec tri_mat(int i) const { return S.tri_mat[i]; }
  __device__ __forceinline__ const CullRec *cull() const { return S.cull_small; }
};
template <>
struct Tabs<true> {
  const DevScene &S;
  __device__ __forceinline__ SphereGeo sph_geo(int i) const { return s_sph_geo[i]; }
  __device__ __forceinline__ MatRec sph_mat(int i) const { return s_sph_mat[i]; }
  __device__ __forceinline__ int32_t sph_info(int k) const { return s_sph_info[k]; }
  __device__ __forceinline__ TriShade tri_shade(int i) const { return s_tri_shade[i]; }
  __device__ __forceinline__ MatRec tri_mat(int i) const { return s_tri_mat[i]; }
  __device__ __forceinline__ const CullRec *cull() const { return s_cull; }
};

__device__ __forceinline__ void stage_small_scene(const DevScene &S)
{
  const int t = (int)threadIdx.x;
  if (t < S.n_sph)
  {
    s_sph_geo[t] = S.sph_geo[t];
    s_sph_mat[t] = S.sph_mat[t];
    s_sph_info[2 * t] = S.sph_info[2 * t];
    s_sph_info[2 * t + 1] = S.sph_info[2 * t + 1];
  }
  if (t < S.n_tri)
  {
    s_tri_shade[t] = S.tri_shade[t];
    s_tri_mat[t] = S.tri_mat[t];
  }
  if (t < 64) s_cull[t] = S.cull_small[t];
}

// 7 waves per SIMD (<= 72 VGPRs, a few spills): the kernel is VALU-issue bound; more waves hide the
// scene-load and texel latencies better than spills cost (tools/ab.py, C3 trace kernel: 6 -> 7 -2.6%;
// 8 waves / 64 VGPRs spill enough to lose 4-7%)
#ifndef RFX_WAVES_PER_EU
#define RFX_WAVES_PER_EU 7
#endif
// waves per workgroup (1, 2 or 4): a wave is an 8x8 pixel tile, a workgroup 8x8 / 16x8 / 16x16 pixels.
// Two: a workgroup's slots free when its slower wave ends, and the per-workgroup LDS staging stays cheap
// (tools/ab.py, C3 trace kernel: 4 -> 2 waves -2.5%, 1 wave +3.6%)
#ifndef RFX_WG_WAVES
#define RFX_WG_WAVES 2
#endif
constexpr uint32_t kWgWaves = RFX_WG_WAVES, kWgThreads = 64 * kWgWaves;
constexpr uint32_t kTileWavesX = kWgWaves >= 2 ? 2 : 1, kTileWavesY = kWgWaves / kTileWavesX;
constexpr uint32_t kTileW = 8 * kTileWavesX, kTileH = 8 * kTileWavesY;
static_assert(kWgWaves == 1 || kWgWaves == 2 || kWgWaves == 4, "RFX_WG_WAVES: 1, 2 or 4");
#define RFX_TRACE_BOUNDS __launch_bounds__(kWgThreads) __attribute__((amdgpu_waves_per_eu(RFX_WAVES_PER_EU)))

// ------------------------------------------------------------- sampling
template <bool STATS>
__device__ __forceinline__ col texel_uv(const DevScene &S, int tex, float u, float v, const float *lut, Cnt &cnt)
{                                                                         // Texture.cpp:231-269
  if (u < 0.0f || u > 1.0f || v < 0.0f || v > 1.0f) { RFX_CNT(C_TEX_OTHER); return mkc(0.0f, 0.0f, 0.0f); }
  TexRec t;
  t.w = 0; t.h = 0; t.offset = 0;
  if (tex >= 0) t = S.texs[tex];
  if (t.w == 0)
  {
    RFX_CNT(C_TEX_CHECKER);
    return (((int)(u * 50) % 2) ^ ((int)(v * 50) % 2)) ? mkc(0.5f, 0.5f, 0.5f) : mkc(0.75f, 0.75f, 0.75f);
  }
  const float fx = clampf(u, 0.0f, 1.0f - kFltEpsilon) * (float)t.w;
  const float fy = clampf(v, 0.0f, 1.0f - kFltEpsilon) * (float)t.h;
  const uint32_t x = (uint32_t)fx, y = (uint32_t)fy;
  const uint32_t *px = S.texels + t.offset;
  if (x < t.w - 1 && y < t.h - 1)
  {
    RFX_CNT(C_TEX_BILINEAR);
    const col c00 = from_argb_lut(px[x + t.w * y], lut), c01 = from_argb_lut(px[x + t.w * (y + 1)], lut);
    const col c10 = from_argb_lut(px[x + 1 + t.w * y], lut), c11 = from_argb_lut(px[x + 1 + t.w * (y + 1)], lut);
    const float uf = fx - floorf(fx), vf = fy - floorf(fy);
    const float uo = 1 - uf, vo = 1 - vf;
    return cadd(cscale(cadd(cscale(c00, uo), cscale(c10, uf)), vo), cscale(cadd(cscale(c01, uo), cscale(c11, uf)), vf));
  }
  RFX_CNT(C_TEX_OTHER);
  const uint32_t xi = (uint32_t)fx, yi = (uint32_t)fy;                 // Texture.cpp:216-229
  if (xi >= t.w || yi >= t.h) return mkc(0.0f, 0.0f, 0.0f);
  return from_argb_lut(px[xi + t.w * yi], lut);
}

template <bool STATS>
__device__ __forceinline__ col skybox_texel(const DevScene &S, v3 ray, const float *lut, Cnt &cnt)  // Skybox.cpp:39-106
{
  const float uLeft = 1.0f / 8.0f, vLeft = 3.0f / 6.0f;
  const float uFront = 3.0f / 8.0f, vFront = 3.0f / 6.0f;
  const float uRight = 5.0f / 8.0f, vRight = 3.0f / 6.0f;
  const float uBack = 7.0f / 8.0f, vBack = 3.0f / 6.0f;
  const float uTop = 3.0f / 8.0f, vTop = 5.0f / 6.0f;
  const float uBottom = 3.0f / 8.0f, vBottom = 1.0f / 6.0f;
  const float hw = S.half_tile_w, hh = S.half_tile_h;
  const v3 n = normalized(ray);
  const float x = n.x, y = n.y, z = n.z;
  const float ax = fabsf(x) + kVerySmall, ay = fabsf(y) + kVerySmall, az = fabsf(z) + kVerySmall;
  // the face's two quotients share their divisor (rfx_math.h div_fast_unit): u0 -/+ p / den * hw, v0 -/+ q / den * hh
  float u0, v0, p, q, den, su, sv;
  if (az >= ax && az >= ay)
  {
    den = az;
    if (z > 0) { u0 = uFront; v0 = vFront; p = x; q = y; su = 1.0f; sv = 1.0f; }
    else { u0 = uBack; v0 = vBack; p = x; q = y; su = -1.0f; sv = 1.0f; }
  }
  else if (ax >= ay && ax >= az)
  {
    den = ax;
    if (x > 0) { u0 = uRight; v0 = vRight; p = z; q = y; su = -1.0f; sv = 1.0f; }
    else { u0 = uLeft; v0 = vLeft; p = z; q = y; su = 1.0f; sv = 1.0f; }
  }
  else
  {
    den = ay;
    if (y > 0) { u0 = uTop; v0 = vTop; p = x; q = z; su = 1.0f; sv = -1.0f; }
    else { u0 = uBottom; v0 = vBottom; p = x; q = z; su = 1.0f; sv = 1.0f; }
  }
  // den in [2^-63, 1 + 2^-63] and |p|, |q| <= den: div_fast_unit's bounds
  const float rden = rcp_refined(den);
  bool okp, okq;
  float pd = div_fast_unit(p, den, rden, okp), qd = div_fast_unit(q, den, rden, okq);
  if (__builtin_expect(!(okp && okq), 0)) { pd = p / den; qd = q / den; }
  // u0 + p / den * hw, or u0 - (p / den * hw): a subtraction of the product, as the reference writes it
  const float pu = pd * hw, qv = qd * hh;
  const float u = su > 0.0f ? u0 + pu : u0 - pu, v = sv > 0.0f ? v0 + qv : v0 - qv;
  return texel_uv<STATS>(S, S.skybox_tex, u, v, lut, cnt);
}

// A textured triangle's material colour at barycentrics (u, v) (Triangle.cpp:89-96): tuvTrans * (u, v, 0)
// (whose _13 and _23 are 0) offset by (tu[0], tv[0]).
template <bool STATS>
__device__ __forceinline__ col tri_texel(const DevScene &S, const TriShade &sh, float u, float v, const float *lut,
                                         Cnt &cnt)
{
  const float tvx = u * sh.t11 + v * sh.t12 + 0.0f;
  const float tvy = u * sh.t21 + v * sh.t22 + 0.0f;
  return texel_uv<STATS>(S, sh.tex, sh.tu0 + tvx, sh.tv0 + tvy, lut, cnt);
}

// ------------------------------------------------------------- primitives
// Per-ray constants of Sphere::trace (Sphere.cpp:50-52,58), hoisted out of the object loop.
struct RayConst {
  v3 ray2;      // 2.0f * ray
  float a4, a2; // 4.0f * a, 2.0f * a  with a = |ray|^2
  bool a_ok;    // a > VERY_SMALL_NUMBER
  DivRcp a2d;   // the divisor 2a of every sphere's t, its reciprocal shared (rfx_math.h div_prep)
};
__device__ __forceinline__ RayConst ray_const(v3 ray)
{
  RayConst k;
  const float a = sqlen(ray);
  k.ray2 = mul(ray, 2.0f);
  k.a4 = 4.0f * a;
  k.a2 = 2.0f * a;
  k.a_ok = a > kVerySmall;
  k.a2d = div_prep(k.a2);
  return k;
}

// Sphere::trace (Sphere.cpp:44-85) for spheres 2j and 2j+1 at once, up to the discriminant: each half
// of an f2 runs the reference's scalar expressions in the reference's order (vco = o - c,
// b = 2ray . vco, c = |vco|^2 - r^2, d = b*b - 4a*c), so v_pk_* results round exactly as scalar ones.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void pair_bd(const SpherePair &g, v3 o, const RayConst &k, f2 &b, f2 &d)
{
  const f2 vx = o.x - f2{g.cx[0], g.cx[1]};
  const f2 vy = o.y - f2{g.cy[0], g.cy[1]};
  const f2 vz = o.z - f2{g.cz[0], g.cz[1]};
  b = k.ray2.x * vx + k.ray2.y * vy + k.ray2.z * vz;
  const f2 c = vx * vx + vy * vy + vz * vz - f2{g.r2[0], g.r2[1]};
  d = b * b - k.a4 * c;
}

// Can either sphere of a pair hit?  d < 0 misses; so does b >= 0 (or NaN), since then -b - sqrt(d) <= 0
// gives t <= 0, which `t > VERY_SMALL_NUMBER` rejects (Sphere.cpp:58-60) -- both are exact rejects.
__device__ __forceinline__ bool pair_may_hit(f2 b, f2 d)
{
  return (d.x >= 0.0f && b.x < 0.0f) || (d.y >= 0.0f && b.y < 0.0f);
}

// The rest of Sphere::trace for one sphere given its b and d: on a hit returns t and |ray t|^2.
// `(ray * t).length() > DELTA` (Sphere.cpp:61-64) is tested as |ray t|^2 >= kSqDeltaSphere: the same
// decision without the square root (rfx_math.h).
// SEL (large-scene loops): one branch, the rest computed and decided without branching.  tools/ab.py, trace ms: C5
// 3.143 -> 3.067 (-2.4%); the small-scene kernel +9% with it (its SGPR spills 23 -> 51), so the small loops keep the
// early outs.
// The large scenes' sphere loops (SEL) keep '/': the shared reciprocal of 2a, live across the BVH walk, raised the C5
// trace kernel's VGPR spills from 15 to 36 and its time by 5.9% (tools/ab.py, profiles/r06/ab/c5_div_sel_prefetch_r6c.jsonl)
#ifndef RFX_DIV_SEL
#define RFX_DIV_SEL 0
#endif
template <bool STATS, bool SHADOW, bool SEL = false>
__device__ __forceinline__ bool sphere_tail(float b, float d, v3 ray, const RayConst &k, float &t_out,
                                            float &sq_out, Cnt &cnt)
{
  RFX_CNT(SHADOW ? C_SH_SPH_TESTS : C_SPH_TESTS);
  if constexpr (STATS)
    if (!(b > 0.0f)) RFX_CNT(SHADOW ? C_SH_SPH_B : C_SPH_B);
  if constexpr (!STATS && SEL)
  {
    if (!(d >= 0.0f && k.a_ok && b < 0.0f)) return false;
    // (RFX_DIV_SEL 0: the large scenes' BVH loops divide with '/', and the shared reciprocal is not live across the walk)
    const float t = RFX_DIV_SEL ? div_by(-b - sqrt_rn(d), k.a2d) : (-b - sqrt_rn(d)) / k.a2;
    const float sq = sqlen(mul(ray, t));
    t_out = t;
    sq_out = sq;
    return t > kVerySmall && sq >= kSqDeltaSphere;
  }
  if (!(d >= 0.0f && k.a_ok)) return false;
  // b >= 0 (or NaN): -b - sqrt(d) <= 0, so t <= 0 and `t > VERY_SMALL_NUMBER` rejects -- exact early out
  if constexpr (!STATS)
    if (!(b < 0.0f)) return false;
  if constexpr (STATS)
    if (!(b > 0.0f)) RFX_CNT(SHADOW ? C_SH_SPH_D : C_SPH_D);
  const float t = div_by(-b - sqrt_rn(d), k.a2d);
  if (!(t > kVerySmall)) return false;
  RFX_CNT(SHADOW ? C_SH_SPH_T : C_SPH_T);
  const float sq = sqlen(mul(ray, t));
  if (!(sq >= kSqDeltaSphere)) return false;
  t_out = t;
  sq_out = sq;
  return true;
}

// Triangle::trace (Triangle.cpp:53-108) up to its hit decision; on a hit returns t, u, v, |ray t|^2.
// axTrans * (o - v0) and axTrans * ray are evaluated row by row with the reference's expressions: the
// z row first, then -- only for t > VERY_SMALL_NUMBER -- the x and y rows as one packed chain
// ((aox, aoy), (arx, ary), (u, v)), each half rounding exactly as the scalar expression.
// PRE: reject plane crossings outside the triangle before the divide (below).  tools/ab.py, trace ms: large-scene
// shadow rays 3.399 -> 3.327 on C5 (-2.1%); small scenes (C3) +0.6% in either loop, closest hit on C5 0%.
template <bool STATS, bool SHADOW, bool PRE = false>
__device__ __forceinline__ bool tri_hit(const TriGeo &g, v3 o, v3 ray, float &t_out, float &u_out, float &v_out,
                                        float &sq_out, Cnt &cnt, const RayConst &k, float best_sq = INFINITY)
{
  RFX_CNT(SHADOW ? C_SH_TRI_TESTS : C_TRI_TESTS);
  const float dx = o.x - g.v0x, dy = o.y - g.v0y, dz = o.z - g.v0z;
  const float aoz = dx * g.a31 + dy * g.a32 + dz * g.a33;
  const float arz = ray.x * g.a31 + ray.y * g.a32 + ray.z * g.a33;
  if (!(fabsf(arz) > kVerySmall)) return false;
  RFX_CNT(SHADOW ? C_SH_TRI_Z : C_TRI_Z);
  // t = -aoz / arz > VERY_SMALL_NUMBER needs -aoz and arz non-zero with equal signs (event counter only)
  const float nz = -aoz;
  const bool same_sign = (nz > 0.0f && arz > 0.0f) || (nz < 0.0f && arz < 0.0f);
  if constexpr (STATS)
    if (same_sign) RFX_CNT(SHADOW ? C_SH_TRI_S : C_TRI_S);
  // exact reject before the division: with opposite signs or a zero (or NaN) numerator, t <= 0 or NaN,
  // which `t > VERY_SMALL_NUMBER` rejects anyway; the divide is skipped when no lane of the wave needs it
  if (!same_sign) return false;
  if constexpr (!STATS)
  {
    // |ray t|^2 = a nz^2 / arz^2 (real, a2 = 2a exactly).  Within DELTA of the origin (a shadow ray or a reflected
    // ray leaving the triangle it starts on, or its coplanar neighbour: nz ~ 0): the reference's sqDistance, within
    // ~10 ulp of it, is at most DELTA^2 under the 2^-15 margin, so `sqDistance > DELTA * DELTA` fails -- exact reject
    // before the divide (tools/ab.py trace ms: C3 -1.1%, C2 d4 -3.4%, C5 -0.4%).
    const float n2a = nz * nz * k.a2, r2 = arz * arz;
    if (n2a < (2.0f * (kDelta * kDelta)) * r2 * 0.99997f) return false;
    // beyond the current closest hit (closest hit only): a 2^-16 margin over the rounding of both sides leaves
    // |ray t| strictly above the best distance after rounding, so the reference could neither take it nor tie
    if constexpr (!SHADOW)
      if (n2a > best_sq * r2 * 2.0000305f) return false;
  }
  const f2 c1{g.a11, g.a21}, c2{g.a12, g.a22}, c3{g.a13, g.a23};
  f2 ao, ar;
  if constexpr (PRE && !STATS)
  {
    ao = dx * c1 + dy * c2 + dz * c3;                         // (aox, aoy)
    ar = ray.x * c1 + ray.y * c2 + ray.z * c3;                // (arx, ary)
    // exact reject of a plane crossing outside the triangle before the correctly rounded divide: with t' = nz rcp(arz)
    // (v_rcp_f32: 1 ulp), u' = aox + t' arx is within (|aox| + |t' arx|) 2^-19 of the reference's rounded u (t
    // within 2^-21 relative, three roundings); the margins are 4x that, so u' < -mu means u < 0, and u' + v' above
    // 1 + mu + mv means u + v > 1.  A NaN keeps the triangle.  A wave whose lanes all cross outside skips the divide.
    const f2 pp = (nz * __builtin_amdgcn_rcpf(arz)) * ar;
    const f2 uvp = ao + pp;
    const float mu = (fabsf(ao.x) + fabsf(pp.x)) * 0x1p-17f, mv = (fabsf(ao.y) + fabsf(pp.y)) * 0x1p-17f;
    if (uvp.x < -mu || uvp.y < -mv || uvp.x + uvp.y > 1.0f + (mu + mv) + 0x1p-20f) return false;
  }
  const float t = qdiv(nz, arz);
  if (!(t > kVerySmall)) return false;
  RFX_CNT(SHADOW ? C_SH_TRI_T : C_TRI_T);
  if constexpr (!(PRE && !STATS))
  {
    ao = dx * c1 + dy * c2 + dz * c3;                         // (aox, aoy)
    ar = ray.x * c1 + ray.y * c2 + ray.z * c3;                // (arx, ary)
  }
  const f2 uv = ao + t * ar;                                  // (u, v)
  const float u = uv.x, v = uv.y;
  if (!(u >= 0.0f && v >= 0.0f && u + v < 1.0f)) return false;
  RFX_CNT(SHADOW ? C_SH_TRI_IN : C_TRI_IN);
  const float sq = sqlen(mul(ray, t));
  if (!(sq > kDelta * kDelta)) return false;
  t_out = t; u_out = u; v_out = v; sq_out = sq;
  return true;
}

// Plane::trace (Plane.cpp:36-73) up to its hit decision; on a hit returns t and |ray t|^2.  a = norm . ray,
// t = norm . (pos - origin) / a, with tri_hit's two exact rejects before the division (opposite signs or a
// zero numerator give t <= 0; a plane hit beyond the closest hit so far cannot win or tie).
template <bool STATS, bool SHADOW>
__device__ __forceinline__ bool plane_hit(const PlaneGeo &g, v3 o, v3 ray, float &t_out, float &sq_out, Cnt &cnt,
                                          const RayConst &k, float best_sq = INFINITY)
{
  RFX_CNT(SHADOW ? C_SH_PLN_TESTS : C_PLN_TESTS);
  const v3 n = mk(g.nx, g.ny, g.nz);
  const float a = dot(n, ray);                                                     // Plane.cpp:41
  if (!(fabsf(a) > kVerySmall)) return false;
  const float num = dot(n, sub(mk(g.px, g.py, g.pz), o));                          // Plane.cpp:40,45
  if (!((num > 0.0f && a > 0.0f) || (num < 0.0f && a < 0.0f))) return false;
  if constexpr (!SHADOW && !STATS)
    if (num * num * k.a2 > best_sq * (a * a) * 2.0000305f) return false;
  const float t = qdiv(num, a);
  if (!(t > kVerySmall)) return false;
  RFX_CNT(SHADOW ? C_SH_PLN_T : C_PLN_T);
  const float sq = sqlen(mul(ray, t));
  if (!(sq > kDelta * kDelta)) return false;                                       // Plane.cpp:50-53
  t_out = t; sq_out = sq;
  return true;
}

// ------------------------------------------------------------- wave ray bundles (exact culling)
// The live rays of a wave form a bundle: origins within rw of (cx, cy, cz) -- the first live lane's
// origin -- and directions within the half-angle acos(cosa) of that lane's direction (ax, ay, az).
// A ray the reference's float test reports as hitting a sphere passes within r + 1.25e-3 |o - c| of the
// centre (rounding of d = b^2 - 4ac is at most 104 u a |vco|^2, DESIGN.md "Exact work skipping"; observed worst
// 7.6e-5, tests/test_cull_bound.py); kCullRel = 2e-3 covers the bound 1.6 times (round 2 used 4e-3: C5 trace -7%
// with 2e-3, tools/ab.py), so an object whose bounding sphere, grown by rw and kCullRel (L + rw), lies outside the bundle's cone
// is missed by every lane of the wave and its exact test is skipped for the whole wave.  Skipping a test
// that misses changes no result: the closest hit and the any-hit only ever take hits.  Every cull
// decision is a conjunction of comparisons, so a NaN anywhere keeps the object.
constexpr float kCullRel = 2e-3f;

// per-view primary masks (prim_cull_kernel): per wave tile, the closest hit's mask and the shadow masks of the
// first kPrimLights lights
constexpr int kPrimLights = 4, kPrimStride = 1 + kPrimLights;
// Per-view masks of SSAA / additive frames (RFX_PRIM_SSAA) and per-view chunk lists of large scenes (RFX_PRIM_LARGE):
// built, parity-tested and measured slower in round 4 (the screenshot frame +4.3%, C5 +3.3%; interleaved A/B,
// profiles/r04/ab/), so compiled out by default
#ifndef RFX_PRIM_SSAA
#define RFX_PRIM_SSAA 0
#endif
// per-view masks of kModeSsaaLanes frames (sampleNum 1 jittered, 2, 4, 8: the wave's own bw x bw pixels)
#ifndef RFX_PRIM_LANES
#define RFX_PRIM_LANES 1
#endif
#ifndef RFX_PRIM_LARGE
#define RFX_PRIM_LARGE 0
#endif
// Large scenes (prim_cull_large_kernel): per wave tile, the chunk cull of its primary bundle -- [0] the number of kept
// 64-sphere chunks (at most kPrimLargeChunks; kPrimLargeNone: no list, the tile culls per launch), [1] the triangle mask,
// [2] the chunk mask (scenes of at most 64 chunks), [4..] the kept chunks' sphere masks in chunk order
constexpr int kPrimLargeChunks = 8, kPrimLargeStride = 4 + kPrimLargeChunks;
constexpr uint64_t kPrimLargeNone = ~0ull;

struct Bundle {
  float cx, cy, cz, rw;
  float ax, ay, az, cosa, sina;
  bool ok;  // wave-uniform: the bound is finite and the cone narrower than ~84 degrees
};

__device__ __forceinline__ float lane_bcast(float v, int lane)
{
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// max over the wave of a value >= 0 (every lane active): the bit patterns of non-negative floats order
// like the floats, and a NaN pattern (above +inf) wins, which makes the bound unusable below.
// DPP inclusive max-scan within each 16-lane row (row_shr 1, 2, 4, 8), then across rows (row_bcast 15,
// row_bcast 31): lane 63 ends with the wave's maximum.  Lanes a shift leaves without a source keep 0.
__device__ __forceinline__ float wave_max_nonneg(float v)
{
  uint32_t u = __float_as_uint(v);
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, false));  // row_shr:1
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x112, 0xf, 0xf, false));  // row_shr:2
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x114, 0xf, 0xf, false));  // row_shr:4
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x118, 0xf, 0xf, false));  // row_shr:8
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x142, 0xa, 0xf, false));  // row_bcast:15
  u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane((int)u, 63));
}

// Sums of products in the bundle and cull bounds (RFX_CULL_FMA): these are conservative decisions with margins far above
// a rounding, not reference values, so they may fuse their multiply-adds.
#ifndef RFX_CULL_FMA
#define RFX_CULL_FMA 1
#endif
__device__ __forceinline__ float cdot(float ax, float ay, float az, float bx, float by, float bz)
{
#if RFX_CULL_FMA
  return __builtin_fmaf(az, bz, __builtin_fmaf(ay, by, ax * bx));
#else
  return ax * bx + ay * by + az * bz;
#endif
}

// Bundle of the rays (o, d) of the `live` lanes.  Call with every lane of the wave active and at least
// one live lane.  Approximate square roots are fine here: every bound is widened well past their error.
__device__ __forceinline__ Bundle make_bundle(v3 o, v3 d, bool live)
{
  Bundle B;
  const int ref = __ffsll((long long)__ballot(live)) - 1;
  B.cx = lane_bcast(o.x, ref); B.cy = lane_bcast(o.y, ref); B.cz = lane_bcast(o.z, ref);
  const float dx = lane_bcast(d.x, ref), dy = lane_bcast(d.y, ref), dz = lane_bcast(d.z, ref);
  const float inv = __builtin_amdgcn_rsqf(cdot(dx, dy, dz, dx, dy, dz));
  B.ax = dx * inv; B.ay = dy * inv; B.az = dz * inv;
  const float ex = o.x - B.cx, ey = o.y - B.cy, ez = o.z - B.cz;
  const float e2 = cdot(ex, ey, ez, ex, ey, ez);
  const float cosl = cdot(d.x, d.y, d.z, B.ax, B.ay, B.az) * __builtin_amdgcn_rsqf(cdot(d.x, d.y, d.z, d.x, d.y, d.z));
  const float dev = 1.0f - cosl;
  // a live lane with a non-finite or degenerate ray disables the bound for the whole wave
  const bool bad = live && !(e2 <= 1.0e30f && dev >= -0.5f && dev <= 2.5f);
  const float e2m = wave_max_nonneg(live ? e2 : 0.0f);
  const float devm = wave_max_nonneg(live ? fmaxf(dev, 0.0f) : 0.0f);
  B.rw = __builtin_amdgcn_sqrtf(e2m) * 1.0001f;
  B.cosa = 1.0f - devm - 4e-6f;                                                // approximate cosines: widen
  B.sina = __builtin_amdgcn_sqrtf(fmaxf(1.0f - B.cosa * B.cosa, 0.0f) + 1e-7f) * 1.001f;
  B.ok = __ballot(bad) == 0 && B.cosa > 0.1f && B.rw <= 1.0e15f;
  return B;
}

#ifdef RFX_HALF_BUNDLES
// make_bundle for each half of the wave (lanes 0-31, 32-63): the DPP scan's row_bcast:15 step leaves each half's maximum
// in its lane 31 / 63.  A half without a live lane gets ok = false (its lanes test nothing).
__device__ __forceinline__ void make_bundle_halves(v3 o, v3 d, bool live, Bundle (&H)[2])
{
  const uint64_t lm = __ballot(live);
  const bool hi = (threadIdx.x & 63u) >= 32u;
  float ax[2], ay[2], az[2], cx[2], cy[2], cz[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
  {
    const uint64_t hm = lm & (h ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull);
    const int ref = hm ? __ffsll((long long)hm) - 1 : 0;
    cx[h] = lane_bcast(o.x, ref); cy[h] = lane_bcast(o.y, ref); cz[h] = lane_bcast(o.z, ref);
    const float dx = lane_bcast(d.x, ref), dy = lane_bcast(d.y, ref), dz = lane_bcast(d.z, ref);
    const float inv = __builtin_amdgcn_rsqf(dx * dx + dy * dy + dz * dz);
    ax[h] = dx * inv; ay[h] = dy * inv; az[h] = dz * inv;
  }
  const float ex = o.x - (hi ? cx[1] : cx[0]), ey = o.y - (hi ? cy[1] : cy[0]), ez = o.z - (hi ? cz[1] : cz[0]);
  const float e2 = ex * ex + ey * ey + ez * ez;
  const float cosl = (d.x * (hi ? ax[1] : ax[0]) + d.y * (hi ? ay[1] : ay[0]) + d.z * (hi ? az[1] : az[0])) *
                     __builtin_amdgcn_rsqf(d.x * d.x + d.y * d.y + d.z * d.z);
  const float dev = 1.0f - cosl;
  const bool bad = live && !(e2 <= 1.0e30f && dev >= -0.5f && dev <= 2.5f);
  const uint64_t badm = __ballot(bad);
  const auto half_max = [](float v, float &lo, float &hi_) {
    uint32_t u = __float_as_uint(v);
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, false));  // row_shr:1
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x112, 0xf, 0xf, false));  // row_shr:2
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x114, 0xf, 0xf, false));  // row_shr:4
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x118, 0xf, 0xf, false));  // row_shr:8
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x142, 0xa, 0xf, false));  // row_bcast:15
    lo = __int_as_float(__builtin_amdgcn_readlane((int)u, 31));
    hi_ = __int_as_float(__builtin_amdgcn_readlane((int)u, 63));
  };
  float e2m[2], devm[2];
  half_max(live ? e2 : 0.0f, e2m[0], e2m[1]);
  half_max(live ? fmaxf(dev, 0.0f) : 0.0f, devm[0], devm[1]);
#pragma unroll
  for (int h = 0; h < 2; ++h)
  {
    Bundle &B = H[h];
    B.cx = cx[h]; B.cy = cy[h]; B.cz = cz[h];
    B.ax = ax[h]; B.ay = ay[h]; B.az = az[h];
    B.rw = __builtin_amdgcn_sqrtf(e2m[h]) * 1.0001f;
    B.cosa = 1.0f - devm[h] - 4e-6f;                                             // approximate cosines: widen
    B.sina = __builtin_amdgcn_sqrtf(fmaxf(1.0f - B.cosa * B.cosa, 0.0f) + 1e-7f) * 1.001f;
    const uint64_t hm = h ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
    B.ok = (lm & hm) != 0 && (badm & hm) == 0 && B.cosa > 0.1f && B.rw <= 1.0e15f;
  }
}
#endif

// Bundle of every ray (o, d + rd R) with |rd| <= 1 of the `live` lanes (the shadow rays toward a light of radius R
// for any randDir, Scene.cpp:128-129): make_bundle's cone widened per lane by the angular radius asin(R / |d|) of
// the direction ball, cos(alpha + beta) = cos a cos b - sin a sin b.  A lane whose ball reaches its own origin's
// side (R >= |d| / 2) disables the bound.  For the per-view primary shadow masks (prim_cull_kernel).
__device__ __forceinline__ Bundle make_bundle_ball(v3 o, v3 d, float R, bool live)
{
  Bundle B;
  const int ref = __ffsll((long long)__ballot(live)) - 1;
  B.cx = lane_bcast(o.x, ref); B.cy = lane_bcast(o.y, ref); B.cz = lane_bcast(o.z, ref);
  const float dx = lane_bcast(d.x, ref), dy = lane_bcast(d.y, ref), dz = lane_bcast(d.z, ref);
  const float inv = __builtin_amdgcn_rsqf(dx * dx + dy * dy + dz * dz);
  B.ax = dx * inv; B.ay = dy * inv; B.az = dz * inv;
  const float ex = o.x - B.cx, ey = o.y - B.cy, ez = o.z - B.cz;
  const float e2 = ex * ex + ey * ey + ez * ez;
  const float d2 = d.x * d.x + d.y * d.y + d.z * d.z;
  const float id = __builtin_amdgcn_rsqf(d2);
  const float ca = fminf((d.x * B.ax + d.y * B.ay + d.z * B.az) * id, 1.0f);      // cos alpha (approximate)
  const float sa = __builtin_amdgcn_sqrtf(fmaxf(1.0f - ca * ca, 0.0f));
  const float sb = fminf(R * id * 1.001f, 1.0f), cb = __builtin_amdgcn_sqrtf(fmaxf(1.0f - sb * sb, 0.0f));
  const float cosl = ca * cb - sa * sb;
  const float dev = 1.0f - cosl;
  const bool bad = live && !(e2 <= 1.0e30f && dev >= -0.5f && dev <= 2.5f && sb < 0.5f);
  const float e2m = wave_max_nonneg(live ? e2 : 0.0f);
  const float devm = wave_max_nonneg(live ? fmaxf(dev, 0.0f) : 0.0f);
  B.rw = __builtin_amdgcn_sqrtf(e2m) * 1.0001f;
  B.cosa = 1.0f - devm - 4e-6f;                                                // approximate cosines: widen
  B.sina = __builtin_amdgcn_sqrtf(fmaxf(1.0f - B.cosa * B.cosa, 0.0f) + 1e-7f) * 1.001f;
  B.ok = __ballot(bad) == 0 && B.cosa > 0.1f && B.rw <= 1.0e15f;
  return B;
}

// Bundle of every ray from o with a direction in the quadrilateral d[0..3] of each `live` lane (the sample rays of an SSAA
// pixel: the directions are a linear image of the pixel's sample rectangle, and the cone is convex, so a cone
// holding the four corners holds every ray between them).  For the per-view masks of SSAA frames (prim_cull_kernel).
__device__ __forceinline__ Bundle make_bundle_quad(v3 o, const v3 (&d)[4], bool live)
{
  Bundle B;
  const int ref = __ffsll((long long)__ballot(live)) - 1;
  B.cx = lane_bcast(o.x, ref); B.cy = lane_bcast(o.y, ref); B.cz = lane_bcast(o.z, ref);
  const float dx = lane_bcast(d[0].x, ref), dy = lane_bcast(d[0].y, ref), dz = lane_bcast(d[0].z, ref);
  const float inv = __builtin_amdgcn_rsqf(dx * dx + dy * dy + dz * dz);
  B.ax = dx * inv; B.ay = dy * inv; B.az = dz * inv;
  const float ex = o.x - B.cx, ey = o.y - B.cy, ez = o.z - B.cz;
  const float e2 = ex * ex + ey * ey + ez * ez;
  float dev = 0.0f;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 4; ++k)
  {
    const v3 v = d[k];
    const float cosl = (v.x * B.ax + v.y * B.ay + v.z * B.az) * __builtin_amdgcn_rsqf(v.x * v.x + v.y * v.y + v.z * v.z);
    const float dk = 1.0f - cosl;
    bad = bad || !(dk >= -0.5f && dk <= 2.5f);
    dev = fmaxf(dev, dk);
  }
  bad = live && (bad || !(e2 <= 1.0e30f));
  const float e2m = wave_max_nonneg(live ? e2 : 0.0f);
  const float devm = wave_max_nonneg(live ? fmaxf(dev, 0.0f) : 0.0f);
  B.rw = __builtin_amdgcn_sqrtf(e2m) * 1.0001f;
  B.cosa = 1.0f - devm - 4e-6f;                                                // approximate cosines: widen
  B.sina = __builtin_amdgcn_sqrtf(fmaxf(1.0f - B.cosa * B.cosa, 0.0f) + 1e-7f) * 1.001f;
  B.ok = __ballot(bad) == 0 && B.cosa > 0.1f && B.rw <= 1.0e15f;
  return B;
}

// Bit l: object first + l (l < n <= 64) of the bounding-sphere array may be hit by a ray of the bundle.
// Call with every lane of the wave active.  Cone test: the ray set meets the grown sphere (centre at
// distance L, radius rp) only if the angle between (centre - c) and the axis is at most
// acos(cosa) + asin(rp / L), i.e. va >= cosa sqrt(L^2 - rp^2) - sina rp.
__device__ __forceinline__ uint64_t cull_chunk(const Bound *bound, int first, int n, const Bundle &B)
{
  const int l = (int)(threadIdx.x & 63u);
  bool keep = false;
  if (l < n)
  {
    const Bound g = bound[first + l];
    const float vx = g.x - B.cx, vy = g.y - B.cy, vz = g.z - B.cz;
    const float L2 = cdot(vx, vy, vz, vx, vy, vz);
    const float L = __builtin_amdgcn_sqrtf(L2);
#if RFX_CULL_FMA
    const float rp = __builtin_fmaf(kCullRel, L + B.rw, g.r + B.rw);
    const float va = cdot(vx, vy, vz, B.ax, B.ay, B.az);
    const float lim = __builtin_fmaf(B.cosa, __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-rp, rp, L2), 0.0f)), -(B.sina * rp));
#else
    const float rp = g.r + B.rw + kCullRel * (L + B.rw);
    const float va = cdot(vx, vy, vz, B.ax, B.ay, B.az);
    const float lim = B.cosa * __builtin_amdgcn_sqrtf(fmaxf(L2 - rp * rp, 0.0f)) - B.sina * rp;
#endif
    keep = !(L > rp && va < lim);
  }
  return __ballot(keep);
}

// Triangle footprint (primary bundles, prim_cull_kernel): when every origin lies more than rw (plus a margin) on
// one side of the plane and every direction heads into it (the cone's least cosine to the normal, ndmin, at
// least 0.1), the crossing points lie in a disk around the axis ray's crossing P0 of radius
//   R = h chord (1 + 1 / an) / ndmin + rw (1 + 1 / ndmin)
// (h: the bundle centre's height over the plane, an: the axis's cosine to the normal, chord = |dir - axis| <=
// sqrt(2 - 2 cosa): |dir / (n.dir) - a / (n.a)| <= |dir - a| (1 + 1 / n.a) / n.dir, and an origin offset d moves
// a crossing by at most |d| (1 + 1 / n.dir)).  If that disk lies outside the triangle in (u, v) -- u or v below
// 0, or u + v above 1, by more than R |gu|, R |gv|, R |gu + gv| -- no ray of the bundle can hit it.  Margins
// cover the reference's float (u, v): its inverse basis and its t differ from the exact ones by a relative
// ~150 eps for cond < 100, amplified at most 10x by 1 / ndmin; the margins are 1e-2 of |g| times the
// distances involved (|o - v0| plus the travel to the plane).
__device__ __forceinline__ bool tri_footprint_misses(const CullTri &q, float side, float an, const Bundle &B)
{
  const float h = fabsf(side), anp = side > 0.0f ? -an : an;  // height, cosine of the axis into the plane
  const float snp = __builtin_amdgcn_sqrtf(fmaxf(1.0f - anp * anp, 0.0f));
  const float ndmin = anp * B.cosa - snp * B.sina;
  if (!(h > B.rw * 1.01f + 1e-4f && ndmin > 0.1f)) return false;
  const float ind = __builtin_amdgcn_rcpf(ndmin) * 1.001f, ian = __builtin_amdgcn_rcpf(anp) * 1.001f;
  const float tp = h * ian * (1.0f / 1.001f);                 // travel of the axis ray to the plane (approximate)
  const float px = B.cx + tp * B.ax - q.v0x, py = B.cy + tp * B.ay - q.v0y, pz = B.cz + tp * B.az - q.v0z;
  const float chord = __builtin_amdgcn_sqrtf(fmaxf(2.0f - 2.0f * B.cosa, 0.0f)) * 1.001f;
  const float R = (h * chord * (1.0f + ian) * ind + B.rw * (1.0f + ind) + 1e-4f * tp) * 1.001f + 1e-6f;
  // distances the reference's rounding scales with: |o - v0| <= |c - v0| + rw, travel <= (h + rw) / ndmin
  const float cvx = B.cx - q.v0x, cvy = B.cy - q.v0y, cvz = B.cz - q.v0z;
  const float mag = __builtin_amdgcn_sqrtf(cvx * cvx + cvy * cvy + cvz * cvz) * 1.001f + B.rw + (h + B.rw) * ind;
  const float m = 1e-2f * mag + 1e-6f;
  const float u0 = q.gux * px + q.guy * py + q.guz * pz, v0 = q.gvx * px + q.gvy * py + q.gvz * pz;
  return u0 + (R + m) * q.nu < 0.0f || v0 + (R + m) * q.nv < 0.0f ||
         u0 + v0 - R * q.nuv - m * (q.nu + q.nv) > 1.0f;
}

// Small scenes: lane l tests cull record l (rfx_types.h CullRec) -- the cone test of cull_chunk, and
// for a triangle also its plane: when every origin lies more than rw (plus a margin) on one side and
// every direction leaves that side (axis . n beyond sin of the cone's half-angle, plus a margin), every
// ray has t <= 0 for the plane.  The reference's float test then sees -ao.z and ar.z of opposite signs
// too: for a basis with cond <= 1000 their rounding error stays below 2e-4 of |o - v0| and |ray|, inside
// the 1e-3 margins.  FOOT (the precomputed primary masks only): triangles also take the footprint test above.
// Bits of lanes without an object are cleared.
template <bool FOOT = false>
__device__ __forceinline__ uint64_t cull_small(const CullRec *tab, uint64_t valid, const Bundle &B,
                                               const CullTri *ttab = nullptr)
{
  const CullRec g = tab[threadIdx.x & 63u];
  const float vx = g.x - B.cx, vy = g.y - B.cy, vz = g.z - B.cz;
  const float L2 = cdot(vx, vy, vz, vx, vy, vz);
  const float L = __builtin_amdgcn_sqrtf(L2);
#if RFX_CULL_FMA
  const float rp = __builtin_fmaf(kCullRel, L + B.rw, g.r + B.rw);
  const float va = cdot(vx, vy, vz, B.ax, B.ay, B.az);
  const float lim = __builtin_fmaf(B.cosa, __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-rp, rp, L2), 0.0f)), -(B.sina * rp));
#else
  const float rp = g.r + B.rw + kCullRel * (L + B.rw);
  const float va = cdot(vx, vy, vz, B.ax, B.ay, B.az);
  const float lim = B.cosa * __builtin_amdgcn_sqrtf(fmaxf(L2 - rp * rp, 0.0f)) - B.sina * rp;
#endif
  const float side = cdot(g.nx, g.ny, g.nz, B.cx, B.cy, B.cz) - g.d;
  const float an = cdot(g.nx, g.ny, g.nz, B.ax, B.ay, B.az);
  const float ms = B.rw + 1e-3f * (L + g.r + B.rw) + 1e-6f, ma = B.sina + 1e-3f;
  const bool away = (side > ms && an > ma) || (side < -ms && an < -ma);
  bool keep = !(L > rp && va < lim) && !away;
  if constexpr (FOOT)
    if ((threadIdx.x & 63u) >= 32u && keep) keep = !tri_footprint_misses(ttab[(threadIdx.x & 63u) - 32u], side, an, B);
  return __ballot(keep) & valid;
}

__device__ __forceinline__ uint64_t all_bits(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

// sphere bits (2q, 2q+1) -> pair bit q
__device__ __forceinline__ uint32_t pair_bits(uint64_t m)
{
  uint64_t x = (m | (m >> 1)) & 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  return (uint32_t)x;
}

// ------------------------------------------------------------- closest hit
// Scene.cpp:86-106: the reference keeps the first object with the minimal distance, i.e. the
// lexicographic minimum of (distance, insertion index); any visiting order gives it.  Distances are
// compared through their squares (dist = sqrt_rn(sq) for both kinds, Sphere.cpp:61-62,
// Triangle.cpp:70-85): for sq < best_sq, dist < best unless both round to the same float, i.e. unless
// sq >= sq_lower_bound(best); for sq >= best_sq, dist >= best (tests/test_sqrt_bounds.py).
struct Hit {
  int obj, kind, i;  // object index (-1: none), 0 sphere / 1 triangle / 2 plane, index within its kind
  float t, u, v, sq;
};

__device__ __forceinline__ bool strictly_closer(float sq, float best_sq)
{
  return sq < best_sq && (best_sq == INFINITY || sq < sq_lower_bound(sqrt_rn(best_sq)));
}

// Outside a 2^-20 band around best_sq the rounded distances are ordered like the squares: sq < RN(best_sq (1 - 2^-20))
// gives sqrt_rn(sq) < sqrt_rn(best_sq), sq > RN(best_sq (1 + 2^-20)) gives sqrt_rn(sq) > sqrt_rn(best_sq) (sqrt_rn and the
// products each round by at most 2^-24 relative; all squares here are normal).  Only candidates inside the band take the
// exact test above (tests/test_sqrt_bounds.py checks both claims).  best_sq = +inf: every finite sq is below.
constexpr float kTakeBelow = 0x1.ffffep-1f;  // 1 - 2^-20
constexpr float kTakeAbove = 0x1.00001p+0f;  // 1 + 2^-20

// the comparison key of a candidate and the two decisions on it (Hit::sq holds the winner's key)
constexpr float kNoHitKey = INFINITY;
__device__ __forceinline__ float hit_key(float sq) { return sq; }
__device__ __forceinline__ bool sph_takes(float sq, float best_sq)
{
  if (sq < best_sq * kTakeBelow) return true;
  return strictly_closer(sq, best_sq);
}
// dist < best || (dist == best && obj < best_obj)
__device__ __forceinline__ bool tri_takes(float sq, float best_sq, int obj, int best_obj)
{
  if (sq < best_sq * kTakeBelow) return true;
  if (!(sq <= best_sq * kTakeAbove)) return false;
  return sq < best_sq ? (obj < best_obj || strictly_closer(sq, best_sq))
                      : (obj < best_obj && sqrt_rn(sq) == sqrt_rn(best_sq));
}

// ------------------------------------------------------------- large scenes: per-ray pair BVH
// Each lane walks the pair BVH (rfx_types.h BvhNode) with its own ray: both children's boxes are tested per
// step, the nearer one is entered first and the farther one pushed on a per-lane stack in LDS.  The boxes are
// widened per ray by the exact-cull margin of the wave bundles (a sphere the reference's float test reports as
// hit lies within r + 1.25e-3 |o - c| of the ray; kCullRel = 2e-3 covers it 1.6 times, with |o - c| bounded
// by the distance to the box centre plus its half-diagonal), so a box the ray misses holds no sphere the
// reference could report: skipping it changes no result.  Closest hit: a child whose entry distance exceeds
// the best hit so far (with 0.1% slack over rounding; sphere distances computed by the reference are at least
// the entry distance into their widened box) cannot win or tie and is skipped too.  Leaves run the exact
// pair test with the (distance, object index) rule, so the visiting order changes no result.
constexpr int kBvhStack = 16;
#ifndef RFX_NARROW_BUNDLE_COS
#define RFX_NARROW_BUNDLE_COS 0.9995f
#endif
constexpr float kNarrowBundleCos = RFX_NARROW_BUNDLE_COS;  // rfx_host.cpp RFX_BVH_STACK: deeper hierarchies fall back to the chunk loops
// Stack slots: int16 node / ~pair indices (the host builds no BVH for 32768 or more nodes or pairs).  Halving the
// stack's LDS against int32 slots (8 -> 4 KB per workgroup) made C5 6.3% faster (tools/ab.py, round 2): workgroups
// holding less LDS fit the CU's LDS with more slack as they finish out of order.
typedef int16_t BvhSlot;
__shared__ BvhSlot s_bvh_stack[kBvhStack * kWgThreads];

// Where the BVH walkers read nodes and keep their per-lane stacks: the scene's node array in global memory and the
// workgroup's LDS stack (kernels of kWgThreads threads), or -- the LDS-staged bounce kernel (RFX_LDS_BVH) -- node
// boxes and links staged in the workgroup's LDS by its kLdsBvhThreads threads.
constexpr int kLdsBvhThreads = 64 * kLdsBvhWaves;
static_assert(kLdsBvhStackSlots == kBvhStack, "rfx_types.h lds_bvh_bytes sizes the stacks");
struct BvhGlobal {
  static constexpr int kStride = kWgThreads;
  __device__ __forceinline__ BvhNode node(const DevScene &S, int i) const { return S.bvh[i]; }
  __device__ __forceinline__ BvhSlot *stack() const { return s_bvh_stack + threadIdx.x; }
};
struct BvhLds {
  const float4 *box;  // 3 per node: the first 48 B of BvhNode (both children's boxes)
  const uint2 *aux;   // DevScene::bvh_aux
  BvhSlot *stk;
  float mstep;
  static constexpr int kStride = kLdsBvhThreads;
  __device__ __forceinline__ BvhNode node(const DevScene &, int i) const
  {
    BvhNode n;
    const float4 a = box[3 * i], b = box[3 * i + 1], c = box[3 * i + 2];
    n.lx[0] = a.x; n.lx[1] = a.y; n.ly[0] = a.z; n.ly[1] = a.w;
    n.lz[0] = b.x; n.lz[1] = b.y; n.hx[0] = b.z; n.hx[1] = b.w;
    n.hy[0] = c.x; n.hy[1] = c.y; n.hz[0] = c.z; n.hz[1] = c.w;
    const uint2 x = aux[i];
    n.child[0] = (int32_t)(int16_t)(x.x & 0xFFFFu);
    n.child[1] = (int32_t)(int16_t)(x.x >> 16);
#if RFX_BVH_PREWIDE
    n.mt[0] = n.mt[1] = 0.0f;  // the boxes are stored grown by their node margin
#else
    n.mt[0] = (float)(x.y & 0xFFFFu) * mstep;
    n.mt[1] = (float)(x.y >> 16) * mstep;
#endif
    return n;
  }
  __device__ __forceinline__ BvhSlot *stack() const { return stk + threadIdx.x; }
};

#ifndef RFX_BVH_FMA
#define RFX_BVH_FMA 1
#endif
#ifndef RFX_BVH_TLIM
#define RFX_BVH_TLIM 0
#endif
// box margins from the node's stored term and one per-ray distance (round 2: C5 -8.5% against a margin per box)
#if RFX_BVH_PREWIDE
#if !RFX_BVH_FMA
#error "RFX_BVH_PREWIDE needs RFX_BVH_FMA (finite reciprocals)"
#endif
#ifndef RFX_BVH_PREWIDE_KEEP
#define RFX_BVH_PREWIDE_KEEP 1  // 1: the six slab constants live across the walk; 0: re-derived per node (fewer registers)
#endif
#if RFX_BVH_PREWIDE_KEEP
// the per-ray slab constants: (o + dm) rcp(d) for the low ends, (o - dm) rcp(d) for the high ends
struct RayInv { float ix, iy, iz, dm, lx, ly, lz, hx, hy, hz; };
#else
struct RayInv { float ix, iy, iz, dm; };
#endif
#else
struct RayInv { float ix, iy, iz, dm; };  // dm: kCullRel |o - bvh_ref|_2 + 1e-6 (approximate root, widened 1e-4)
#endif
__device__ __forceinline__ RayInv ray_inv(const DevScene &S, v3 o, v3 ray)
{
  const float ex = o.x - S.bvh_rx, ey = o.y - S.bvh_ry, ez = o.z - S.bvh_rz;
  const float dm = kCullRel * (__builtin_amdgcn_sqrtf(ex * ex + ey * ey + ez * ez) * 1.0001f) + 1e-6f;
#if RFX_BVH_FMA
  // finite reciprocals for the fused slabs: with rcp(0) = inf the fused form's inf - inf would leave one NaN slab end, and
  // fminf / fmaxf would then take the other end for both (a false cull of an axis-parallel ray, tests/test_bvh_box_bound.py)
  const auto fin = [](float v) { return fminf(fmaxf(v, -1e30f), 1e30f); };
#if RFX_BVH_PREWIDE
  const float ix = fin(__builtin_amdgcn_rcpf(ray.x)), iy = fin(__builtin_amdgcn_rcpf(ray.y)),
              iz = fin(__builtin_amdgcn_rcpf(ray.z));
#if RFX_BVH_PREWIDE_KEEP
  return RayInv{ix, iy, iz, dm, (o.x + dm) * ix, (o.y + dm) * iy, (o.z + dm) * iz,
                (o.x - dm) * ix, (o.y - dm) * iy, (o.z - dm) * iz};
#else
  return RayInv{ix, iy, iz, dm};
#endif
#else
  return RayInv{fin(__builtin_amdgcn_rcpf(ray.x)), fin(__builtin_amdgcn_rcpf(ray.y)), fin(__builtin_amdgcn_rcpf(ray.z)), dm};
#endif
#else
  return RayInv{__builtin_amdgcn_rcpf(ray.x), __builtin_amdgcn_rcpf(ray.y), __builtin_amdgcn_rcpf(ray.z), dm};
#endif
}

// child c of node n against the ray: hit (conservative), and the entry parameter t (>= 0) of the widened box.
// Every decision is a comparison that a NaN fails in the keeping direction.
__device__ __forceinline__ bool bvh_box(const BvhNode &n, int c, v3 o, const RayInv &ri, float &tn)
{
  const float lx = n.lx[c], ly = n.ly[c], lz = n.lz[c], hx = n.hx[c], hy = n.hy[c], hz = n.hz[c];
  // |o - c|_2 + half-diagonal <= |o - ref|_2 + mt[c] (c the box centre): the margin is at least
  // kCullRel (|o - c|_2 + half-diagonal) + 1e-6, the per-box bound of the culling argument
#if RFX_BVH_PREWIDE
  // boxes grown by kCullRel mt[c] on the host; the per-ray margin dm sits in the slab constants
#if RFX_BVH_PREWIDE_KEEP
  const float olx = ri.lx, oly = ri.ly, olz = ri.lz, ohx = ri.hx, ohy = ri.hy, ohz = ri.hz;
#else
  const float olx = (o.x + ri.dm) * ri.ix, oly = (o.y + ri.dm) * ri.iy, olz = (o.z + ri.dm) * ri.iz;
  const float ohx = (o.x - ri.dm) * ri.ix, ohy = (o.y - ri.dm) * ri.iy, ohz = (o.z - ri.dm) * ri.iz;
#endif
  const float ax = __builtin_fmaf(lx, ri.ix, -olx), bx = __builtin_fmaf(hx, ri.ix, -ohx);
  const float ay = __builtin_fmaf(ly, ri.iy, -oly), by = __builtin_fmaf(hy, ri.iy, -ohy);
  const float az = __builtin_fmaf(lz, ri.iz, -olz), bz = __builtin_fmaf(hz, ri.iz, -ohz);
#elif RFX_BVH_FMA
  // The slab parameters as (bound - m) ix - o ix with one fused multiply-add each.  This is a cull decision with a
  // margin, not a reference value: it rounds once where the unfused form rounds twice, so the margin covers it as
  // before.  A 0 * inf NaN (axis-parallel ray, or bound - m and o on the same side) drops that axis: conservative.
  const float m = __builtin_fmaf(kCullRel, n.mt[c], ri.dm);
  const float oxi = o.x * ri.ix, oyi = o.y * ri.iy, ozi = o.z * ri.iz;
  const float ax = __builtin_fmaf(lx - m, ri.ix, -oxi), bx = __builtin_fmaf(hx + m, ri.ix, -oxi);
  const float ay = __builtin_fmaf(ly - m, ri.iy, -oyi), by = __builtin_fmaf(hy + m, ri.iy, -oyi);
  const float az = __builtin_fmaf(lz - m, ri.iz, -ozi), bz = __builtin_fmaf(hz + m, ri.iz, -ozi);
#else
  const float m = ri.dm + kCullRel * n.mt[c];
  const float ax = (lx - m - o.x) * ri.ix, bx = (hx + m - o.x) * ri.ix;
  const float ay = (ly - m - o.y) * ri.iy, by = (hy + m - o.y) * ri.iy;
  const float az = (lz - m - o.z) * ri.iz, bz = (hz + m - o.z) * ri.iz;
#endif
  // fminf / fmaxf return the other operand for a NaN (0 * inf on an axis-parallel ray): that axis is ignored
  const float t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
  const float t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
  tn = t0;
  return !(t0 > t1 * 1.00001f + 1e-30f);
}

// closest sphere hit of one lane's ray over the BVH (Scene.cpp:86-106 restricted to the spheres)
template <bool STATS, class NS>
__device__ __forceinline__ void closest_spheres_bvh(const DevScene &S, v3 origin, v3 ray, const RayConst &k, Hit &h,
                                                    Cnt &cnt, const NS &ns)
{
  const RayInv ri = ray_inv(S, origin, ray);
  const float a = 0.5f * k.a2;                // |ray|^2 (exact: a2 = 2a)
#if RFX_BVH_TLIM
  // the entry parameter beyond which a child cannot hold a closer (or tying) sphere, sqrt(1.001 best / a), kept per
  // ray and re-derived on each new best hit: one compare per child instead of three multiplies.  Approximate rcp and
  // sqrt (1 ulp each) under a 1e-4 widening keep it above the exact bound, so it skips no child the product form keeps.
  const float ia = __builtin_amdgcn_rcpf(a);
  float tlim = __builtin_amdgcn_sqrtf(h.sq * 1.001f * ia) * 1.0001f;
#endif
  BvhSlot *stack = ns.stack();
  int sp = 0, node = 0;
  for (;;)
  {
    if (node >= 0)
    {
      const BvhNode n = ns.node(S, node);
      float t0, t1;
      // a child entered beyond the best hit cannot hold a closer (or tying) sphere
#if RFX_BVH_TLIM
      const bool h0 = bvh_box(n, 0, origin, ri, t0) && !(t0 > tlim);
      const bool h1 = bvh_box(n, 1, origin, ri, t1) && !(t1 > tlim);
#else
      const bool h0 = bvh_box(n, 0, origin, ri, t0) && !(t0 * t0 * a > h.sq * 1.001f);
      const bool h1 = bvh_box(n, 1, origin, ri, t1) && !(t1 * t1 * a > h.sq * 1.001f);
#endif
      if (h0 && h1)
      {
        const bool first0 = !(t1 < t0);
        stack[NS::kStride * sp++] = first0 ? n.child[1] : n.child[0];
        node = first0 ? n.child[0] : n.child[1];
        continue;
      }
      if (h0 || h1)
      {
        node = h0 ? n.child[0] : n.child[1];
        continue;
      }
    }
    else
    {
#pragma unroll
      for (int e = 0; e < RFX_BVH_LEAF_PAIRS; ++e)
      {
        const int j = RFX_BVH_LEAF_PAIRS * ~node + e;
        f2 b, d;
        pair_bd(S.sph_pair[j], origin, k, b, d);
        if (pair_may_hit(b, d))
        {
          float t, sq;
          if (sphere_tail<STATS, false, true>(b.x, d.x, ray, k, t, sq, cnt))
          {
            const int obj = S.sph_info[4 * j];
            if (tri_takes(sq, h.sq, obj, h.obj)) { h.sq = sq; h.obj = obj; h.i = 2 * j; h.t = t; }
          }
          if (sphere_tail<STATS, false, true>(b.y, d.y, ray, k, t, sq, cnt))
          {
            const int obj = S.sph_info[4 * j + 2];
            if (tri_takes(sq, h.sq, obj, h.obj)) { h.sq = sq; h.obj = obj; h.i = 2 * j + 1; h.t = t; }
          }
#if RFX_BVH_TLIM
          tlim = __builtin_amdgcn_sqrtf(h.sq * 1.001f * ia) * 1.0001f;
#endif
        }
      }
    }
    if (sp == 0) break;
    node = stack[NS::kStride * --sp];
  }
}

// any sphere but skip_sph occludes the shadow ray (Scene.cpp:129-141 restricted to the spheres): the occluding pair's
// index, or -1.  hint (wave-uniform, RFX_OCC_HINT): a pair that occluded a lane of this wave before, tested first -- an
// occluder is an occluder whatever the order (Scene.cpp:132-141 breaks at the first), so a lane it occludes skips its walk.
#ifndef RFX_OCC_HINT
#define RFX_OCC_HINT 1
#endif
template <bool STATS, class NS>
__device__ __forceinline__ int occluded_spheres_bvh(const DevScene &S, v3 o, v3 ray, const RayConst &k, int skip_sph,
                                                    Cnt &cnt, const NS &ns, int hint = -1)
{
  float t, sq;
  if (RFX_OCC_HINT && hint >= 0)
  {
    f2 b, d;
    pair_bd(S.sph_pair[hint], o, k, b, d);
    if (pair_may_hit(b, d) &&
        ((sphere_tail<STATS, true, true>(b.x, d.x, ray, k, t, sq, cnt) && 2 * hint != skip_sph) ||
         (sphere_tail<STATS, true, true>(b.y, d.y, ray, k, t, sq, cnt) && 2 * hint + 1 != skip_sph)))
      return hint;
  }
  const RayInv ri = ray_inv(S, o, ray);
  BvhSlot *stack = ns.stack();
  int sp = 0, node = 0;
  for (;;)
  {
    if (node >= 0)
    {
      const BvhNode n = ns.node(S, node);
      float t0, t1;
      const bool h0 = bvh_box(n, 0, o, ri, t0), h1 = bvh_box(n, 1, o, ri, t1);
      if (h0 && h1)
      {
        stack[NS::kStride * sp++] = n.child[1];
        node = n.child[0];
        continue;
      }
      if (h0 || h1)
      {
        node = h0 ? n.child[0] : n.child[1];
        continue;
      }
    }
    else
    {
#pragma unroll
      for (int e = 0; e < RFX_BVH_LEAF_PAIRS; ++e)
      {
        const int j = RFX_BVH_LEAF_PAIRS * ~node + e;
        f2 b, d;
        pair_bd(S.sph_pair[j], o, k, b, d);
        // the hit object is filtered out after its test, which does not change the boolean
        if (pair_may_hit(b, d) &&
            ((sphere_tail<STATS, true, true>(b.x, d.x, ray, k, t, sq, cnt) && 2 * j != skip_sph) ||
             (sphere_tail<STATS, true, true>(b.y, d.y, ray, k, t, sq, cnt) && 2 * j + 1 != skip_sph)))
          return j;
      }
    }
    if (sp == 0) return -1;
    node = stack[NS::kStride * --sp];
  }
}

// The planes (Scene::addPlane extension, Plane.cpp:36-73) for one lane, after the other kinds: every lane that
// traces tests every plane (an infinite plane has no bounding sphere to cull with).
template <bool STATS>
__device__ __forceinline__ void closest_planes(const DevScene &S, v3 origin, v3 ray, const RayConst &k, Hit &h, Cnt &cnt)
{
  for (int i = 0; i < S.n_pln; ++i)
  {
    const PlaneGeo g = S.pln_geo[i];
    float t, sq;
    if (plane_hit<STATS, false>(g, origin, ray, t, sq, cnt, k, h.sq) && tri_takes(sq, h.sq, g.obj, h.obj))
    {
      h.sq = sq; h.obj = g.obj; h.kind = 2; h.i = i; h.t = t;
    }
  }
}

// any-hit over the planes but the hit one (skip_pln)
template <bool STATS>
__device__ __forceinline__ bool occluded_planes(const DevScene &S, v3 o, v3 ray, const RayConst &k, int skip_pln, Cnt &cnt)
{
  float t, sq;
  for (int i = 0; i < S.n_pln; ++i)
  {
    if constexpr (STATS)
    {
      if (i != skip_pln && plane_hit<STATS, true>(S.pln_geo[i], o, ray, t, sq, cnt, k)) return true;
    }
    else if (plane_hit<STATS, true>(S.pln_geo[i], o, ray, t, sq, cnt, k) && i != skip_pln)
      return true;
  }
  return false;
}

// Call with every lane of the wave active; `live` lanes trace (origin, ray).  B: the bundle, or null.
// Large scenes: the spheres are stored in spatial order (recursive median splits), 64 to a chunk with a bounding sphere;
// the bundle culls whole chunks (one lane per chunk), then the spheres of the surviving chunks.  The
// visiting order is then not the insertion order, so spheres take the general (distance, object) rule.
template <bool STATS, bool PLANES, class NS = BvhGlobal>
__device__ __forceinline__ void closest_hit(const DevScene &S, v3 origin, v3 ray, bool live, const Bundle *B, Hit &h,
                                            Cnt &cnt, const NS &ns = NS{}, const uint64_t *pl = nullptr)
{
  if (live) RFX_CNT(C_SEGMENTS);
  h.obj = -1; h.kind = 0; h.i = 0; h.t = 0.0f; h.u = 0.0f; h.v = 0.0f; h.sq = kNoHitKey;
  const RayConst k = ray_const(ray);
  const bool cull = B && B->ok;
#ifdef RFX_DEBUG_PROF
  uint32_t st_chunks = 0, st_sph = 0, st_pairs = 0;
#endif
  RFX_PROF_BEGIN(P_SPH);
  // a narrow bundle (the primary rays of a tile: one origin, a cone of ~0.1 degree) culls the spatial chunks and
  // their spheres for the whole wave at once; wider ones walk the BVH lane by lane
  // a per-view list (the tile's primary rays, prim_cull_large_kernel): the kept chunks and their sphere masks as listed
  const bool listed = pl != nullptr;
  const bool use_bvh = !listed && !STATS && S.bvh != nullptr && !(cull && B->cosa > kNarrowBundleCos);
  if (use_bvh && live) closest_spheres_bvh<STATS>(S, origin, ray, k, h, cnt, ns);
  for (int cfirst = 0; !use_bvh && cfirst < S.n_chunk; cfirst += 64)
  {
    uint64_t cm = listed ? pl[2]
                         : cull ? cull_chunk(S.chunk_bound, cfirst, min(64, S.n_chunk - cfirst), *B)
                                : all_bits(min(64, S.n_chunk - cfirst));
#ifdef RFX_DEBUG_PROF
    st_chunks += __popcll(cm);
#endif
    int e = 4;
    while (cm)
    {
      const int first = 64 * (cfirst + __builtin_ctzll(cm));
      cm &= cm - 1ull;
      const int n = min(64, S.n_sph - first);
      const uint64_t m = listed ? pl[e++] : cull ? cull_chunk(S.bound, first, n, *B) : all_bits(n);
      uint32_t pm = pair_bits(m);
#ifdef RFX_DEBUG_PROF
      st_sph += __popcll(m);
      st_pairs += __popc(pm);
#endif
      while (pm)
      {
        const int j = (first >> 1) + __builtin_ctz(pm);
        pm &= pm - 1u;
        f2 b, d;
        pair_bd(S.sph_pair[j], origin, k, b, d);
        if (!live) continue;
        if constexpr (!STATS)
          if (!pair_may_hit(b, d)) continue;  // both miss: one branch
        float t, sq;
        if (sphere_tail<STATS, false, true>(b.x, d.x, ray, k, t, sq, cnt))
        {
          const float key = hit_key(sq);
          const int obj = S.sph_info[4 * j];
          if (tri_takes(key, h.sq, obj, h.obj)) { h.sq = key; h.obj = obj; h.i = 2 * j; h.t = t; }
        }
        if ((!STATS || 2 * j + 1 < S.n_sph) && sphere_tail<STATS, false, true>(b.y, d.y, ray, k, t, sq, cnt))
        {
          const float key = hit_key(sq);
          const int obj = S.sph_info[4 * j + 2];
          if (tri_takes(key, h.sq, obj, h.obj)) { h.sq = key; h.obj = obj; h.i = 2 * j + 1; h.t = t; }
        }
      }
    }
  }
  RFX_PROF_END(P_SPH);
#ifdef RFX_DEBUG_PROF
  RFX_CULL_STAT_LARGE(2, cull, __ballot(live), st_chunks, st_sph, st_pairs);
#endif
  RFX_PROF_BEGIN(P_TRI);
  for (int first = 0; first < S.n_tri; first += 64)
  {
    const int n = min(64, S.n_tri - first);
    uint64_t m = listed ? pl[1] : (B && B->ok) ? cull_chunk(S.bound, S.n_sph + first, n, *B) : all_bits(n);
    while (m)
    {
      const int i = first + __builtin_ctzll(m);
      m &= m - 1ull;
      if (!live) continue;
      float t, u, v, sq;
      if (tri_hit<STATS, false>(S.tri_geo[i], origin, ray, t, u, v, sq, cnt, k, h.sq))
      {
        RFX_CNT(C_TRI_D);
        const int obj = S.tri_shade[i].obj;
        const float key = hit_key(sq);
        if (tri_takes(key, h.sq, obj, h.obj))
        {
          h.sq = key; h.obj = obj; h.kind = 1; h.i = i; h.t = t; h.u = u; h.v = v;
        }
      }
    }
  }
  if constexpr (PLANES)
    if (live) closest_planes<STATS>(S, origin, ray, k, h, cnt);
  RFX_PROF_END(P_TRI);
}

// ------------------------------------------------------------- small scenes (<= 64 objects)
// One cull mask covers the whole scene (bit l: object l of the bound array, spheres then triangles), so
// the object loops need no wave-wide step and run only in the lanes that trace -- a lane leaves the
// any-hit loop at its first occluder.
// lane-layout masks (CullRec): pair q <- lanes q and 16 + q; triangle i <- lane 32 + i
__device__ __forceinline__ uint32_t small_pairs(uint64_t om) { return (uint32_t)((om | (om >> 16)) & 0xFFFFull); }
__device__ __forceinline__ uint64_t small_tris(uint64_t om) { return om >> 32; }

template <bool STATS, bool PLANES>
__device__ __forceinline__ void closest_hit_small(const DevScene &S, v3 origin, v3 ray, uint64_t om, Hit &h, Cnt &cnt)
{
  RFX_CNT(C_SEGMENTS);
  h.obj = -1; h.kind = 0; h.i = 0; h.t = 0.0f; h.u = 0.0f; h.v = 0.0f; h.sq = kNoHitKey;
  const RayConst k = ray_const(ray);
  RFX_PROF_BEGIN(P_SPH);
  // spheres in index order carry increasing object indices, so among spheres a strict `<` already keeps
  // the first of equal distances
  uint32_t pm = small_pairs(om);
  while (pm)
  {
    const int j = __builtin_ctz(pm);
    pm &= pm - 1u;
    f2 b, d;
    pair_bd(S.sph_pair[j], origin, k, b, d);
    if constexpr (!STATS)
      if (!pair_may_hit(b, d)) continue;  // both miss: one branch
    float t, sq;
    if (sphere_tail<STATS, false>(b.x, d.x, ray, k, t, sq, cnt))
    {
      const float key = hit_key(sq);
      if (sph_takes(key, h.sq)) { h.sq = key; h.obj = 2 * j; h.t = t; }
    }
    if ((!STATS || 2 * j + 1 < S.n_sph) && sphere_tail<STATS, false>(b.y, d.y, ray, k, t, sq, cnt))
    {
      const float key = hit_key(sq);
      if (sph_takes(key, h.sq)) { h.sq = key; h.obj = 2 * j + 1; h.t = t; }
    }
  }
  if (h.obj >= 0)
  {
    h.i = h.obj;
    h.obj = Tabs<true>{S}.sph_info(2 * h.i);
  }
  RFX_PROF_END(P_SPH);
  RFX_PROF_BEGIN(P_TRI);
  uint64_t tm = small_tris(om);
  while (tm)
  {
    const int i = __builtin_ctzll(tm);
    tm &= tm - 1ull;
    float t, u, v, sq;
    if (tri_hit<STATS, false>(S.tri_geo[i], origin, ray, t, u, v, sq, cnt, k, h.sq))
    {
      RFX_CNT(C_TRI_D);
      const int obj = S.tri_shade[i].obj;
      const float key = hit_key(sq);
      if (tri_takes(key, h.sq, obj, h.obj))
      {
        h.sq = key; h.obj = obj; h.kind = 1; h.i = i; h.t = t; h.u = u; h.v = v;
      }
    }
  }
  if constexpr (PLANES) closest_planes<STATS>(S, origin, ray, k, h, cnt);
  RFX_PROF_END(P_TRI);
}

// Scene.cpp:129-141 for a small scene (see occluded below for the order and counter notes)
template <bool STATS, bool PLANES>
__device__ __forceinline__ bool occluded_small(const DevScene &S, v3 o, v3 ray, int skip_sph, int skip_tri, int skip_pln,
                                               uint64_t om, Cnt &cnt)
{
  const RayConst k = ray_const(ray);
  float t, sq, u, v;
  uint32_t pm = small_pairs(om);
  while (pm)
  {
    const int j = __builtin_ctz(pm);
    pm &= pm - 1u;
    f2 b, d;
    pair_bd(S.sph_pair[j], o, k, b, d);
    if constexpr (STATS)
    {
      if (2 * j != skip_sph && sphere_tail<STATS, true>(b.x, d.x, ray, k, t, sq, cnt)) return true;
      if (2 * j + 1 != skip_sph && 2 * j + 1 < S.n_sph && sphere_tail<STATS, true>(b.y, d.y, ray, k, t, sq, cnt))
        return true;
    }
    else
    {
      // a miss on both spheres (the common case) costs one branch; the hit object is filtered out after
      // its test, which does not change the boolean
      if (!pair_may_hit(b, d)) continue;
      if (sphere_tail<STATS, true>(b.x, d.x, ray, k, t, sq, cnt) && 2 * j != skip_sph) return true;
      if (sphere_tail<STATS, true>(b.y, d.y, ray, k, t, sq, cnt) && 2 * j + 1 != skip_sph) return true;
    }
  }
  uint64_t tm = small_tris(om);
  while (tm)
  {
    const int i = __builtin_ctzll(tm);
    tm &= tm - 1ull;
    if constexpr (STATS)
    {
      if (i != skip_tri && tri_hit<STATS, true>(S.tri_geo[i], o, ray, t, u, v, sq, cnt, k)) return true;
    }
    else if (tri_hit<STATS, true>(S.tri_geo[i], o, ray, t, u, v, sq, cnt, k) && i != skip_tri)
      return true;
  }
  if constexpr (PLANES) return occluded_planes<STATS>(S, o, ray, k, skip_pln, cnt);
  return false;
}

// ------------------------------------------------------------- shadow any-hit
// Scene.cpp:129-141: every object but the hit one (skip_sph / skip_tri: its sphere or triangle index,
// -1 for the other kind); the boolean does not depend on the order.  Call with every lane of the wave
// active; `live` lanes test (o, ray).  A lane stops at its first occluder and the wave once every live
// lane has one.  (Spheres precede triangles, the reference's order for scenes whose objects are added
// spheres-first -- then even the event counters match it: the second sphere of a pair is counted only
// when the first did not occlude.)
template <bool STATS, bool PLANES, class NS = BvhGlobal>
__device__ __forceinline__ bool occluded(const DevScene &S, v3 o, v3 ray, bool live, int skip_sph, int skip_tri,
                                         int skip_pln, const Bundle *B, Cnt &cnt, const NS &ns = NS{}, int *hint = nullptr)
{
  const RayConst k = ray_const(ray);
  const bool cull = B && B->ok;
  bool occ = false;
  float t, sq, u, v;
  const bool use_bvh = !STATS && S.bvh != nullptr;
  if (use_bvh)
  {
    int found = -1;
    if (live) found = occluded_spheres_bvh<STATS>(S, o, ray, k, skip_sph, cnt, ns, hint ? *hint : -1);
    occ = found >= 0;
    if (RFX_OCC_HINT && hint)
    {
      // the next query's hint: the occluder of this wave's lowest occluded lane
      const uint64_t fm = __ballot(found >= 0);
      if (fm) *hint = __builtin_amdgcn_readlane(found, (int)__builtin_ctzll(fm));
    }
  }
  for (int cfirst = 0; !use_bvh && cfirst < S.n_chunk; cfirst += 64)
  {
    if (__ballot(live && !occ) == 0) return occ;
    uint64_t cm = cull ? cull_chunk(S.chunk_bound, cfirst, min(64, S.n_chunk - cfirst), *B)
                       : all_bits(min(64, S.n_chunk - cfirst));
    while (cm)
    {
      const int first = 64 * (cfirst + __builtin_ctzll(cm));
      cm &= cm - 1ull;
      const int n = min(64, S.n_sph - first);
      const uint64_t m = cull ? cull_chunk(S.bound, first, n, *B) : all_bits(n);
      uint32_t pm = pair_bits(m);
      while (pm)
      {
        const int j = (first >> 1) + __builtin_ctz(pm);
        pm &= pm - 1u;
        f2 b, d;
        pair_bd(S.sph_pair[j], o, k, b, d);
        if (live && !occ)
        {
          if constexpr (STATS)
          {
            if (2 * j != skip_sph && sphere_tail<STATS, true>(b.x, d.x, ray, k, t, sq, cnt)) occ = true;
            else if (2 * j + 1 != skip_sph && 2 * j + 1 < S.n_sph &&
                     sphere_tail<STATS, true>(b.y, d.y, ray, k, t, sq, cnt))
              occ = true;
          }
          else if (pair_may_hit(b, d))
          {
            // the hit object is filtered out after its test, which does not change the boolean
            if (sphere_tail<STATS, true, true>(b.x, d.x, ray, k, t, sq, cnt) && 2 * j != skip_sph) occ = true;
            else if (sphere_tail<STATS, true, true>(b.y, d.y, ray, k, t, sq, cnt) && 2 * j + 1 != skip_sph) occ = true;
          }
        }
        if (__ballot(live && !occ) == 0) return occ;
      }
    }
  }
  for (int first = 0; first < S.n_tri; first += 64)
  {
    if (__ballot(live && !occ) == 0) return occ;
    const int n = min(64, S.n_tri - first);
    uint64_t m = (B && B->ok) ? cull_chunk(S.bound, S.n_sph + first, n, *B) : all_bits(n);
    while (m)
    {
      const int i = first + __builtin_ctzll(m);
      m &= m - 1ull;
      if (live && !occ)
      {
        if constexpr (STATS)
        {
          if (i != skip_tri && tri_hit<STATS, true>(S.tri_geo[i], o, ray, t, u, v, sq, cnt, k)) occ = true;
        }
        else if (tri_hit<STATS, true, true>(S.tri_geo[i], o, ray, t, u, v, sq, cnt, k) && i != skip_tri)
          occ = true;
      }
      if (__ballot(live && !occ) == 0) return occ;
    }
  }
  if constexpr (PLANES)
    if (live && !occ) occ = occluded_planes<STATS>(S, o, ray, k, skip_pln, cnt);
  return occ;
}


// ------------------------------------------------------------- Scene::trace
// Scene::trace (Scene.cpp:73-236) for one trace per lane, the bounce loop run wave-wide: every
// iteration is one segment of every live lane -- closest hit, then per light the facing test and the
// shadow any-hit (Scene.cpp:117-141; the occlusion tests depend on nothing the shading computes, so
// they run first, with few registers live), then material, shading and the next ray or the sky.
// CULL: wave bundles skip objects no live lane can hit (closest hit and shadow rays); MANYL: more than
// 32 lights (shadow masks and shading in blocks of 32); PLANES: the scene holds planes.  Call with every lane
// of the wave active; `valid` lanes trace.  Returns the trace's colour (zero for invalid lanes).
// Parking (ray regrouping): where the bounce loop would start segment `park` of a trace, the trace's state is
// appended to the queue instead (one atomic per wave, packed lane order) and the trace ends here; the bounce
// kernel resumes it from exactly that state, so every float op is the same.
struct Park {
  int after;           // segments before parking (<= 0: never)
  QRay *queue;
  uint32_t *count;
  uint32_t trace, out;  // this lane's randDir trace index and output pixel
  static constexpr bool kRefill = false;
  __device__ __forceinline__ void ids(uint32_t &t, uint32_t &o) const { t = trace; o = out; }
  __device__ __forceinline__ uint32_t *keys() const { return nullptr; }
  __device__ __forceinline__ BvhGlobal bvh() const { return BvhGlobal{}; }
};

// Regroup sort key of a parked trace (RFX_QUEUE_SORT): its direction octant and the Morton index of its origin's cell
// in an 8 x 8 x 8 grid over the BVH root box -- traces of one bucket walk similar BVH paths.  Only the order in which
// the bounce kernel takes the traces depends on it, never a value (every trace resumes from its own state).
__device__ __forceinline__ uint32_t queue_key(const DevScene &S, v3 o, v3 d)
{
  const auto cell = [](float v, float lo, float s) -> uint32_t {
    return (uint32_t)fminf(fmaxf((v - lo) * s, 0.0f), 7.0f);  // NaN: fmaxf takes the 0
  };
  const uint32_t cx = cell(o.x, S.key_lx, S.key_sx), cy = cell(o.y, S.key_ly, S.key_sy), cz = cell(o.z, S.key_lz, S.key_sz);
  uint32_t m = 0;
#pragma unroll
  for (int b = 0; b < 3; ++b)
    m |= (((cx >> b) & 1u) << (3 * b)) | (((cy >> b) & 1u) << (3 * b + 1)) | (((cz >> b) & 1u) << (3 * b + 2));
  const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
  return oct << 9 | m;
}

// Per wave: the epilogue's staging of the wave's 64 pixels (store_wave_tile: 192 RGB floats + 64 ARGB words)
__shared__ __attribute__((aligned(16))) uint32_t s_out[kWgWaves][256];

// Scene::trace from a mid-trace state (mulc, pix after `refl` segments); park: see Park.  *parked: this lane's
// trace was queued and its returned colour is not final.
// Kernel arguments re-read where they are used (round 4, on by default; RFX_NO_LAUNDER turns it off): the DevScene in
// every bounce segment of the large-scene kernels, the FrameParams after the bounce loop.  Kept in SGPRs across the loops, they
// spilled to VGPR lanes (C5 trace kernel: 102 -> 25 SGPR spills, C5 trace + bounce -1.6%; C3: 23 -> 8, -0.3%;
// interleaved A/B, profiles/r04/ab/).
#ifndef RFX_NO_LAUNDER
#define RFX_LAUNDER_SCENE
#define RFX_LAUNDER_PARAMS
#endif
#ifdef RFX_LAUNDER_SCENE
typedef const __attribute__((address_space(4))) DevScene *ConstScenePtr;
// The record is read through the kernarg segment pointer: every kernel that reaches trace_from (trace_kernel,
// bounce_kernel, bounce_kernel_lds) takes the DevScene as its first argument, at offset 0.  (Taking the address of
// the by-value parameter instead makes the compiler copy it to scratch, and a constant-space pointer to that copy
// faults.)
template <bool ON>
__device__ __forceinline__ const DevScene &launder_scene(const DevScene &S)
{
  if constexpr (!ON) return S;
  ConstScenePtr p = (ConstScenePtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const DevScene *)p;
}
#define RFX_SCENE_PARAM S_in
#else
#define RFX_SCENE_PARAM S
#endif
// The frame parameters (the kernels' second argument, after the DevScene) read through the kernarg segment pointer, laundered
// by an empty asm: every use reloads them with scalar loads where it stands, so their values are not held in SGPRs
// across a bounce loop (with RFX_LAUNDER_PARAMS: the epilogue and the park ids; the RFX_SSAA_LDS_STATE sample loop)
constexpr size_t kParamsOff = (sizeof(DevScene) + alignof(FrameParams) - 1) / alignof(FrameParams) * alignof(FrameParams);
// The layout both readers assume, checked where it is defined (host and device passes): by-value kernel arguments are
// laid out like the members of a struct, so (DevScene, FrameParams, ...) puts the record at 0 and the parameters at
// kParamsOff.  Every kernel that reads them this way asserts its own signature (kKernargSig, in its body), and
// tests/test_gpu_kat.py::test_kernarg_layout compares the laundered reads with the by-value arguments on the device.
struct KernargPair { DevScene S; FrameParams P; };
static_assert(offsetof(KernargPair, S) == 0 && offsetof(KernargPair, P) == kParamsOff,
              "kernel-argument layout: DevScene at offset 0, FrameParams at kParamsOff");
template <class F>
constexpr bool kKernargSig = std::is_same<F, void (*)(DevScene, FrameParams)>::value;
template <bool LAUNDER = true>  // false: the plain kernarg reference, which the compiler may keep in registers
__device__ __forceinline__ const FrameParams &kernarg_params()
{
  typedef const __attribute__((address_space(4))) char *KP;
  KP p = (KP)__builtin_amdgcn_kernarg_segment_ptr();
  if constexpr (LAUNDER) asm volatile("" : "+s"(p));
  return *(const FrameParams *)(const __attribute__((address_space(4))) FrameParams *)(p + kParamsOff);
}

template <bool STATS, bool CULL, bool MANYL, bool SMALL, bool PLANES, bool PARK, class PK, bool ONEL = false>
__device__ __forceinline__ col trace_from(const DevScene &RFX_SCENE_PARAM, v3 origin, v3 ray, col mulc, col pix, int refl,
                                          int depth, v3 rd, const float *lut, Cnt &cnt, bool valid, const PK &park,
                                          bool &parked, const uint64_t *pm_tile = nullptr, bool pm_shadow = true)
{
#ifdef RFX_LAUNDER_SCENE
  const DevScene &S = S_in;
#endif
  // the first segment of a plain small-scene trace: this tile's per-view masks (prim_cull_kernel) -- the closest
  // hit's, then one per light for its shadow rays
  bool seg0 = pm_tile != nullptr;
  parked = false;
  if (valid && refl == 0) RFX_CNT(C_RAYS);
  const Tabs<SMALL> T{S};
  bool alive = valid && refl < depth;
  int occ_hint = -1;  // large scenes: the shadow rays' occluder hint (occluded_spheres_bvh)
#ifdef RFX_DEBUG_SEGS
  int nseg = 0;  // diagnostic build only (tools/segstats.py): the trace's segment count replaces its colour
#endif
  RFX_PROF_BEGIN(P_SEG);
  while (__ballot(alive))
  {
#ifdef RFX_DEBUG_SEGS
    if (alive) ++nseg;
#endif
#ifdef RFX_LAUNDER_SCENE
    // experiment: the scene record re-read (scalar loads from the kernarg segment) in every segment instead of its
    // fields held in SGPRs across the bounce loop, where they spill to VGPR lanes
    const DevScene &S = launder_scene<!SMALL>(S_in);  // large scenes only: the small-scene kernel spills VGPRs with it
    const Tabs<SMALL> T{S};
#endif
    Hit h;
    if constexpr (SMALL)
    {
      uint64_t om = S.cull_valid;
      if constexpr (CULL)
      {
        if (seg0)
          om = pm_tile[0];  // the primary bundle's mask, precomputed for this tile's view (prim_cull_kernel)
        else
        {
          const Bundle B = make_bundle(origin, ray, alive);
          if (B.ok) om = cull_small(T.cull(), S.cull_valid, B);
#ifdef RFX_HALF_BUNDLES
          else  // too wide for one cone: a cone per half wave, and the objects either half may hit
          {
            Bundle H[2];
            make_bundle_halves(origin, ray, alive, H);
            om = (H[0].ok ? cull_small(T.cull(), S.cull_valid, H[0]) : S.cull_valid) |
                 (H[1].ok ? cull_small(T.cull(), S.cull_valid, H[1]) : S.cull_valid);
          }
#endif
          RFX_CULL_STAT(0, B.ok, __ballot(alive), om, S.cull_valid);
        }
      }
      if (alive) closest_hit_small<STATS, PLANES>(S, origin, ray, om, h, cnt);
      else h.obj = -1;
    }
    else
    {
      // the first segment of a plain trace: the tile's per-view chunk list (prim_cull_large_kernel), when it has one
      const uint64_t *pl = RFX_PRIM_LARGE && CULL && seg0 && pm_tile[0] != kPrimLargeNone ? pm_tile : nullptr;
      Bundle B;
      if constexpr (CULL) B = make_bundle(origin, ray, alive);
      closest_hit<STATS, PLANES>(S, origin, ray, alive, CULL ? &B : nullptr, h, cnt, park.bvh(), pl);
    }
    const bool hit = alive && h.obj >= 0;
    // re-derive the winner's outputs with the reference's expressions
    v3 drop = origin, norm = mk(0.0f, 0.0f, 0.0f);
    RFX_PROF_BEGIN(P_WIN);
    if (hit)
    {
      drop = add(origin, mul(ray, h.t));
      if (h.kind == 0)
      {
        RFX_CNT(C_HIT_SPH);
        const SphereGeo g = T.sph_geo(h.i);
        norm = sub(drop, mk(g.cx, g.cy, g.cz));                                // Sphere.cpp:67
      }
      else if (!PLANES || h.kind == 1)
      {
        RFX_CNT(C_HIT_TRI);
        const TriShade sh = T.tri_shade(h.i);
        norm = mk(sh.nx, sh.ny, sh.nz);
      }
      else
      {
        RFX_CNT(C_HIT_PLN);
        const PlaneGeo g = S.pln_geo[h.i];
        norm = mk(g.nx, g.ny, g.nz);                                               // Plane.cpp:58-59
      }
    }
    RFX_PROF_END(P_WIN);
    const int skip_sph = h.kind == 0 ? h.i : -1, skip_tri = h.kind == 1 ? h.i : -1;
    const int skip_pln = PLANES && h.kind == 2 ? h.i : -1;
    MatRec m{0.0f, 0.0f, 0.0f, 0.0f};
    int diel = 0;
    v3 reflv = mk(0.0f, 0.0f, 0.0f);
    float rayLen = 0.0f, normLen = 0.0f, reflectLen = 0.0f;
    col sumL = mkc(0.0f, 0.0f, 0.0f), sumS = mkc(0.0f, 0.0f, 0.0f);
    for (int base = 0;; base += 32)                                            // Scene.cpp:117-181
    {
      RFX_PROF_BEGIN(P_SHADOW);
      uint32_t lit = 0;
      const int nl = ONEL ? 1 : min(32, S.n_light - base);  // ONEL: the scene has exactly one light
      for (int q = 0; q < nl; ++q)
      {
        const LightRec L = S.lights[base + q];
        bool facing = false;
        v3 sray = mk(0.0f, 0.0f, 0.0f);
        if (hit)
        {
          RFX_CNT(C_L_EVAL);
          const v3 dtl = sub(mk(L.ox, L.oy, L.oz), drop);
          if (dot(dtl, norm) > kVerySmall)
          {
            RFX_CNT(C_L_FACING);
            facing = true;
            sray = add(dtl, mul(rd, L.radius));                                  // Scene.cpp:129
          }
        }
        if (__ballot(facing))
        {
          if constexpr (SMALL)
          {
            uint64_t om = S.cull_valid;
            if constexpr (CULL)
            {
              if (!MANYL && seg0 && pm_shadow && q < kPrimLights)
                om = pm_tile[1 + q];  // the primary hits' shadow mask for light q, precomputed for the view
              else
              {
                const Bundle SB = make_bundle(drop, sray, facing);
                if (SB.ok) om = cull_small(T.cull(), S.cull_valid, SB);
                RFX_CULL_STAT(1, SB.ok, __ballot(facing), om, S.cull_valid);
              }
            }
            if (facing && !occluded_small<STATS, PLANES>(S, drop, sray, skip_sph, skip_tri, skip_pln, om, cnt))
              lit |= 1u << q;
          }
          else
          {
            Bundle SB;
            if constexpr (CULL) SB = make_bundle(drop, sray, facing);
            const bool occ = occluded<STATS, PLANES>(S, drop, sray, facing, skip_sph, skip_tri, skip_pln,
                                                     CULL ? &SB : nullptr, cnt, park.bvh(), &occ_hint);
            if (facing && !occ) lit |= 1u << q;
          }
        }
      }
      RFX_PROF_END(P_SHADOW);
      RFX_PROF_BEGIN(P_LIGHT);
      if (hit)
      {
        if (!MANYL || base == 0)
        {
          // the hit object's material, texel, reflection and lengths (Sphere.cpp:66-80, Triangle.cpp:86-105)
          if (h.kind == 0)
          {
            m = T.sph_mat(h.i);
            diel = T.sph_info(2 * h.i + 1);
          }
          else if (PLANES && h.kind == 2)
          {
            m = S.pln_mat[h.i];                                                  // untextured (Plane.cpp:67-68)
            diel = S.pln_geo[h.i].dielectric;
          }
          else
          {
            const TriShade sh = T.tri_shade(h.i);
            m = T.tri_mat(h.i);
            diel = sh.dielectric;
            if (sh.tex >= 0)
            {
              const col c = tri_texel<STATS>(S, sh, h.u, h.v, lut, cnt);
              m.r = c.r; m.g = c.g; m.b = c.b;
            }
          }
          reflv = reflect(mul(ray, h.t), norm);                                // trace_math.cpp:14-23
          rayLen = len(ray); normLen = len(norm); reflectLen = len(reflv);
        }
        for (int q = 0; q < nl; ++q)
        {
          if (!((lit >> q) & 1u)) continue;
          RFX_CNT(C_L_LIT);
          const LightRec L = S.lights[base + q];
          const v3 dtl = sub(mk(L.ox, L.oy, L.oz), drop);
          const float dlen = len(dtl);
          float aa = dlen * normLen;
          const float cosl = (aa > kVerySmall) ? qdiv(dot(dtl, norm), aa) : 0.0f;
          const col lc = mkc(L.r, L.g, L.b);
          if (L.power > kVerySmall) sumL = cadd(sumL, cscale(cscale(lc, cosl), L.power));
          aa = sqlen(dtl);
          const float ang = (aa > kVerySmall) ? 1.0f - qdiv(L.radius * L.radius, aa) : 0.0f;
          if (ang > 0)
          {
            RFX_CNT(C_L_SPEC);
            const v3 dlr = add(normalized(dtl), mul(rd, 1.0f - m.refl));
            aa = len(dlr) * reflectLen;
            float sc = (aa > kVerySmall) ? qdiv(dot(dlr, reflv), aa) : 0.0f;
            sc = clampf(sc + (1.0f - sqrt_rn(ang)), 0.0f, 1.0f);
            if (sc > kVerySmall && L.radius > kVerySmall)
            {
              RFX_CNT(C_L_POW);
              const float sp = powf_dev(sc, 1 + qdiv(3 * m.refl * dlen, L.radius)) * m.refl;
              sumS = cadd(sumS, cscale(lc, sp));
            }
          }
        }
      }
      RFX_PROF_END(P_LIGHT);
      if (!MANYL || base + 32 >= S.n_light) break;
    }
    if (hit)
    {
      RFX_PROF_BEGIN(P_MAT);
      sumL = cadd(mkc(S.amb_r, S.amb_g, S.amb_b), sumL);                        // Scene.cpp:186
      const col color = mkc(m.r, m.g, m.b);
      col fin;
      if (diel)                                                                  // Scene.cpp:189-201
      {
        RFX_CNT(C_DIELECTRIC);
        const float aa = rayLen * normLen;
        const float cosA = (aa > kVerySmall) ? clampf(qdiv(dot(ray, neg(norm)), aa), 0.0f, 1.0f) : 0.0f;
        const float r = 0.2f + 0.8f * powf3_dev(1.0f - cosA);
        fin = cadd(cmul(cscale(color, 1.0f - r), sumL), sumS);
        fin = cmul(fin, mulc);
        mulc = cscale(mulc, r);
      }
      else                                                                       // Scene.cpp:202-212
      {
        RFX_CNT(C_METAL);
        const float r = 0.8f;
        fin = cadd(cmul(cscale(color, 1.0f - r), sumL), sumS);
        fin = cmul(fin, mulc);
        mulc = cmul(mulc, cscale(color, r));
      }
      pix = cclamp(cadd(pix, fin));                                              // Scene.cpp:215-216
      RFX_PROF_END(P_MAT);
      if (mulc.r < 0.01f && mulc.g < 0.01f && mulc.b < 0.01f)                    // Scene.cpp:219-220
        alive = false;
      else
      {
        RFX_CNT(C_CONTINUE);
        origin = drop;                                                           // Scene.cpp:223-224
        ray = add(normalized(reflv), mul(rd, 1.0f - m.refl));
        if (++refl >= depth) alive = false;                                      // Scene.cpp:78
      }
    }
    else if (alive)                                                              // Scene.cpp:226-231
    {
      RFX_CNT(C_SKY);
      RFX_PROF_BEGIN(P_SKY);
      pix = cclamp(cadd(pix, cmul(cmul(mulc, skybox_texel<STATS>(S, ray, lut, cnt)), mkc(S.env_r, S.env_g, S.env_b))));
      RFX_PROF_END(P_SKY);
      alive = false;
    }
    seg0 = false;
    if constexpr (!STATS && PARK)
    {
      if (refl == park.after && __ballot(alive))
      {
        // every lane of the wave is here (wave-uniform loop); the live ones append their state
        const uint64_t pm = __ballot(alive);
        uint32_t base = 0;
        if (__lane_id() == (uint32_t)(__ffsll((long long)pm) - 1)) base = atomicAdd(park.count, (uint32_t)__popcll(pm));
        base = __builtin_amdgcn_readlane(base, __ffsll((long long)pm) - 1);
        if (alive)
        {
          QRay q;
          q.ox = origin.x; q.oy = origin.y; q.oz = origin.z; q.dx = ray.x;
          q.dy = ray.y; q.dz = ray.z; q.mr = mulc.r; q.mg = mulc.g;
          q.mb = mulc.b; q.pr = pix.r; q.pg = pix.g; q.pb = pix.b;
          uint32_t qt, qo;
          park.ids(qt, qo);
          q.trace = qt; q.out = qo; q.refl = (uint32_t)refl; q.pad = 0;
          const uint32_t slot = base + (uint32_t)__popcll(pm & ((1ull << __lane_id()) - 1ull));
          park.queue[slot] = q;
          if (uint32_t *keys = park.keys()) keys[slot] = queue_key(S, origin, ray);
          parked = true;
          alive = false;
        }
      }
    }
    // the bounce kernel: traces that ended this segment write their pixels, idle lanes take new ones (Refill)
    if constexpr (PK::kRefill) park.refill(alive, origin, ray, mulc, pix, refl, rd);
  }
  RFX_PROF_END(P_SEG);
#ifdef RFX_DEBUG_SEGS
  return mkc((float)nseg, 0.0f, 0.0f);
#else
  return pix;
#endif
}

template <bool STATS, bool CULL, bool MANYL, bool SMALL, bool PLANES, bool ONEL = false>
__device__ __forceinline__ col trace(const DevScene &S, v3 origin, v3 ray, int depth, v3 rd, const float *lut,
                                     Cnt &cnt, bool valid, const uint64_t *pm_tile = nullptr, bool pm_shadow = true)
{
  bool parked;
  return trace_from<STATS, CULL, MANYL, SMALL, PLANES, false, Park, ONEL>(S, origin, ray, mkc(1.0f, 1.0f, 1.0f), mkc(0.0f, 0.0f, 0.0f), 0,
                                                       depth, rd, lut, cnt, valid, Park{0, nullptr, nullptr, 0, 0},
                                                       parked, pm_tile, pm_shadow);
}

template <bool STATS>
__device__ __forceinline__ void flush_counters(const FrameParams &P, Cnt &cnt)
{
  if constexpr (STATS)
  {
#pragma unroll
    for (int k = 0; k < C_COUNT; ++k)
    {
      unsigned long long v = cnt.c[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(&P.counters[k], v);
    }
  }
}

__device__ __forceinline__ uint32_t strip_row_to_y(uint32_t r, const FrameParams &P)
{
  if (P.nranks <= 1) return r;
  const uint32_t blk = r / P.row_block, w = r % P.row_block;
  return (blk * P.nranks + P.rank) * P.row_block + w;
}

// the wave's schedule tile (index into the wave-tile grid), kept in LDS across the bounce loop
__shared__ uint32_t s_tile8[kWgWaves];

// Park info of a plain-pixel trace-kernel lane: its randDir trace index and output pixel are re-derived from the
// wave's tile index in LDS when the trace parks (a fresh lane id through an empty asm), instead of being kept
// live across the bounce loop (C3 park instantiation: 13 -> 2 VGPR spills)
struct ParkTile {
  int after;
  QRay *queue;
  uint32_t *count;
  const FrameParams &P;
  uint32_t wv, w8;
  __device__ __forceinline__ void ids(uint32_t &t, uint32_t &o) const
  {
    const uint32_t t8 = ((volatile uint32_t *)s_tile8)[wv];
    uint32_t le = __lane_id();
    asm volatile("" : "+v"(le));
#ifdef RFX_LAUNDER_PARAMS
    const FrameParams &P = kernarg_params();
#endif
    const uint32_t gx = (t8 % w8) * 8u + (le & 7u), gy = (t8 / w8) * 8u + (le >> 3);
    const uint32_t y = P.nranks > 1 ? strip_row_to_y(gy, P) : gy + P.row0;
    const uint32_t orow = P.nranks > 1 ? gy : y;
    t = (uint32_t)((uint64_t)y * P.W + gx - P.p_begin);
    o = (uint32_t)((size_t)orow * P.W + gx);
  }
  static constexpr bool kRefill = false;
  __device__ __forceinline__ uint32_t *keys() const { return P.queue_key; }
  __device__ __forceinline__ BvhGlobal bvh() const { return BvhGlobal{}; }
};

// trace i's randomInsideSphere draw (Vector3.cpp:176-188) from the LCG state before its accepted triple
__device__ __forceinline__ v3 rd_from_state(uint32_t s)
{
  const uint32_t s1 = lcg_step(s), s2 = lcg_step(s1), s3 = lcg_step(s2);
  return mk(rand_component_dev(lcg_out(s1)), rand_component_dev(lcg_out(s2)), rand_component_dev(lcg_out(s3)));
}

__device__ __forceinline__ v3 load_rd(const FrameParams &P, uint64_t i) { return rd_from_state(P.rd_state[i]); }

// Diagnostic build only (RFX_DEBUG_WAVES, tools/wave_timeline.py): each plain-mode wave's start and end on the
// chip's constant 100 MHz clock (s_memrealtime), by wave tile, for the last launch -- the shape of a launch's
// critical path (dispatch ramp, tile durations, tail).
#ifdef RFX_DEBUG_WAVES
constexpr uint32_t kWaveTimeMax = 1u << 18;
constexpr uint32_t kBounceTimeBase = 1u << 17;  // the bounce kernel's 64-trace batches, after the trace kernel's tiles
static __device__ unsigned long long g_wave_time[2 * kWaveTimeMax];
__device__ __forceinline__ uint64_t realtime64()
{
  uint64_t c;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c));
  return c;
}
#define RFX_WAVE_T0() const uint64_t wave_t0_ = realtime64()
#define RFX_WAVE_T1(tile)                                                                  \
  do {                                                                                      \
    const uint64_t t1_ = realtime64();                                                     \
    if (__lane_id() == 0 && (tile) < kWaveTimeMax)                                         \
    {                                                                                       \
      g_wave_time[2 * (tile)] = wave_t0_;                                                   \
      g_wave_time[2 * (tile) + 1] = t1_;                                                    \
    }                                                                                       \
  } while (0)
#else
constexpr uint32_t kBounceTimeBase = 0;
#define RFX_WAVE_T0() \
  do {                \
  } while (0)
#define RFX_WAVE_T1(tile) \
  do {                    \
  } while (0)
#endif

// Shader clock, low 32 bits.  A plain asm statement (no side effects declared, so the compiler may still
// serve the scene loads that follow through the scalar cache -- __builtin_readcyclecounter would count as a
// memory clobber for them); it waits for its own result.
__device__ __forceinline__ uint32_t clock32()
{
  uint64_t c;
  asm("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c));
  return (uint32_t)c;
}


// A wave's 8x8 pixels (lane = 8 row + column) at output row `row0`, column `x0`: the colours go through the
// wave's LDS slot and leave as ONE 16-B-per-lane store -- lanes 0-47 write the 8 rows of 8 RGB floats
// (96 B = 6 x 16 B per row, Render.cpp:185's interleaved Color layout), lanes 48-63 the 8 rows of 8 ARGB words
// (32 B = 2 x 16 B per row).  Call with every lane valid; needs W % 4 == 0 and 16-B-aligned images.
__device__ __forceinline__ void store_wave_tile(const FrameParams &P, uint32_t x0, uint32_t row0, col out,
                                                uint32_t lane, uint32_t wave)
{
  uint32_t *s = s_out[wave];
  s[3 * lane] = __float_as_uint(out.r);
  s[3 * lane + 1] = __float_as_uint(out.g);
  s[3 * lane + 2] = __float_as_uint(out.b);
  s[192 + lane] = argb(out);
  __builtin_amdgcn_wave_barrier();
  const bool rgb = lane < 48;
  const uint32_t k = rgb ? lane : lane - 48;
  const uint32_t r = rgb ? k / 6u : k >> 1, c = rgb ? k % 6u : k & 1u;
  const uint4 v = *reinterpret_cast<const uint4 *>(s + (rgb ? r * 24u + 4u * c : 192u + r * 8u + 4u * c));
  const size_t pix = (size_t)(row0 + r) * P.W + x0;
  uint32_t *dst = rgb ? reinterpret_cast<uint32_t *>(P.img) + pix * 3 + 4u * c : P.argb + pix + 4u * c;
  if (rgb || P.argb) *reinterpret_cast<uint4 *>(dst) = v;
}

// Pixel loop variants of Render::renderNext: block preview (sampleNum < 0), one plain trace per pixel
// (sampleNum == 1, no jitter, no accumulation -- the benchmark frame), and the general SSAA / additive
// loop.  The plain variant drops the sample loops and their live state (no spills before the bounce loop).
enum TraceMode { kModeSsaa = 0, kModeBlock = 1, kModePlain = 2, kModeSsaaLanes = 3, kModeSsaaChunks = 4 };
// kModeSsaaLanes (sampleNum 1 with jitter or accumulation, 2, 4, 8): one lane per sample -- a wave is a bw x bw block of
// pixels (ss_lane_block), each pixel's ss x ss samples in consecutive lanes, and the wave sums each pixel's samples in the
// reference's order afterwards; kModeSsaaChunks (sampleNum > 8): the same with the wave on one pixel, its samples 64 at
// a time (a separate mode: the chunk loop around the bounce loop costs registers); sampleNum 3, 5, 6, 7 run kModeSsaa
// (one lane per pixel, its samples in turn)
__host__ __device__ constexpr uint32_t ss_lane_block(int ss)
{
  return ss == 1 ? 8u : ss == 2 ? 4u : ss == 4 ? 2u : ss >= 8 ? 1u : 0u;
}
#ifndef RFX_SSAA_LANES
#define RFX_SSAA_LANES 1
#endif
// CFG bits: kCfgCull -- wave-bundle culling (every non-stats launch); kCfgManyLights -- more than 32 lights;
// kCfgSmall -- at most 32 spheres and 32 triangles (one lane-layout cull mask for the whole scene)
// kCfgPlanes -- the scene holds planes (Scene::addPlane extension); kCfgPark -- plain pixels park their traces
// for the bounce kernel (ray regrouping; rfx_trace_plain_park.hip)
constexpr int kCfgCull = 1, kCfgManyLights = 2, kCfgSmall = 4, kCfgPlanes = 8, kCfgPark = 16, kCfgOneLight = 32;
#ifndef RFX_ONE_LIGHT
#define RFX_ONE_LIGHT 1
#endif

// one workgroup = kTileW x kTileH output pixels (block mode: block corners), one wave = an 8x8 tile (ray coherence).
// Every lane of a wave reaches trace() -- lanes outside the frame or the cursor span as invalid -- so the
// bounce loop can use wave-wide bundles.
#ifndef RFX_WAVES_PER_EU_LARGE
#define RFX_WAVES_PER_EU_LARGE RFX_WAVES_PER_EU  // large-scene (BVH) trace kernels' occupancy target (experiment)
#endif
#ifndef RFX_SSAA_CHANNEL_SUM
#define RFX_SSAA_CHANNEL_SUM 1  // SSAA epilogues: one lane per colour channel runs the ordered sample sum
#endif
template <bool STATS, int MODE, int CFG>
__global__ __launch_bounds__(kWgThreads) __attribute__((amdgpu_waves_per_eu(
    (CFG & kCfgSmall) ? RFX_WAVES_PER_EU : RFX_WAVES_PER_EU_LARGE))) void trace_kernel(DevScene S, FrameParams P)
{
  static_assert(kKernargSig<decltype(&trace_kernel<STATS, MODE, CFG>)>, "launder_scene / kernarg_params layout");
  constexpr bool CULL = (CFG & kCfgCull) != 0, MANYL = (CFG & kCfgManyLights) != 0, SMALL = (CFG & kCfgSmall) != 0;
  constexpr bool PLANES = (CFG & kCfgPlanes) != 0, PARK = MODE == kModePlain && !STATS && (CFG & kCfgPark) != 0;
  constexpr bool ONEL = (CFG & kCfgOneLight) != 0;  // exactly one light: the light loops unrolled
  RFX_WAVE_T0();
  __shared__ float lut[256];
  for (uint32_t i = threadIdx.x; i < 256; i += kWgThreads) lut[i] = (float)i / 255.0f;  // Color.cpp:11-13
  stage_powf_tables();
  if constexpr (SMALL) stage_small_scene(S);
  RFX_PROF_INIT();
  // tile cost: the workgroup's start clock (low 32 bits) waits in LDS, so the bounce loop keeps no register for it
  __shared__ uint32_t s_clk0;
  if (P.tile_cost && threadIdx.x == 0) s_clk0 = clock32();
  __syncthreads();
  Cnt cnt;
  if constexpr (STATS)
  {
#pragma unroll
    for (int k = 0; k < C_COUNT; ++k) cnt.c[k] = 0;
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  // the schedule's unit is the wave's 8x8 tile (round 2: -2.7% trace against the workgroup's 16x8): wave v of
  // workgroup w renders tile tile_order[kWgWaves w + v] of the (kTileWavesX gridDim.x) x (kTileWavesY gridDim.y)
  // tile grid -- with a tile order (longest-processing-time first, from an earlier launch's measured tile costs)
  // the most expensive tiles start first and the cheap ones fill the tail; without, the workgroup's own tiles
  const uint32_t wv = __builtin_amdgcn_readfirstlane(wave), wid = blockIdx.y * gridDim.x + blockIdx.x;
  const uint32_t w8 = kTileWavesX * gridDim.x;
  const uint32_t t8 = P.tile_order ? P.tile_order[kWgWaves * wid + wv]
                                   : (blockIdx.y * kTileWavesY + wv / kTileWavesX) * w8 + blockIdx.x * kTileWavesX + wv % kTileWavesX;
  const uint32_t gx = (t8 % w8) * 8u + (lane & 7u), gy = (t8 / w8) * 8u + (lane >> 3);
  // the tile index waits in LDS across the bounce loop: the epilogue re-derives the output coordinates from it
  // instead of keeping (spilling) them
  if (lane == 0) s_tile8[wv] = t8;
  m33 view;
  view.m11 = P.v11; view.m12 = P.v12; view.m13 = P.v13;
  view.m21 = P.v21; view.m22 = P.v22; view.m23 = P.v23;
  view.m31 = P.v31; view.m32 = P.v32; view.m33 = P.v33;
  const v3 eye = mk(P.eye_x, P.eye_y, P.eye_z);

  if constexpr (MODE == kModeSsaaLanes || MODE == kModeSsaaChunks)
  {
    // Render.cpp:174-194 with the sample loops (181-187) across lanes.  sampleNum 2 / 4: lane = ss^2 q + (ss sx + sy) of
    // pixel q of the wave's bw x bw block; sampleNum >= 8: the wave is one pixel, its ss^2 samples taken 64 at a time
    // (lane = sample - 64 chunk).  Trace index (pixel - p_begin) ss^2 + ss sx + sy, as the reference draws them; the
    // pixel's samples are summed in the reference's order (finColor += trace) through the wave's LDS slot, chunk by
    // chunk onto a running sum kept there (s_out words 192-194).
    constexpr bool CHUNKS = MODE == kModeSsaaChunks;
    const uint32_t ss = (uint32_t)P.ss, ss2 = ss * ss, bw = CHUNKS ? 1u : ss_lane_block(P.ss);
    const uint32_t nchunk = CHUNKS ? (ss2 + 63) / 64 : 1;
    float *sm = reinterpret_cast<float *>(s_out[wv]);
    for (uint32_t chunk = 0; chunk < nchunk; ++chunk)
    {
      // every chunk derives its lanes' state afresh (a laundered lane id and frame parameters), so nothing of it is
      // hoisted out of the chunk loop and held across the bounce loop
      uint32_t lane = threadIdx.x & 63u;
      if constexpr (CHUNKS) asm volatile("" : "+v"(lane));
#ifdef RFX_LAUNDER_PARAMS
      const FrameParams &P = kernarg_params<CHUNKS>();
#endif
      const uint32_t q = bw == 1 ? 0 : lane / ss2, kk = bw == 1 ? 64 * chunk + lane : lane - q * ss2;
      const uint32_t sx = kk / ss, sy = kk - sx * ss;
      const uint32_t lx = (t8 % w8) * bw + q % bw, ly = (t8 / w8) * bw + q / bw;
      const uint32_t x = lx;
      const uint32_t y = P.nranks > 1 ? strip_row_to_y(ly, P) : ly + P.row0;
      const uint64_t p = (uint64_t)y * P.W + x;
      const bool valid = lx < P.W && ly < P.grid_rows && p >= P.p_begin && p < P.p_end && kk < ss2;
      const uint64_t pr = p - P.p_begin;
      float rndx = 0.0f, rndy = 0.0f;
      if (P.additive && valid)                                                     // Render.cpp:177-178
      {
        const uint32_t s1 = lcg_jump(P.jitter_seed, 2 * pr + 1);
        rndx = (float)lcg_out(s1) / (float)0x7FFF;
        rndy = (float)lcg_out(lcg_step(s1)) / (float)0x7FFF;
      }
      const float ssf = (float)(int)ss;
      // float(0) / ss == +0 exactly, so the first sample's offsets need no division
      const float ox = sx ? (float)(int)sx / ssf : 0.0f, oy = sy ? (float)(int)sy / ssf : 0.0f;
      const float rx = (float)x - P.wh, ry = (float)y - P.hh;                     // Render.cpp:152-153
      const v3 ray = mmul(view, mk(rx + ox + rndx, ry + oy + rndy, P.rz));         // Render.cpp:183-184
      v3 rd = mk(0.0f, 0.0f, 0.0f);
      if (valid) rd = load_rd(P, pr * (uint64_t)ss2 + kk);
      // the tile's per-view masks (prim_cull_kernel<., true>; chunks: the pixel's closest-hit mask, every chunk)
      const uint64_t *pm = RFX_PRIM_LANES && SMALL && CULL && !STATS && P.prim_mask
                               ? P.prim_mask + (size_t)kPrimStride * t8 : nullptr;
      const col c = trace<STATS, CULL, MANYL, SMALL, PLANES, ONEL>(S, eye, ray, P.depth, rd, lut, cnt, valid, pm,
                                                                  P.prim_shadow != 0);
      {
#ifdef RFX_LAUNDER_PARAMS
        const FrameParams &P = kernarg_params();  // shadows the by-value parameter: re-read after the bounce loop
#endif
        // the lane's pixel again, from the tile index in LDS and a fresh lane id (not kept live across the bounce loop)
        const uint32_t t8e = ((volatile uint32_t *)s_tile8)[wv];
        uint32_t le = lane;
        asm volatile("" : "+v"(le));
        const uint32_t ss = (uint32_t)P.ss, ss2 = ss * ss, bw = CHUNKS ? 1u : ss_lane_block(P.ss);
        const uint32_t q = bw == 1 ? 0 : le / ss2, kk = bw == 1 ? 64 * chunk + le : le - q * ss2;
        const uint32_t lx = (t8e % w8) * bw + q % bw, ly = (t8e / w8) * bw + q / bw;
        const uint32_t x = lx;
        const uint32_t y = P.nranks > 1 ? strip_row_to_y(ly, P) : ly + P.row0;
        const uint64_t p = (uint64_t)y * P.W + x;
        const bool pvalid = lx < P.W && ly < P.grid_rows && p >= P.p_begin && p < P.p_end;
        sm[3 * le] = c.r;
        sm[3 * le + 1] = c.g;
        sm[3 * le + 2] = c.b;
        __builtin_amdgcn_wave_barrier();
        const uint32_t first = bw == 1 ? 64 * chunk : 0;  // the pixel's sum starts at its sample 0
#if RFX_SSAA_CHANNEL_SUM
        // Color::operator+= adds the three channels independently (r += c.r, ...), so the pixel's first three lanes
        // each run one channel's chain of adds in the reference's order -- a third of the serial sum one lane ran.
        // The final channels wait in the pixel's first sample's words (only lane ch reads word 3 lead + ch), where the
        // pixel's first lane assembles the ARGB word.
        if (ss2 >= 3)
        {
          const uint32_t lead = bw == 1 ? 0u : le - kk, ch = le - lead;  // kk: the lane's sample in its pixel
          const uint32_t n = min(ss2 - first, bw == 1 ? 64u : ss2);
          const bool last = first + n >= ss2;
          if (pvalid && ch < 3)
          {
            float fc = first ? sm[192 + ch] : 0.0f;
#pragma unroll 8
            for (uint32_t j = 0; j < n; ++j) fc = fc + sm[3 * (lead + j) + ch];
            if (!last)
              sm[192 + ch] = fc;  // more chunks to come: the running sum waits in LDS
            else
            {
              const float sq = (float)(int)ss2;                                    // Render.cpp:189
              if (fabsf(sq) > kVerySmall) fc = fc / sq;
              const size_t o = (size_t)(P.nranks > 1 ? ly : y) * P.W + x;
              float *d = P.img + o * 3;
              if (P.accumulate) fc = d[ch] + fc;                                   // Render.cpp:191-194
              d[ch] = fc;
              sm[3 * lead + ch] = fc;
            }
          }
          __builtin_amdgcn_wave_barrier();
          if (last && pvalid && ch == 0 && P.argb)                                 // Render::copyImage
            P.argb[(size_t)(P.nranks > 1 ? ly : y) * P.W + x] = argb(mkc(sm[3 * lead], sm[3 * lead + 1], sm[3 * lead + 2]));
        }
        else
#endif
        if (pvalid && (bw == 1 ? le == 0 : kk == 0))
        {
          col fin = first ? mkc(sm[192], sm[193], sm[194]) : mkc(0.0f, 0.0f, 0.0f);
          const uint32_t n = min(ss2 - first, bw == 1 ? 64u : ss2);
          for (uint32_t j = 0; j < n; ++j)
            fin = cadd(fin, mkc(sm[3 * (le + j)], sm[3 * (le + j) + 1], sm[3 * (le + j) + 2]));
          if (first + n < ss2)  // more chunks to come: the running sum waits in LDS
          {
            sm[192] = fin.r;
            sm[193] = fin.g;
            sm[194] = fin.b;
          }
          else
          {
            const float sq = (float)(int)ss2;                                      // Render.cpp:189
            if (fabsf(sq) > kVerySmall) fin = mkc(fin.r / sq, fin.g / sq, fin.b / sq);
            const size_t o = (size_t)(P.nranks > 1 ? ly : y) * P.W + x;
            float *d = P.img + o * 3;
            if (P.accumulate) fin = mkc(d[0] + fin.r, d[1] + fin.g, d[2] + fin.b);  // Render.cpp:191-194
            d[0] = fin.r; d[1] = fin.g; d[2] = fin.b;
            if (P.argb) P.argb[o] = argb(fin);                                       // Render::copyImage
          }
        }
        __builtin_amdgcn_wave_barrier();
        if (chunk + 1 == nchunk)
        {
          if (P.tile_cost && __lane_id() == 0) P.tile_cost[t8e] = clock32() - s_clk0;
          RFX_WAVE_T1(t8e);
        }
      }
    }
  }
  else if constexpr (MODE == kModeBlock)
  {
    // block preview (Render.cpp:158-172): only block corners inside the cursor span are traced;
    // trace order = raster order of corners, so corner (cx, cy) is trace cy * bw + cx.
    const uint32_t n = (uint32_t)(-P.ss);
    const uint32_t bw = (P.W + n - 1) / n, bh = (P.H + n - 1) / n;
    const uint32_t cx = gx, cy = gy + P.row0;
    const uint32_t x = cx * n, y = cy * n;
    const uint64_t p = (uint64_t)y * P.W + x;
    const bool valid = gy < P.grid_rows && cx < bw && cy < bh && p >= P.p_begin && p < P.p_end;
    const v3 ray = mmul(view, mk((float)x - P.wh, (float)y - P.hh, P.rz));
    v3 rd = mk(0.0f, 0.0f, 0.0f);
    if (valid) rd = load_rd(P, (uint64_t)cy * bw + cx - P.trace_base);
    const col c = trace<STATS, CULL, MANYL, SMALL, PLANES, ONEL>(S, eye, ray, P.depth, rd, lut, cnt, valid);
    if (valid)
    {
      const uint32_t ex = min(P.W, x + n), ey = min(P.H, y + n);
      const uint32_t a = argb(c);
      for (uint32_t qy = y; qy < ey; ++qy)
        for (uint32_t qx = x; qx < ex; ++qx)
        {
          float *d = P.img + ((size_t)qy * P.W + qx) * 3;
          d[0] = c.r; d[1] = c.g; d[2] = c.b;
          if (P.argb) P.argb[(size_t)qy * P.W + qx] = a;
        }
    }
  }
  else
  {
    const uint32_t x = gx;
    const uint32_t y = P.nranks > 1 ? strip_row_to_y(gy, P) : gy + P.row0;
    const uint64_t p = (uint64_t)y * P.W + x;
    const bool valid = gx < P.W && gy < P.grid_rows && p >= P.p_begin && p < P.p_end;
    const uint64_t pr = p - P.p_begin;
    const float rx = (float)x - P.wh, ry = (float)y - P.hh;                       // Render.cpp:152-153
    col out;
    bool parked = false;
    if constexpr (MODE == kModePlain)
    {
      // Render.cpp:183 with ssx = ssy = 0, sampleNum = 1, no jitter: float(0) / 1 == +0, rnd == 0
      const v3 ray = mmul(view, mk(rx + 0.0f + 0.0f, ry + 0.0f + 0.0f, P.rz));
      v3 rd = mk(0.0f, 0.0f, 0.0f);
      if (valid) rd = load_rd(P, pr);
      const ParkTile park{P.park_after, P.queue, P.queue_count, P, wv, w8};
      const uint64_t *pm_tile = (SMALL || RFX_PRIM_LARGE) && CULL && !STATS && P.prim_mask
                                    ? P.prim_mask + (size_t)(SMALL ? kPrimStride : kPrimLargeStride) * t8 : nullptr;
      const col c = trace_from<STATS, CULL, MANYL, SMALL, PLANES, PARK, ParkTile, ONEL>(S, eye, ray, mkc(1.0f, 1.0f, 1.0f),
                                                                  mkc(0.0f, 0.0f, 0.0f), 0, P.depth, rd, lut, cnt,
                                                                  valid, park, parked, pm_tile);
      out = cadd(mkc(0.0f, 0.0f, 0.0f), c);                                      // Render.cpp:185 (/ 1.0f exact)
    }
    else
    {
      // SSAA / additive (Render.cpp:174-194): each lane runs its pixel's ss x ss traces in turn
#ifdef RFX_SSAA_LDS_STATE
      // Experiment (round 4, off: +3.7% on the screenshot frame, interleaved A/B).  The per-lane state that outlives
      // each sample's bounce loop -- the running sum and the additive jitter -- waits in the wave's epilogue staging
      // slot (s_out: 192 words of sum, 64 of jitter), and the pixel's coordinates are re-derived from the tile index in
      // LDS for every sample, so the bounce loop runs with fewer live values (22 -> 9 VGPR spills, small scenes).
      uint32_t *slot = s_out[wv];
      uint32_t jit = 0;
      if (P.additive && valid)                                                     // Render.cpp:177-178
      {
        const uint32_t s1 = lcg_jump(P.jitter_seed, 2 * pr + 1);
        jit = lcg_out(s1) | lcg_out(lcg_step(s1)) << 16;  // two 15-bit draws
      }
      slot[192 + lane] = jit;
      slot[3 * lane] = 0u;  // +0.0f: Color finColor(0, 0, 0)
      slot[3 * lane + 1] = 0u;
      slot[3 * lane + 2] = 0u;
      const int ss = P.ss;
      const float ssf = (float)ss;
      for (int sx = 0; sx < ss; ++sx)                                              // Render.cpp:181-187
        for (int sy = 0; sy < ss; ++sy)
        {
          const FrameParams &P = kernarg_params();  // shadows the by-value parameter: reloaded per sample
          m33 view;
          view.m11 = P.v11; view.m12 = P.v12; view.m13 = P.v13;
          view.m21 = P.v21; view.m22 = P.v22; view.m23 = P.v23;
          view.m31 = P.v31; view.m32 = P.v32; view.m33 = P.v33;
          const v3 eye = mk(P.eye_x, P.eye_y, P.eye_z);
          const uint32_t t8s = ((volatile uint32_t *)s_tile8)[wv];
          uint32_t ls = lane;
          asm volatile("" : "+v"(ls));  // a fresh lane value: the coordinates are recomputed, not kept live
          const uint32_t sgx = (t8s % w8) * 8u + (ls & 7u), sgy = (t8s / w8) * 8u + (ls >> 3);
          const uint32_t sy_ = P.nranks > 1 ? strip_row_to_y(sgy, P) : sgy + P.row0;
          const uint64_t sp = (uint64_t)sy_ * P.W + sgx;
          const bool svalid = sgx < P.W && sgy < P.grid_rows && sp >= P.p_begin && sp < P.p_end;
          const uint32_t jw = ((volatile uint32_t *)slot)[192 + ls];
          const float rndx = P.additive ? (float)(jw & 0xFFFFu) / (float)0x7FFF : 0.0f;
          const float rndy = P.additive ? (float)(jw >> 16) / (float)0x7FFF : 0.0f;
          // float(0) / ss == +0 exactly, so the first sample's offsets need no division
          const float ox = sx ? (float)sx / ssf : 0.0f, oy = sy ? (float)sy / ssf : 0.0f;
          v3 ray = mk((float)sgx - P.wh + ox + rndx, (float)sy_ - P.hh + oy + rndy, P.rz);
          ray = mmul(view, ray);
          v3 rd = mk(0.0f, 0.0f, 0.0f);
          if (svalid) rd = load_rd(P, (sp - P.p_begin) * (uint64_t)(ss * ss) + (uint64_t)(sx * ss + sy));
          // the tile's per-view masks cover every sample's primary rays (prim_cull_kernel)
          const uint64_t *pm = RFX_PRIM_SSAA && SMALL && CULL && !STATS && P.prim_mask
                                   ? P.prim_mask + (size_t)kPrimStride * t8s : nullptr;
          const col c = trace<STATS, CULL, MANYL, SMALL, PLANES>(S, eye, ray, P.depth, rd, lut, cnt, svalid, pm,
                                                                 P.prim_shadow != 0);
          float *f = reinterpret_cast<float *>(slot) + 3 * ls;
          f[0] = f[0] + c.r;
          f[1] = f[1] + c.g;
          f[2] = f[2] + c.b;
        }
      const float *f = reinterpret_cast<const float *>(slot) + 3 * lane;
      col fin = mkc(f[0], f[1], f[2]);
      if (ss != 1)                                                                 // Render.cpp:189 (x / 1.0f == x)
      {
        const float sq = (float)(ss * ss);
        if (fabsf(sq) > kVerySmall) fin = mkc(fin.r / sq, fin.g / sq, fin.b / sq);
      }
      out = fin;
#else
      float rndx = 0.0f, rndy = 0.0f;
      if (P.additive && valid)                                                     // Render.cpp:177-178
      {
        const uint32_t s1 = lcg_jump(P.jitter_seed, 2 * pr + 1);
        rndx = (float)lcg_out(s1) / (float)0x7FFF;
        rndy = (float)lcg_out(lcg_step(s1)) / (float)0x7FFF;
      }
      const int ss = P.ss;
      const float ssf = (float)ss;
      col fin = mkc(0.0f, 0.0f, 0.0f);
      for (int sx = 0; sx < ss; ++sx)                                              // Render.cpp:181-187
        for (int sy = 0; sy < ss; ++sy)
        {
          // float(0) / ss == +0 exactly, so the first sample's offsets need no division
          const float ox = sx ? (float)sx / ssf : 0.0f, oy = sy ? (float)sy / ssf : 0.0f;
          v3 ray = mk(rx + ox + rndx, ry + oy + rndy, P.rz);
          ray = mmul(view, ray);
          v3 rd = mk(0.0f, 0.0f, 0.0f);
          if (valid) rd = load_rd(P, pr * (uint64_t)(ss * ss) + (uint64_t)(sx * ss + sy));
          const uint64_t *pm = RFX_PRIM_SSAA && SMALL && CULL && !STATS && P.prim_mask
                                   ? P.prim_mask + (size_t)kPrimStride * t8 : nullptr;
          fin = cadd(fin, trace<STATS, CULL, MANYL, SMALL, PLANES>(S, eye, ray, P.depth, rd, lut, cnt, valid, pm,
                                                                   P.prim_shadow != 0));
        }
      if (ss != 1)                                                                 // Render.cpp:189 (x / 1.0f == x)
      {
        const float sq = (float)(ss * ss);
        if (fabsf(sq) > kVerySmall) fin = mkc(fin.r / sq, fin.g / sq, fin.b / sq);
      }
      out = fin;
#endif
    }
    // output coordinates again, from the tile index in LDS (volatile: re-read, not kept live)
#ifdef RFX_LAUNDER_PARAMS
    const FrameParams &P = kernarg_params();  // shadows the by-value parameter: re-read after the bounce loop
#endif
    const uint32_t t8e = ((volatile uint32_t *)s_tile8)[wv];
    uint32_t le = lane;
    asm volatile("" : "+v"(le));  // a fresh lane value: its row/column are recomputed, not kept live
    const uint32_t x0e = (t8e % w8) * 8u, row0e = (t8e / w8) * 8u + (P.nranks > 1 ? 0u : P.row0);
    const uint32_t xe = x0e + (le & 7u), rowe = row0e + (le >> 3), wslot = wv;
    if (MODE == kModeSsaa && P.accumulate && valid)                                  // Render.cpp:191-194
    {
      const float *d = P.img + ((size_t)rowe * P.W + xe) * 3;
      out = mkc(d[0] + out.r, d[1] + out.g, d[2] + out.b);
    }
    const bool staged = (P.W & 3u) == 0 &&
                        ((reinterpret_cast<uintptr_t>(P.img) | reinterpret_cast<uintptr_t>(P.argb)) & 15u) == 0 &&
                        __builtin_amdgcn_ballot_w64(valid && !parked) == ~0ull;
    if (staged)
      store_wave_tile(P, x0e, row0e, out, le, wslot);  // Render::copyImage too
    else if (valid && !parked)
    {
      const size_t o = (size_t)rowe * P.W + xe;
      float *d = P.img + o * 3;
      d[0] = out.r; d[1] = out.g; d[2] = out.b;
      if (P.argb) P.argb[o] = argb(out);                                           // Render::copyImage
    }
    if (P.tile_cost && __lane_id() == 0)  // per wave tile, from its output coordinates
      P.tile_cost[(P.nranks > 1 ? rowe : rowe - P.row0) / 8u * P.tiles_x + xe / 8u] = clock32() - s_clk0;
    RFX_WAVE_T1(t8e);
  }
  flush_counters<STATS>(P, cnt);
  RFX_PROF_FLUSH();

}

// Per-view masks of a small scene's plain or SSAA frame (FrameParams::prim_mask), kPrimStride words per wave tile t8:
// [0] the cull mask of the tile's primary bundle, [1 + q] that of its primary hits' shadow rays toward light q
// for every randDir (q < kPrimLights).  Wave t8 builds its tile's primary rays exactly as trace_kernel does (same
// tile mapping, same validity), their bundle (one origin: the eye) and cull mask -- with the triangle footprint
// test, which the trace kernel could not afford per segment -- then the primary hits with the same closest-hit
// code and that mask, and per light the bundle of all shadow rays of the facing lanes (make_bundle_ball).  The
// masks depend only on the view (camera, frame geometry, scene), so the host builds them once per view.
// LANES: the tiles of a kModeSsaaLanes frame (sampleNum 1 jittered, 2, 4, 8): wave t8 covers bw x bw pixels, one sample
// per lane, exactly as trace_kernel's lanes branch maps them; its masks cover the lanes' own rays (jittered: each lane's
// unit jitter square), so the shadow masks need one primary hit per lane.  A kModeSsaaChunks frame (sampleNum > 8, the
// wave is one pixel): the closest-hit mask of the pixel's whole sample rectangle, which every chunk of its samples reuses;
// no shadow masks (they would need the primary hit of every sample).
template <bool PLANES, bool LANES = false>
__global__ RFX_TRACE_BOUNDS void prim_cull_kernel(DevScene S, FrameParams P, uint64_t *masks)
{
  stage_small_scene(S);
  __syncthreads();
  const Tabs<true> T{S};
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t w8 = kTileWavesX * gridDim.x;
  const uint32_t t8 = (blockIdx.y * kTileWavesY + wv / kTileWavesX) * w8 + blockIdx.x * kTileWavesX + wv % kTileWavesX;
  uint32_t gx, gy, kk = 0;
  float lox = 0.0f, loy = 0.0f;  // LANES: the lane's sample offsets (Render.cpp:183), as trace_kernel forms them
  const bool chunks = LANES && P.ss > 8;
  if constexpr (LANES)
  {
    const uint32_t ss = (uint32_t)P.ss, ss2 = ss * ss, bw = ss_lane_block(P.ss);
    const uint32_t q = bw == 1 ? 0 : lane / ss2;
    kk = chunks ? 0 : bw == 1 ? lane : lane - q * ss2;
    const uint32_t sx = kk / ss, sy = kk - sx * ss;
    gx = (t8 % w8) * bw + q % bw;
    gy = (t8 / w8) * bw + q / bw;
    const float ssf = (float)(int)ss;
    lox = sx ? (float)(int)sx / ssf : 0.0f;
    loy = sy ? (float)(int)sy / ssf : 0.0f;
  }
  else
  {
    gx = (t8 % w8) * 8u + (lane & 7u);
    gy = (t8 / w8) * 8u + (lane >> 3);
  }
  const uint32_t x = gx;
  const uint32_t y = P.nranks > 1 ? strip_row_to_y(gy, P) : gy + P.row0;
  const uint64_t p = (uint64_t)y * P.W + x;
  const bool valid = gx < P.W && gy < P.grid_rows && p >= P.p_begin && p < P.p_end && P.depth > 0 &&
                     (!LANES || kk < (uint32_t)(P.ss * P.ss));
  m33 view;
  view.m11 = P.v11; view.m12 = P.v12; view.m13 = P.v13;
  view.m21 = P.v21; view.m22 = P.v22; view.m23 = P.v23;
  view.m31 = P.v31; view.m32 = P.v32; view.m33 = P.v33;
  const v3 eye = mk(P.eye_x, P.eye_y, P.eye_z);
  const float rx = (float)x - P.wh, ry = (float)y - P.hh;                       // Render.cpp:152-153
  uint64_t *out = masks + (size_t)kPrimStride * t8;
  // one sample per pixel without jitter: the plain rays themselves; SSAA and jittered (additive) frames: every ray of
  // the pixel's sample rectangle [rx, rx + omax] x [ry, ry + omax] (Render.cpp:177-183: offsets (ss - 1) / ss at most,
  // plus a jitter of at most 1 in additive frames), through its four corners
  const int ss = P.ss;
  const bool exact = (LANES || ss == 1) && !P.additive && !chunks;
  uint64_t om = 0;
  if (__ballot(valid))
  {
    Bundle B;
    if (exact)  // as trace_kernel (plain: rx + 0 + 0; lanes: rx + float(sx) / ss + 0)
      B = make_bundle(eye, mmul(view, mk(rx + lox + 0.0f, ry + loy + 0.0f, P.rz)), valid);
    else
    {
      // LANES: the lane's jitter square; else (and chunks) the pixel's sample rectangle
      const float bx = rx + lox, by = ry + loy;
      const float omax = LANES && !chunks ? 1.0f : (float)(ss - 1) / (float)ss + (P.additive ? 1.0f : 0.0f);
      const v3 q[4] = {mmul(view, mk(bx, by, P.rz)), mmul(view, mk(bx + omax, by, P.rz)),
                       mmul(view, mk(bx, by + omax, P.rz)), mmul(view, mk(bx + omax, by + omax, P.rz))};
      B = make_bundle_quad(eye, q, valid);
    }
    om = B.ok ? cull_small<true>(T.cull(), S.cull_valid, B, S.cull_tri) : S.cull_valid;
  }
  if (lane == 0) out[0] = om;
  // the primary hits of every sample, as trace_from's first segment finds them with this mask (Scene.cpp:86-106), and
  // per light the union of their shadow bundles' masks.  Jittered frames: the hits are not known ahead, no shadow masks
  // (FrameParams::prim_shadow; the trace kernel builds those bundles itself).
  const int nl = P.additive || chunks ? 0 : min(S.n_light, kPrimLights);
  uint64_t sm[kPrimLights] = {0, 0, 0, 0};
  const float ssf = (float)ss;
  const int nss = LANES ? 1 : ss;  // LANES: the lane's one sample
  for (int sx = 0; nl > 0 && sx < nss; ++sx)
    for (int sy = 0; sy < nss; ++sy)
    {
      // the sample's ray exactly as trace_kernel forms it (plain: rx + 0 + 0; SSAA: rx + float(sx) / ss + 0)
      const float ox = LANES ? lox : sx ? (float)sx / ssf : 0.0f, oy = LANES ? loy : sy ? (float)sy / ssf : 0.0f;
      const v3 ray = mmul(view, mk(rx + ox + 0.0f, ry + oy + 0.0f, P.rz));
      Cnt cnt;
      Hit h;
      if (valid) closest_hit_small<false, PLANES>(S, eye, ray, om, h, cnt);
      else h.obj = -1;
      const bool hit = valid && h.obj >= 0;
      v3 drop = eye, norm = mk(0.0f, 0.0f, 0.0f);
      if (hit)
      {
        drop = add(eye, mul(ray, h.t));
        if (h.kind == 0)
        {
          const SphereGeo g = T.sph_geo(h.i);
          norm = sub(drop, mk(g.cx, g.cy, g.cz));                                // Sphere.cpp:67
        }
        else if (!PLANES || h.kind == 1)
        {
          const TriShade sh = T.tri_shade(h.i);
          norm = mk(sh.nx, sh.ny, sh.nz);
        }
        else
        {
          const PlaneGeo g = S.pln_geo[h.i];
          norm = mk(g.nx, g.ny, g.nz);                                           // Plane.cpp:58-59
        }
      }
      for (int q = 0; q < nl; ++q)
      {
        const LightRec L = S.lights[q];
        const v3 dtl = sub(mk(L.ox, L.oy, L.oz), drop);
        const bool facing = hit && dot(dtl, norm) > kVerySmall;                  // Scene.cpp:125
        if (__ballot(facing))
        {
          const Bundle SB = make_bundle_ball(drop, dtl, L.radius, facing);
          sm[q] |= SB.ok ? cull_small(T.cull(), S.cull_valid, SB) : S.cull_valid;
        }
      }
    }
  for (int q = 0; q < nl; ++q)
    if (lane == 0) out[1 + q] = sm[q];
}

// Per-view chunk lists of a large scene's plain frame (FrameParams::prim_mask, kPrimLargeStride words per wave tile t8):
// the primary bundle of the tile -- the same rays, validity and bundle as trace_from's first segment -- and, when it is
// narrow enough for the chunk path (closest_hit), its chunk cull and the sphere cull of each kept chunk, stored as a
// list the trace kernel walks instead of culling again; the triangle cull too.  More than kPrimLargeChunks kept chunks,
// more than 64 triangles, or a bundle the chunk path would not take: kPrimLargeNone (the tile culls per launch).
template <int UNUSED = 0>  // a template, as every kernel this header defines: one definition across the TUs
__global__ RFX_TRACE_BOUNDS void prim_cull_large_kernel(DevScene S, FrameParams P, uint64_t *masks)
{
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t w8 = kTileWavesX * gridDim.x;
  const uint32_t t8 = (blockIdx.y * kTileWavesY + wv / kTileWavesX) * w8 + blockIdx.x * kTileWavesX + wv % kTileWavesX;
  const uint32_t gx = (t8 % w8) * 8u + (lane & 7u), gy = (t8 / w8) * 8u + (lane >> 3);
  const uint32_t x = gx;
  const uint32_t y = P.nranks > 1 ? strip_row_to_y(gy, P) : gy + P.row0;
  const uint64_t p = (uint64_t)y * P.W + x;
  const bool valid = gx < P.W && gy < P.grid_rows && p >= P.p_begin && p < P.p_end && P.depth > 0;
  m33 view;
  view.m11 = P.v11; view.m12 = P.v12; view.m13 = P.v13;
  view.m21 = P.v21; view.m22 = P.v22; view.m23 = P.v23;
  view.m31 = P.v31; view.m32 = P.v32; view.m33 = P.v33;
  const v3 eye = mk(P.eye_x, P.eye_y, P.eye_z);
  const float rx = (float)x - P.wh, ry = (float)y - P.hh;                       // Render.cpp:152-153
  const v3 ray = mmul(view, mk(rx + 0.0f + 0.0f, ry + 0.0f + 0.0f, P.rz));     // as trace_kernel (plain)
  uint64_t *out = masks + (size_t)kPrimLargeStride * t8;
  uint64_t w[kPrimLargeStride];
#pragma unroll
  for (int i = 0; i < kPrimLargeStride; ++i) w[i] = 0;
  bool listed = false;
  if (__ballot(valid) && S.n_tri <= 64 && S.n_chunk <= 64)
  {
    const Bundle B = make_bundle(eye, ray, valid);
    // the bundles closest_hit takes through the chunk path (the others walk the BVH per lane)
    if (B.ok && (S.bvh == nullptr || B.cosa > kNarrowBundleCos))
    {
      const uint64_t cm = cull_chunk(S.chunk_bound, 0, S.n_chunk, B);
      listed = __popcll(cm) <= kPrimLargeChunks;
      if (listed)
      {
        w[0] = (uint64_t)__popcll(cm);
        w[2] = cm;
        int e = 4;
        for (uint64_t c = cm; c; c &= c - 1ull)
        {
          const int first = 64 * __builtin_ctzll(c);
          w[e++] = cull_chunk(S.bound, first, min(64, S.n_sph - first), B);
        }
        if (S.n_tri > 0) w[1] = cull_chunk(S.bound, S.n_sph, S.n_tri, B);
      }
    }
  }
  if (!listed) w[0] = kPrimLargeNone;
  if (lane == 0)
  {
#pragma unroll
    for (int i = 0; i < kPrimLargeStride; ++i) out[i] = w[i];
  }
}

// The parked traces (rfx_types.h QRay) of a plain-pixel launch resumed in packed waves: each wave claims 64
// queue entries at a time (one atomic), runs the rest of their bounce loops and writes their pixels exactly
// as the trace kernel would have (Render.cpp:185 and the ARGB epilogue).  Waves exit once the queue is
// drained; the queue holds traces from all over the frame, so waves no longer idle on lanes whose traces
// ended (the trace kernel's tail of 1-2 live lanes per wave at depth 3+).
// The bounce kernel's lanes (ray regrouping, large scenes) take a new parked trace as soon as theirs ends: at the end of
// every segment a lane whose trace ended writes its pixel (Render.cpp:185), and the wave's idle lanes claim the next
// queue entries with one atomic -- so a wave stays full while its traces end at different segments, until the queue
// is drained.  Each trace resumes from its own parked state, so every float op is the one the trace kernel would have
// run.
__shared__ uint32_t s_refill_out[kWgWaves][64];  // per lane: the output pixel of its trace in flight (~0u: none)

template <class NS = BvhGlobal>
struct Refill {
  const FrameParams &P;
  uint32_t n;             // queue entries
  uint32_t *outs;         // LDS: the output pixel of each lane's trace in flight (~0u: none), 64 per wave
  NS ns;                  // where the BVH walkers find the nodes
  mutable bool drained;   // wave-uniform: every entry has been claimed
  static constexpr bool kRefill = true;
  __device__ __forceinline__ void ids(uint32_t &t, uint32_t &o) const { t = o = 0u; }  // (never parks)
  __device__ __forceinline__ uint32_t *keys() const { return nullptr; }
  __device__ __forceinline__ const NS &bvh() const { return ns; }
  __device__ __forceinline__ void refill(bool &alive, v3 &origin, v3 &ray, col &mulc, col &pix, int &refl, v3 &rd) const
  {
    const uint32_t lane = __lane_id();
    uint32_t out = outs[lane];
    if (!alive && out != ~0u)
    {
      const col o = cadd(mkc(0.0f, 0.0f, 0.0f), pix);                               // Render.cpp:185
      float *d = P.img + (size_t)out * 3;
      d[0] = o.r; d[1] = o.g; d[2] = o.b;
      if (P.argb) P.argb[out] = argb(o);
      out = ~0u;
    }
    const uint64_t idle = __ballot(out == ~0u);
    if (idle && !drained)
    {
      const int first = __ffsll((long long)idle) - 1;
      const uint32_t k = (uint32_t)__popcll(idle);
      uint32_t base = 0;
      if (lane == (uint32_t)first) base = atomicAdd(P.queue_next, k);
      base = __builtin_amdgcn_readlane(base, first);
      if (base + k >= n) drained = true;
      const uint32_t slot = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
      if (out == ~0u && slot < n)
      {
        const QRay q = P.queue[P.queue_order ? P.queue_order[slot] : slot];
        origin = mk(q.ox, q.oy, q.oz);
        ray = mk(q.dx, q.dy, q.dz);
        mulc = mkc(q.mr, q.mg, q.mb);
        pix = mkc(q.pr, q.pg, q.pb);
        refl = (int)q.refl;
        rd = load_rd(P, q.trace);
        out = q.out;
        alive = refl < P.depth;
      }
    }
    outs[lane] = out;
  }
};

template <int CFG>
__global__ RFX_TRACE_BOUNDS void bounce_kernel(DevScene S, FrameParams P)
{
  static_assert(kKernargSig<decltype(&bounce_kernel<CFG>)>, "launder_scene / kernarg_params layout");
  constexpr bool CULL = (CFG & kCfgCull) != 0, MANYL = (CFG & kCfgManyLights) != 0, SMALL = (CFG & kCfgSmall) != 0;
  constexpr bool PLANES = (CFG & kCfgPlanes) != 0;
  __shared__ float lut[256];
  for (uint32_t i = threadIdx.x; i < 256; i += kWgThreads) lut[i] = (float)i / 255.0f;  // Color.cpp:11-13
  stage_powf_tables();
  if constexpr (SMALL) stage_small_scene(S);
  __syncthreads();
  Cnt cnt;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s_refill_out[wv][__lane_id()] = ~0u;
  const Refill<> rf{P, *P.queue_count, s_refill_out[wv], BvhGlobal{}, false};
  bool alive = false;
  v3 origin = mk(0.0f, 0.0f, 0.0f), ray = origin, rd = origin;
  col mulc = mkc(0.0f, 0.0f, 0.0f), pix = mulc;
  int refl = 0;
  rf.refill(alive, origin, ray, mulc, pix, refl, rd);  // the wave's first 64 traces
  RFX_WAVE_T0();
  bool parked;
  (void)trace_from<false, CULL, MANYL, SMALL, PLANES, false, decltype(rf), (CFG & kCfgOneLight) != 0>(
      S, origin, ray, mulc, pix, refl, P.depth, rd, lut, cnt, alive, rf, parked);
  RFX_WAVE_T1(kBounceTimeBase + kWgWaves * blockIdx.x + wv);
}

// The bounce kernel with the BVH staged in LDS (RFX_LDS_BVH; large scenes whose nodes fit): one workgroup of
// kLdsBvhThreads threads per CU copies the node boxes (48 B each) and links + margin terms (8 B, DevScene::bvh_aux)
// into its LDS, then its 16 waves take parked traces as bounce_kernel's do -- the walkers' node fetches become LDS
// reads instead of L2 round trips.  Dynamic LDS: lds_bvh_bytes(n_bvh) (rfx_types.h).
template <int CFG>
__global__ __launch_bounds__(kLdsBvhThreads) __attribute__((amdgpu_waves_per_eu(4)))
void bounce_kernel_lds(DevScene S, FrameParams P)
{
  static_assert(kKernargSig<decltype(&bounce_kernel_lds<CFG>)>, "launder_scene / kernarg_params layout");
  constexpr bool CULL = (CFG & kCfgCull) != 0, MANYL = (CFG & kCfgManyLights) != 0, SMALL = (CFG & kCfgSmall) != 0;
  constexpr bool PLANES = (CFG & kCfgPlanes) != 0;
  static_assert(!SMALL, "large scenes only");
  extern __shared__ float4 s_dyn[];
  const int nn = S.n_bvh;
  float4 *box = s_dyn;
  uint2 *aux = reinterpret_cast<uint2 *>(box + 3 * nn);
  BvhSlot *stk = reinterpret_cast<BvhSlot *>(aux + nn);
  uint32_t *outs = reinterpret_cast<uint32_t *>(stk + kBvhStack * kLdsBvhThreads);
  __shared__ float lut[256];
  for (uint32_t i = threadIdx.x; i < 256; i += kLdsBvhThreads) lut[i] = (float)i / 255.0f;  // Color.cpp:11-13
  stage_powf_tables();
  const float4 *gb = reinterpret_cast<const float4 *>(S.bvh);
  const uint2 *ga = reinterpret_cast<const uint2 *>(S.bvh_aux);
  for (int i = (int)threadIdx.x; i < nn; i += kLdsBvhThreads)
  {
    box[3 * i] = gb[4 * i];
    box[3 * i + 1] = gb[4 * i + 1];
    box[3 * i + 2] = gb[4 * i + 2];
    aux[i] = ga[i];
  }
  __syncthreads();
  Cnt cnt;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  outs[64 * wv + __lane_id()] = ~0u;
  const Refill<BvhLds> rf{P, *P.queue_count, outs + 64 * wv, BvhLds{box, aux, stk, S.bvh_mstep}, false};
  bool alive = false;
  v3 origin = mk(0.0f, 0.0f, 0.0f), ray = origin, rd = origin;
  col mulc = mkc(0.0f, 0.0f, 0.0f), pix = mulc;
  int refl = 0;
  rf.refill(alive, origin, ray, mulc, pix, refl, rd);
  bool parked;
  (void)trace_from<false, CULL, MANYL, SMALL, PLANES, false, decltype(rf), (CFG & kCfgOneLight) != 0>(
      S, origin, ray, mulc, pix, refl, P.depth, rd, lut, cnt, alive, rf, parked);
}

// ------------------------------------------------------------- launch of one family (the rfx_trace_*.hip TUs)
template <bool STATS, int MODE, int CFG>
inline void launch_one(dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  if constexpr (!STATS || !(CFG & kCfgCull))  // the stats build never culls
    hipLaunchKernelGGL((trace_kernel<STATS, MODE, CFG>), grid, dim3(kWgThreads), 0, st, S, P);
}

template <bool STATS, int MODE>
inline void launch_cfg(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  if (cfg & kCfgOneLight)  // scenes with exactly one light: the culling configurations have unrolled light loops
  {
    switch (cfg & ~kCfgOneLight)
    {
      case 1: launch_one<STATS, MODE, 1 | kCfgOneLight>(grid, S, P, st); return;
      case 5: launch_one<STATS, MODE, 5 | kCfgOneLight>(grid, S, P, st); return;
      case 9: launch_one<STATS, MODE, 9 | kCfgOneLight>(grid, S, P, st); return;
      case 13: launch_one<STATS, MODE, 13 | kCfgOneLight>(grid, S, P, st); return;
      default: cfg &= ~kCfgOneLight;
    }
  }
  switch (cfg)
  {
    case 0: launch_one<STATS, MODE, 0>(grid, S, P, st); break;
    case 1: launch_one<STATS, MODE, 1>(grid, S, P, st); break;
    case 2: launch_one<STATS, MODE, 2>(grid, S, P, st); break;
    case 3: launch_one<STATS, MODE, 3>(grid, S, P, st); break;
    case 4: launch_one<STATS, MODE, 4>(grid, S, P, st); break;
    case 5: launch_one<STATS, MODE, 5>(grid, S, P, st); break;
    case 6: launch_one<STATS, MODE, 6>(grid, S, P, st); break;
    case 7: launch_one<STATS, MODE, 7>(grid, S, P, st); break;
    case 8: launch_one<STATS, MODE, 8>(grid, S, P, st); break;
    case 9: launch_one<STATS, MODE, 9>(grid, S, P, st); break;
    case 10: launch_one<STATS, MODE, 10>(grid, S, P, st); break;
    case 11: launch_one<STATS, MODE, 11>(grid, S, P, st); break;
    case 12: launch_one<STATS, MODE, 12>(grid, S, P, st); break;
    case 13: launch_one<STATS, MODE, 13>(grid, S, P, st); break;
    case 14: launch_one<STATS, MODE, 14>(grid, S, P, st); break;
    case 15: launch_one<STATS, MODE, 15>(grid, S, P, st); break;
  }
}

// one trace_kernel family (rfx_trace_<mode>_<stats>.hip)
#define RFX_DECLARE_TRACE_FAMILY(name) \
  void name(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
RFX_DECLARE_TRACE_FAMILY(launch_trace_plain_fast);
RFX_DECLARE_TRACE_FAMILY(launch_trace_plain_stats);
RFX_DECLARE_TRACE_FAMILY(launch_trace_ssaa_fast);
RFX_DECLARE_TRACE_FAMILY(launch_trace_ssaa_stats);
RFX_DECLARE_TRACE_FAMILY(launch_trace_lanes_fast);
RFX_DECLARE_TRACE_FAMILY(launch_trace_lanes_stats);
RFX_DECLARE_TRACE_FAMILY(launch_trace_chunks_fast);
RFX_DECLARE_TRACE_FAMILY(launch_trace_chunks_stats);
RFX_DECLARE_TRACE_FAMILY(launch_trace_block_fast);
RFX_DECLARE_TRACE_FAMILY(launch_trace_block_stats);
RFX_DECLARE_TRACE_FAMILY(launch_trace_plain_park);
RFX_DECLARE_TRACE_FAMILY(launch_bounce);

}  // namespace rfx
