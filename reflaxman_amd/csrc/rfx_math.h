// Float math of ReflaxMan's L0 value types, restated operation-for-operation so
// the device kernels (gfx950) and the host-side scene precompute produce the
// reference's exact IEEE results.  Compile with -ffp-contract=off and without
// fast-math: no FMA contraction, correctly rounded '/' and sqrtf, denormals kept.
//
// Citations: /root/reference/src/common/<file>:<line>.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RFX_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define RFX_HD static inline
#endif

#pragma clang fp contract(off)

namespace rfx {

// trace_math.h:17-18 (sqrtf(FLT_MIN) == 2^-63 exactly)
constexpr float kVerySmall = 1.0842021724855044e-19f;
constexpr float kDelta = 0.0001f;
constexpr float kFltEpsilon = 1.1920928955078125e-07f;
constexpr float kFltMax = 3.402823466e+38f;

// Correctly rounded f32 square root.  On gfx950 the IEEE lowering of sqrtf is: scale inputs below
// 2^-96 by 2^32, v_sqrt_f32, fix the result by +-1 ulp from the signs of two fma residuals, unscale,
// and pass +-0 / +inf through.  For x >= 2^-96 (and +inf) the scaling and the special-value select are
// identities, so the device path runs the remaining instructions -- the same ones, in the same order,
// hence the same bits -- and keeps the full sequence for the other inputs.
RFX_HD float sqrt_rn(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
  if (x >= 0x1p-96f)
  {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u), s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, x), r_up = __builtin_fmaf(-s_up, s, x);
    const float t = r_dn <= 0.0f ? s_dn : s;
    return r_up > 0.0f ? s_up : t;
  }
#endif
  return sqrtf(x);
}

// Correctly rounded f32 division.  gfx950's IEEE lowering of a / b is eleven instructions:
//   b' = v_div_scale(b), a' = v_div_scale(a) (VCC: a rescale is pending), r = v_rcp(b'), e = fma(-b', r, 1),
//   r' = fma(e, r, r), q0 = a' r', t1 = fma(-b', q0, a'), q1 = fma(t1, r', q0), t2 = fma(-b', q1, a'),
//   q2 = v_div_fmas(t2, r', q1) (an fma, scaled by 2^+-64 when VCC), v_div_fixup(q2, b, a) (special values, sign).
// v_div_scale rescales an operand (or raises VCC) only for: a zero operand, b denormal, 1/b denormal, a/b denormal,
// exponent(a) - exponent(b) >= 96, or exponent(a) <= 23; v_div_fixup departs from sign(a) sign(b) |q2| only for NaN /
// infinite / zero operands and quotients beyond 2^+-150.  For b in [2^-40, 2^100] and a quotient in [2^-60, 2^60] none
// of them holds (|a| = |a/b| |b| lies in [2^-100, 2^160]: exponent(a) > 23, and the quotient's bounds exclude the rest
// with margins of 2^3 and more over the fast quotient's few-ulp error), so the scales and the fixup are identities and
// v_div_fmas is an fma: the eight remaining instructions, run in the same order, give the same bits.  The divisor's
// part (r, e, r') is shared by every quotient over one divisor (div_prep); a quotient outside the range is recomputed
// with '/'.  tests/test_div_guard.py replays the range argument in float32; rfx_kat_div checks the device path against
// IEEE '/' on 2^27+ operand pairs, both edges of every bound included.
#ifndef RFX_DIV_FAST
#define RFX_DIV_FAST 1  // 0: every quotient as the compiler lowers '/'; 2: no guard (timing builds only)
#endif
// the divisor and its refined reciprocal -- NaN when the divisor is outside [2^-40, 2^100], so that every fast quotient
// by it is NaN and fails the quotient's range test (one register for the guard's divisor half, not two)
struct DivRcp { float b, r; };
RFX_HD DivRcp div_prep(float b)
{
  DivRcp d;
  d.b = b;
#if defined(__HIP_DEVICE_COMPILE__) && RFX_DIV_FAST
  const float r = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, r, 1.0f);
  const float r1 = __builtin_fmaf(e, r, r);
  d.r = (RFX_DIV_FAST == 2 || (fabsf(b) >= 0x1p-40f && fabsf(b) <= 0x1p100f)) ? r1 : __builtin_nanf("");
#else
  d.r = 0.0f;
#endif
  return d;
}
// the quotient a / d.b by the shared reciprocal; ok: it is in the guarded range (else it must be recomputed)
RFX_HD float div_fast(float a, const DivRcp &d, bool &ok)
{
#if defined(__HIP_DEVICE_COMPILE__) && RFX_DIV_FAST
  const float q0 = a * d.r;
  const float t1 = __builtin_fmaf(-d.b, q0, a);
  const float q1 = __builtin_fmaf(t1, d.r, q0);
  const float t2 = __builtin_fmaf(-d.b, q1, a);
  const float q = __builtin_fmaf(t2, d.r, q1);
  ok = RFX_DIV_FAST == 2 || (fabsf(q) >= 0x1p-60f && fabsf(q) <= 0x1p60f);  // false for NaN (an out-of-range divisor)
  return q;
#else
  ok = false;
  return a / d.b;
#endif
}
RFX_HD float div_by(float a, const DivRcp &d)
{
  bool ok;
  const float q = div_fast(a, d, ok);
  if (__builtin_expect(!ok, 0)) return a / d.b;
  return q;
}
RFX_HD float div_rn(float a, float b) { return div_by(a, div_prep(b)); }
// a lone quotient (no divisor to share): the fast path saves three instructions and pays two compares and a branch for
// it, so it is a build option (RFX_DIV_SINGLE, tools/ab.py)
#ifndef RFX_DIV_SINGLE
#define RFX_DIV_SINGLE 0
#endif
RFX_HD float qdiv(float a, float b)
{
#if RFX_DIV_SINGLE
  return div_rn(a, b);
#else
  return a / b;
#endif
}

struct v3 { float x, y, z; };
struct col { float r, g, b; };
// Matrix33 element order _11.._33 (Matrix33.h:13-22)
struct m33 { float m11, m12, m13, m21, m22, m23, m31, m32, m33; };

RFX_HD v3 mk(float x, float y, float z) { v3 v; v.x = x; v.y = y; v.z = z; return v; }
RFX_HD v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }          // Vector3.cpp:106
RFX_HD v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }          // Vector3.cpp:111
RFX_HD v3 mul(v3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }              // Vector3.cpp:116,121
RFX_HD v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }                                 // Vector3.cpp:166
RFX_HD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }          // Vector3.cpp:126
RFX_HD float sqlen(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }              // Vector3.cpp:48
RFX_HD float len(v3 a) { return sqrt_rn(a.x * a.x + a.y * a.y + a.z * a.z); }       // Vector3.cpp:43
RFX_HD v3 cross(v3 a, v3 b)                                                          // Vector3.cpp:138
{
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RFX_HD v3 divv(v3 a, float f)                                                        // Vector3.cpp:143-151
{
  if (fabsf(f) > kVerySmall) return mk(a.x / f, a.y / f, a.z / f);
  return a;
}
// q = a / b by the fast path where the caller has already bounded the operands: |b| in (2^-63, 2^64] and |a| <= |b| (1
// + 2^-20) -- a vector component over the vector's length (a finite sum of squares is at most 2^128, so its root is at
// most 2^64), a direction component over its largest one.  Then |q| <= 1 + 2^-20, 1/b is normal, and |q| >= 2^-38 gives
// |a| >= 2^-102 (exponent(a) > 23) and a/b normal: the range test is one compare.  The reciprocal r is div_prep's.
RFX_HD float div_fast_unit(float a, float b, float r, bool &ok)
{
#if defined(__HIP_DEVICE_COMPILE__) && RFX_DIV_FAST
  const float q0 = a * r;
  const float t1 = __builtin_fmaf(-b, q0, a);
  const float q1 = __builtin_fmaf(t1, r, q0);
  const float t2 = __builtin_fmaf(-b, q1, a);
  const float q = __builtin_fmaf(t2, r, q1);
  ok = RFX_DIV_FAST == 2 || fabsf(q) >= 0x1p-38f;  // false for NaN
  return q;
#else
  ok = false;
  return a / b;
#endif
}
RFX_HD float rcp_refined(float b)  // div_prep's reciprocal, without its range test (div_fast_unit's callers bound b)
{
#if defined(__HIP_DEVICE_COMPILE__) && RFX_DIV_FAST
  const float r = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
#else
  return 1.0f / b;
#endif
}
// Vector3::normalized (Vector3.cpp:63-72) == Tracemath::normalize (trace_math.cpp:3-12)
RFX_HD v3 normalized(v3 a)
{
  const float l = len(a);
  if (l > kVerySmall)
  {
#if defined(__HIP_DEVICE_COMPILE__) && RFX_DIV_FAST
    // divv(a, l) with one reciprocal for the three quotients, one range compare each (div_fast_unit: |a_i| <= l <= 2^64)
    const float r = rcp_refined(l);
    bool ox, oy, oz;
    const v3 q = mk(div_fast_unit(a.x, l, r, ox), div_fast_unit(a.y, l, r, oy), div_fast_unit(a.z, l, r, oz));
    if (__builtin_expect(ox && oy && oz, 1)) return q;
#endif
    return divv(a, l);
  }
  return a;
}
// Tracemath::reflect (trace_math.cpp:14-23): v - (2n) * ((v.n) / (n.n))
RFX_HD v3 reflect(v3 v, v3 n)
{
  const float dn = dot(n, n);
  if (dn > kVerySmall) return sub(v, mul(mul(n, 2.0f), qdiv(dot(v, n), dn)));
  return v;
}
RFX_HD float clampf(float v, float lo, float hi) { return v < lo ? lo : v > hi ? hi : v; } // trace_math.h:24

// Distances compared through their squares.  sqrt_rn is monotone, so for dist = sqrt_rn(sq):
//   dist >= y  <=>  sq >= sq_lower_bound(y)     (y > 0 finite)
// where sq_lower_bound(y) is the smallest float whose rounded square root is >= y.  sqrt_rn(x) >= y iff
// sqrt(x) lies above the midpoint m between y and its predecessor; sqrt(x) is never exactly such a
// midpoint (an odd 25-bit significand squared has no 24-bit form), so the bound is the first float above
// m^2, which double arithmetic gets exactly (m has 25 significant bits, m^2 at most 50).
RFX_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
RFX_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
RFX_HD float sq_lower_bound(float y)
{
  const double m = ((double)u2f(f2u(y) - 1u) + (double)y) * 0.5;
  const double m2 = m * m;
  float f = (float)m2;
  if ((double)f <= m2) f = u2f(f2u(f) + 1u);
  return f;
}
// Sphere.cpp:62-64 `(ray * t).length() > DELTA` as a test on the squared length:
// sqrt_rn(sq) > 1e-4f  <=>  sq >= sq_lower_bound(succ(1e-4f)) (tests/test_sqrt_bounds.py)
constexpr float kSqDeltaSphere = 0x1.5798fp-27f;

// Matrix33(u, v, n): columns (Matrix33.cpp:10-15)
RFX_HD m33 from_cols(v3 u, v3 v, v3 n)
{
  m33 m;
  m.m11 = u.x; m.m12 = v.x; m.m13 = n.x;
  m.m21 = u.y; m.m22 = v.y; m.m23 = n.y;
  m.m31 = u.z; m.m32 = v.z; m.m33 = n.z;
  return m;
}
// Matrix33 * Vector3 (Matrix33.cpp:230-235)
RFX_HD v3 mmul(const m33 &m, v3 v)
{
  return mk(v.x * m.m11 + v.y * m.m12 + v.z * m.m13,
            v.x * m.m21 + v.y * m.m22 + v.z * m.m23,
            v.x * m.m31 + v.y * m.m32 + v.z * m.m33);
}
// Matrix33::invert (Matrix33.cpp:50-79)
RFX_HD m33 inverted(const m33 &a)
{
  const float d = a.m11 * (a.m22 * a.m33 - a.m32 * a.m23) +
                  a.m21 * (a.m32 * a.m13 - a.m12 * a.m33) +
                  a.m31 * (a.m12 * a.m23 - a.m13 * a.m22);
  m33 r;
  if (fabsf(d) > kVerySmall)
  {
    r.m11 = (a.m22 * a.m33 - a.m23 * a.m32) / d;
    r.m12 = (a.m13 * a.m32 - a.m12 * a.m33) / d;
    r.m13 = (a.m12 * a.m23 - a.m13 * a.m22) / d;
    r.m21 = (a.m23 * a.m31 - a.m21 * a.m33) / d;
    r.m22 = (a.m11 * a.m33 - a.m13 * a.m31) / d;
    r.m23 = (a.m13 * a.m21 - a.m11 * a.m23) / d;
    r.m31 = (a.m21 * a.m32 - a.m22 * a.m31) / d;
    r.m32 = (a.m12 * a.m31 - a.m11 * a.m32) / d;
    r.m33 = (a.m11 * a.m22 - a.m12 * a.m21) / d;
  }
  else
  {
    r.m11 = 1; r.m12 = 0; r.m13 = 0; r.m21 = 0; r.m22 = 1; r.m23 = 0; r.m31 = 0; r.m32 = 0; r.m33 = 1;
  }
  return r;
}

// Color (Color.cpp)
RFX_HD col mkc(float r, float g, float b) { col c; c.r = r; c.g = g; c.b = b; return c; }
RFX_HD col cadd(col a, col b) { return mkc(a.r + b.r, a.g + b.g, a.b + b.b); }      // :78
RFX_HD col cmul(col a, col b) { return mkc(a.r * b.r, a.g * b.g, a.b * b.b); }      // :108
RFX_HD col cscale(col a, float f) { return mkc(a.r * f, a.g * f, a.b * f); }        // :88,93
RFX_HD col cclamp(col a)                                                              // :119-124
{
  return mkc(clampf(a.r, 0.0f, 1.0f), clampf(a.g, 0.0f, 1.0f), clampf(a.b, 0.0f, 1.0f));
}
RFX_HD col from_argb(uint32_t c)                                                      // :9-14
{
  return mkc((float)((c >> 16) & 0xFFu) / 255.0f, (float)((c >> 8) & 0xFFu) / 255.0f, (float)(c & 0xFFu) / 255.0f);
}
// Color::argb (Color.cpp:114-117, Color.h:11-15): trunc(c * 255.999f), low byte, alpha 0.
// Out-of-range sums (additive copyImage) take the low byte of the int32 conversion, as x86-64 g++ does.
RFX_HD uint32_t q8(float f)
{
  const float lim = 2147483648.0f;
  const int32_t i = (f < lim && f > -lim) ? (int32_t)f : (int32_t)0x80000000;
  return (uint32_t)(uint8_t)i;
}
RFX_HD uint32_t argb(col c)
{
  return q8(c.r * 255.999f) << 16 | q8(c.g * 255.999f) << 8 | q8(c.b * 255.999f);
}

// LCG (trace_math.h:34-39): s = 214013 s + 2531011 (mod 2^32), out (s >> 16) & 0x7FFF
RFX_HD uint32_t lcg_step(uint32_t s) { return 214013u * s + 2531011u; }
RFX_HD uint32_t lcg_out(uint32_t s) { return (s >> 16) & 0x7FFFu; }
// s advanced by n steps: affine map (A, C) composed by binary powering
RFX_HD uint32_t lcg_jump(uint32_t s, uint64_t n)
{
  uint32_t a = 214013u, c = 2531011u, A = 1u, C = 0u;
  while (n)
  {
    if (n & 1u) { A = a * A; C = a * C + c; }
    c = a * c + c;
    a = a * a;
    n >>= 1;
  }
  return A * s + C;
}
// one component of Vector3::randomInsideSphere (Vector3.cpp:182-184)
RFX_HD float rand_component(uint32_t k) { return (float)k / ((float)0x7FFF / 2) - 1.f; }
// The same value without the f32 divide (the RNG pre-pass kernels), and the subtraction of 1 is the
// reference's own.  For every k in [0, 0x7FFF] the quotient (float)k / 16383.5f equals
//   host:   (float)((double)k * (1.0 / 16383.5))
//   device: q = k * r, e = fma(-q, 16383.5, k), q + e * r as one fma (r = f32(1 / 16383.5)),
// f32 only (f64 multiplies and conversions run at a fraction of the f32 rate) -- both checked
// exhaustively by tests/test_rng_exact.py.
RFX_HD float rand_component_dev(uint32_t k)
{
#if defined(__HIP_DEVICE_COMPILE__)
  const float kf = (float)k, r = 1.0f / 16383.5f;
  const float q = kf * r;
  const float e = __builtin_fmaf(-q, 16383.5f, kf);
  return __builtin_fmaf(e, r, q) - 1.f;
#else
  return (float)((double)k * (1.0 / 16383.5)) - 1.f;
#endif
}

}  // namespace rfx
