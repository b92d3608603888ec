// glibc powf, restated for the device.
//
// The reference calls pow(float, float) -> glibc 2.35 `powf@@GLIBC_2.27` at
// Scene.cpp:175 (specular) and Scene.cpp:196 (Fresnel).  That function is a
// third-party dependency absent from /root/reference: glibc 2.35
// (Ubuntu 2.35-0ubuntu3.x), sysdeps/ieee754/flt-32/e_powf.c -- the ARM
// optimized-routines algorithm: log2(x) from a 16-entry (invc, log2 c) table and
// a degree-5 polynomial in double, y*log2(x) in double, exp2 from a 32-entry
// 2^(k/32) table and a degree-3 polynomial, one final double->float rounding.
// On x86-64 hosts with FMA+AVX2 (the survey container and the GPU box's EPYC)
// the ifunc selects the `-mfma` build, whose polynomial steps are fused
// multiply-adds.  Every constant below and every fma/mul/add choice was read
// from the installed libm.so.6 (disassembly of the ifunc target and its
// .rodata); tests/test_powf.py checks this restatement bit-for-bit against the
// live libm powf on >10^7 inputs of both call sites' domains.
//
// Domain note: the renderer only calls it with x in [0, 1], y >= 1 finite.  The
// special-case branches of glibc are restated for x >= 0 (zero, subnormal,
// inf/nan) and negative x with integer y, so KATs outside the domain also hold.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RFX_PHD __host__ __device__ __forceinline__
#define RFX_PCONST __device__ __constant__
#else
#include <math.h>
#define RFX_PHD static inline
#define RFX_PCONST static const
#endif

#pragma clang fp contract(off)

namespace rfx {

// __powf_log2_data.tab: {invc, logc} (POWF_LOG2_TABLE_BITS = 4)
RFX_PCONST double kPowfLog2Tab[16][2] = {
  {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
  {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
  {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
  {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
  {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
  {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
  {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
  {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
// __exp2f_data.tab: bits of 2^(i/32) minus (i << 47)  (EXP2F_TABLE_BITS = 5)
RFX_PCONST uint64_t kExp2fTab[32] = {
  0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
  0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
  0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
  0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
  0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
  0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
  0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
  0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};

RFX_PHD uint32_t pw_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
RFX_PHD float pw_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
RFX_PHD uint64_t pw_asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
RFX_PHD double pw_asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }
#if defined(__HIPCC__)
RFX_PHD double pw_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
#else
RFX_PHD double pw_fma(double a, double b, double c) { return fma(a, b, c); }
#endif

// 0: not an integer, 1: odd integer, 2: even integer (e_powf.c checkint)
RFX_PHD int pw_checkint(uint32_t iy)
{
  int e = iy >> 23 & 0xff;
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}
RFX_PHD int pw_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }

// The three polynomial addends that are not inline constants.  An f64 fma on gfx950 reads at most one
// scalar operand, so with the multiplier in SGPRs each addend needs a VGPR pair; as literals they are
// hoisted out of the trace loop and spilled to scratch.  Read from a table (the trace kernel's LDS copy)
// at an index the compiler cannot fold -- (ix >> 31), always 0 there -- they are loaded at the call.
RFX_PCONST double kPowfAdd[2][4] = {{-0x1.71969a075c67ap-2, -0x1.7154748bef6c8p-1, 0x1.ebfce50fac4f3p-3, 0.0},
                                    {-0x1.71969a075c67ap-2, -0x1.7154748bef6c8p-1, 0x1.ebfce50fac4f3p-3, 0.0}};

// logtab / exptab / addtab: kPowfLog2Tab / kExp2fTab / kPowfAdd or copies of them (the trace kernel keeps
// copies in LDS)
RFX_PHD float powf_glibc_t(float x, float y, const double (*logtab)[2], const uint64_t *exptab,
                           const double (*addtab)[4])
{
  uint32_t sign_bias = 0;
  uint32_t ix = pw_asuint(x), iy = pw_asuint(y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || pw_zeroinfnan(iy))
  {
    if (pw_zeroinfnan(iy))
    {
      if (2 * iy == 0) return 1.0f;
      if (ix == 0x3f800000u) return 1.0f;
      if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
      if (2 * ix == 2 * 0x3f800000u) return 1.0f;
      if ((2 * ix < 2 * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
      return y * y;
    }
    if (pw_zeroinfnan(ix))
    {
      float x2 = x * x;
      if ((ix & 0x80000000u) && pw_checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000u) ? 1 / x2 : x2;
    }
    if (ix & 0x80000000u)
    {
      const int yint = pw_checkint(iy);
      if (yint == 0) return (x - x) / (x - x);  // invalid -> NaN
      if (yint == 1) sign_bias = 1u << 16;
      ix &= 0x7fffffffu;
    }
    if (ix < 0x00800000u)
    {
      ix = pw_asuint(pw_asfloat(ix) * 0x1p23f);
      ix &= 0x7fffffffu;
      ix -= 23u << 23;
    }
  }
  // log2_inline (e_powf.c), fused as the FMA ifunc variant emits it
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16);
  const uint32_t top = tmp & 0xff800000u;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double invc = logtab[i][0], logc = logtab[i][1];
  const double *add = addtab[ix >> 31];  // ix < 2^31 here: row 0
  const double z = (double)pw_asfloat(iz);
  const double r = pw_fma(z, invc, -1.0);
  const double y0 = logc + (double)k;
  const double r2 = r * r;
  double yy = pw_fma(r, 0x1.27616c9496e0bp-2, add[0]);      // -0x1.71969a075c67ap-2
  const double p = pw_fma(r, 0x1.ec70a6ca7baddp-2, add[1]);  // -0x1.7154748bef6c8p-1
  const double r4 = r2 * r2;
  double q = pw_fma(r, 0x1.71547652ab82bp+0, y0);
  q = pw_fma(r2, p, q);
  const double logx = pw_fma(yy, r4, q);
  const double ylogx = (double)y * logx;
  if ((pw_asuint64(ylogx) >> 47 & 0xffff) >= pw_asuint64(126.0) >> 47)
  {
    if (ylogx > 0x1.fffffffd1d571p+6)  // __math_oflowf
      return sign_bias ? -0x1p97f * 0x1p97f : 0x1p97f * 0x1p97f;
    if (ylogx <= -150.0)               // __math_uflowf
      return sign_bias ? -0x1p-95f * 0x1p-95f : 0x1p-95f * 0x1p-95f;
    if (ylogx < -149.0)                // __math_may_uflowf
      return sign_bias ? -0x1.4p-75f * 0x1.4p-75f : 0x1.4p-75f * 0x1.4p-75f;
  }
  // exp2_inline
  const double shift = 0x1.8p+47;
  double kd = ylogx + shift;
  const uint64_t ki = pw_asuint64(kd);
  kd -= shift;
  const double rr = ylogx - kd;
  uint64_t t = exptab[ki % 32];
  t += (ki + sign_bias) << 47;
  const double s = pw_asdouble(t);
  const double zz = pw_fma(rr, 0x1.c6af84b912394p-5, add[2]);  // 0x1.ebfce50fac4f3p-3
  const double rr2 = rr * rr;
  double e = pw_fma(rr, 0x1.62e42ff0c52d6p-1, 1.0);
  e = pw_fma(zz, rr2, e);
  e = e * s;
  return (float)e;
}

RFX_PHD float powf_glibc(float x, float y) { return powf_glibc_t(x, y, kPowfLog2Tab, kExp2fTab, kPowfAdd); }

// powf(x, 3) for x in [0, 1] (Scene.cpp:196, the Fresnel term) without glibc's log2/exp2 in the common case.  x^3 in
// double (x^2 is exact, one rounding) lies within 2^-52 of the true cube; when every value within 2^-32 (relative) of it
// rounds to the same float, so do the true cube and glibc's pre-rounding result, and that float is glibc powf's
// result.  Returns false (the caller runs powf_glibc_t) for x below 2^-12 and for cubes that close to a rounding
// midpoint (~0.6% of the floats in [2^-12, 1]).  2^-32 covers glibc's pre-rounding error at y = 3 on this domain
// with nothing to spare: checked on every float in [0, 1] against the live libm (tests/test_powf.py; 2^-34 leaves
// 16,306 mismatches), and the device copy against powf_glibc_t(x, 3) on the same floats (rfx_kat_powf_cube).
RFX_PHD bool powf_cube_fast(float x, float &out)
{
  const double xd = (double)x;
  const double c = xd * xd * xd;
  const float lo = (float)(c * (1.0 - 0x1p-32)), hi = (float)(c * (1.0 + 0x1p-32));
  out = lo;
  return x >= 0x1p-12f && lo == hi;
}

}  // namespace rfx
