// clrrt_glibcf.hpp — glibc 2.35's float atanf, atan2f, acosf and asinf restated for gfx950 (and the host
// tests).
//
// The reference's nearest-node key (dubinsDistance, rrt/src/rrtplanner.cpp:371-406) is computed in
// float with atan2(float, float), acos(float) and asin(float) — std:: overloads resolving to glibc's
// atan2f / acosf / asinf (sysdeps/ieee754/flt-32: e_atan2f.c, s_atanf.c, e_acosf.c, e_asinf.c, derived
// from fdlibm; x86-64 has no FMA variants of them, so no multiply-add is fused).  The GPU math library
// rounds ~35% of their results differently, which reorders near-tied keys; these restatements make the
// device keys the reference's keys bit for bit.  Checked against the host libm on every float argument
// (atanf, acosf, asinf) and on 10^8 random and edge-case pairs (atan2f): tests/native/glibcf_check.cpp.
// Provenance: glibc 2.35's float atan/atan2/acos/asin derive from Sun Microsystems' fdlibm ("Copyright (C)
// 1993 by Sun Microsystems, Inc. ... Permission to use, copy, modify, and distribute this software is
// freely granted, provided that this notice is preserved"); glibc distributes them under the GNU Lesser
// General Public License v2.1 or later.
#pragma once
#include <stdint.h>
#include <string.h>

#ifndef CLRRT_HD
#if defined(__HIPCC__)
#define CLRRT_HD __host__ __device__
#else
#define CLRRT_HD
#endif
#endif

namespace clrrt {
namespace glibcf {

CLRRT_HD inline int32_t fword(float x) {
  int32_t u;
  memcpy(&u, &x, 4);
  return u;
}
CLRRT_HD inline float fromword(int32_t u) {
  float x;
  memcpy(&x, &u, 4);
  return x;
}
CLRRT_HD inline float fabs_(float x) { return fromword(fword(x) & 0x7fffffff); }
CLRRT_HD inline float sqrt_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_sqrtf(x);  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
#else
  return __builtin_sqrtf(x);
#endif
}

// s_atanf.c
CLRRT_HD inline float atanf(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
              atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
              atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  const float one = 1.0f;
  float w, s1, s2, z;
  int32_t ix, hx, id;
  hx = fword(x);
  ix = hx & 0x7fffffff;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;  // NaN
    if (hx > 0) return atanhi3 + atanlo3;
    return -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = fabs_(x);
    if (ix < 0x3f980000) {    // |x| < 1.1875
      if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0f * x - one) / (2.0f + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - one) / (x + one);
      }
    } else {
      if (ix < 0x401c0000) {  // |x| < 2.4375
        id = 2;
        x = (x - 1.5f) / (one + 1.5f * x);
      } else {  // 2.4375 <= |x| < 2^25
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  z = x * x;
  w = z * z;
  s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  const float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return (hx < 0) ? -z : z;
}

// e_atan2f.c
CLRRT_HD inline float atan2f(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
              pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  float z;
  int32_t k, m, hx, hy, ix, iy;
  hx = fword(x);
  ix = hx & 0x7fffffff;
  hy = fword(y);
  iy = hy & 0x7fffffff;
  if ((ix > 0x7f800000) || (iy > 0x7f800000)) return x + y;  // NaN
  if (hx == 0x3f800000) return atanf(y);                     // x = 1.0
  m = ((hy >> 31) & 1) | ((hx >> 30) & 2);                   // 2*sign(x) + sign(y)
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  k = (iy - ix) >> 23;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;  // |y/x| > 2^60
  else if (hx < 0 && k < -60) z = 0.0f;   // |y|/x < -2^60
  else z = atanf(fabs_(y / x));
  switch (m) {
    case 0: return z;
    case 1: return fromword(fword(z) ^ (int32_t)0x80000000);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// e_acosf.c
CLRRT_HD inline float acosf(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
              pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
              pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f,
              qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f,
              qS4 = 7.7038154006e-02f;
  float z, p, q, r, w, s, c, df;
  int32_t hx, ix;
  hx = fword(x);
  ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {  // |x| == 1
    if (hx > 0) return 0.0f;
    return pi + 2.0f * pio2_lo;
  } else if (ix > 0x3f800000) {
    return (x - x) / (x - x);  // NaN
  }
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;  // |x| <= 2^-26
    z = x * x;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {  // x < -0.5
    z = (one + x) * 0.5f;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    s = sqrt_(z);
    r = p / q;
    w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  } else {  // x > 0.5
    z = (one - x) * 0.5f;
    s = sqrt_(z);
    df = fromword(fword(s) & (int32_t)0xfffff000);
    c = (z - df * df) / (s + df);
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    w = r * s + c;
    return 2.0f * (df + w);
  }
}

// e_asinf.c
CLRRT_HD inline float asinf(float x) {
  const float one = 1.0f, pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
              pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-1f, p1 = 7.495297643e-2f,
              p2 = 4.547037598e-2f, p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  float t, w, p, q, c, r, s;
  int32_t hx, ix;
  hx = fword(x);
  ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;  // asin(+-1) = +-pi/2
  if (ix > 0x3f800000) return (x - x) / (x - x);           // NaN
  if (ix < 0x3f000000) {                                   // |x| < 0.5
    if (ix < 0x32000000) return x;                         // |x| < 2^-27
    t = x * x;
    w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    return x + x * w;
  }
  // 1 > |x| >= 0.5
  w = one - fabs_(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = sqrt_(t);
  if (ix >= 0x3F79999A) {  // |x| > 0.975
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = fromword(fword(s) & (int32_t)0xfffff000);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

}  // namespace glibcf
}  // namespace clrrt
