// clrrt_dubins_lb.hpp — a cheap lower bound on dubinsDistance (rrtplanner.cpp:371-406) for the
// nearest-node prefilter.  Host/device: tests/native/dubins_lb_check.cpp validates it against a float
// restatement of the key on many random points.
//
// In the node frame (qx, qy), qy folded to >= 0, rho = 4.77, a point outside both turning circles has
//   key = sqrt(dc^2 - rho^2) + rho * (thc - acos(rho / dc)),  dc = |(qx, qy - rho)|,
//   thc = atan2(qx, rho - qy) in [0, 2pi).
// The bound evaluates thc and acos with a polynomial atan (|error| <= 1e-5 rad, Abramowitz & Stegun
// 4.4.49) and subtracts margins that cover the float rounding of both this bound and the key itself
// (acos(rho/dc) is ill-conditioned near the circle: <= ~5e-4 rad either way): 2e-3 rad on the arc
// angle and 1e-2 m absolute.  Points inside a circle get rho * pi - 0.08 (the key's minimum there is
// rho * pi = 14.985).
#pragma once
#include <math.h>

#ifndef CLRRT_HD
#if defined(__HIPCC__)
#define CLRRT_HD __host__ __device__
#else
#define CLRRT_HD
#endif
#endif

namespace clrrt {

CLRRT_HD inline float atan01(float x) {  // atan on [0, 1], |error| <= 1e-5
  const float x2 = x * x;
  return x * (0.9998660f + x2 * (-0.3302995f + x2 * (0.1801410f + x2 * (-0.0851330f + x2 * 0.0208351f))));
}

// atan2(y, x) wrapped like dubins_key: values < 0 get + 2 pi (|error| <= ~2e-5).
CLRRT_HD inline float atan2_wrap(float y, float x) {
  const float ay = fabsf(y), ax = fabsf(x);
  float a;
  if (ay <= ax) a = ax > 0.f ? atan01(ay / ax) : 0.f;
  else a = 1.57079633f - atan01(ax / ay);
  if (x < 0.f) a = 3.14159265f - a;
  if (signbit(y)) a = -a;
  if (a < 0.f) a += 6.28318531f;
  return a;
}

// Lower bound on the float Dubins key of a sample at (qx, qy) in the node frame (qy >= 0).
CLRRT_HD inline float dubins_lb(float qx, float qy) {
  const float rho = 4.77f;
  const bool inside = (qx * qx + (qy + rho) * (qy + rho) <= rho * rho) | (qx * qx + (qy - rho) * (qy - rho) <= rho * rho);
  if (inside) return 14.9f;
  const float dc2 = qx * qx + (qy - rho) * (qy - rho);
  const float dc = sqrtf(dc2);
  const float T = sqrtf(fmaxf(dc2 - rho * rho, 0.f));
  const float thc = atan2_wrap(qx, rho - qy);
  const float r = fminf(rho / dc, 1.f);
  const float ac = atan2_wrap(sqrtf(fmaxf(1.f - r * r, 0.f)), r);  // acos(r) in [0, pi/2]
  return T * (1.f - 1e-5f) + rho * (thc - ac - 2e-3f) - 1e-2f;
}

}  // namespace clrrt
