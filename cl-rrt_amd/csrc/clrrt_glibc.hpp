// clrrt_glibc.hpp — glibc 2.35's double sin, cos and tan restated for gfx950 (and the host tests).
//
// The reference computes its closed-loop rollouts with glibc's libm (rrt/src/simulation.cpp:13-16,
// controller.cpp:56-57,115-132).  Its goal-biased rollouts are ill-conditioned: getGoalReference
// duplicates the joint point of its two segments (reference.cpp:56-63), so the 3-point Lagrange
// interpolation of getLateralError divides by ~0 there (controller.cpp:134-148) and the sign of the
// saturated steering command depends on the last bit of every earlier sin/cos/tan.  Matching the
// reference's trees therefore needs these three functions bit for bit.  On x86-64 CPUs with
// FMA+AVX2 (the oracle's and the GPU box's hosts), libm's ifunc runs the FMA-compiled variants of
// sysdeps/ieee754/dbl-64/s_sin.c and s_tan.c (IBM Accurate Mathematical Library); this file follows
// their algorithm — table-driven do_sin/do_cos with the Cody-Waite reduce_sincos, and tan's xfg
// table path — and fuses exactly the multiply-adds that build fuses, so every rounding is identical.
//
// Domain restated: |x| < 105414350 for sin/cos (beyond that glibc switches to __branred: we fall
// back to the GPU libm, outside anything the planner evaluates); |x| <= 0.787 for tan (steering
// angles are clamped to +-0.52 rad; larger arguments fall back likewise).  NaN/Inf propagate.
// Provenance: the algorithms, constants and tables restated here are glibc's (GNU C Library 2.35, libm;
// the IBM Accurate Mathematical Library sources, (C) IBM Corp. and the Free Software Foundation), which
// glibc distributes under the GNU Lesser General Public License v2.1 or later.
#pragma once
#include <stdint.h>
#include <string.h>

#include <cmath>

#include "clrrt_glibc_data.hpp"

#ifndef CLRRT_HD
#if defined(__HIPCC__)
#define CLRRT_HD __host__ __device__
#else
#define CLRRT_HD
#endif
#endif

namespace clrrt {
namespace glibc {

#if defined(__HIPCC__)
static __device__ __constant__ double d_sincostab[SINCOSTAB_N] = CLRRT_GLIBC_SINCOSTAB;
static __device__ __constant__ double d_xfg[XFG_ROWS * 4] = CLRRT_GLIBC_XFG;
// Per-block LDS copies: the table index depends on the argument, so lanes gather from scattered
// addresses; from LDS that costs ~100 cycles instead of a cache-missing global load.  Every kernel
// that evaluates these functions calls stage_tables() first.
static __shared__ double s_sincostab[SINCOSTAB_N];
static __shared__ double s_xfg[XFG_ROWS * 4];
__device__ inline void stage_tables() {
  for (int i = threadIdx.x; i < SINCOSTAB_N; i += blockDim.x) s_sincostab[i] = d_sincostab[i];
  for (int i = threadIdx.x; i < XFG_ROWS * 4; i += blockDim.x) s_xfg[i] = d_xfg[i];
  __syncthreads();
}
#endif
static const double h_sincostab[SINCOSTAB_N] = CLRRT_GLIBC_SINCOSTAB;
static const double h_xfg[XFG_ROWS * 4] = CLRRT_GLIBC_XFG;

CLRRT_HD inline const double* sincostab() {
#if defined(__HIP_DEVICE_COMPILE__)
  return s_sincostab;
#else
  return h_sincostab;
#endif
}
CLRRT_HD inline const double* xfg() {
#if defined(__HIP_DEVICE_COMPILE__)
  return s_xfg;
#else
  return h_xfg;
#endif
}

CLRRT_HD inline uint64_t bits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
CLRRT_HD inline uint32_t hi_word(double x) { return (uint32_t)(bits(x) >> 32); }
CLRRT_HD inline int32_t lo_word(double x) { return (int32_t)(uint32_t)bits(x); }
CLRRT_HD inline double fma_(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return std::fma(a, b, c);
#endif
}
CLRRT_HD inline double copysign_(double m, double s) {
  uint64_t u = (bits(m) & 0x7fffffffffffffffull) | (bits(s) & 0x8000000000000000ull);
  double r;
  memcpy(&r, &u, 8);
  return r;
}

// TAYLOR_SIN (s_sin.c): a + ((poly(xx)*a - 0.5*da)*xx + da)
CLRRT_HD inline double taylor_sin(double a, double da) {
  double xx = a * a;
  double t = fma_(xx, s5, s4);
  t = fma_(xx, t, s3);
  t = fma_(xx, t, s2);
  t = fma_(xx, t, s1);
  double u = fma_(t, a, -(0.5 * da));
  double w = fma_(xx, u, da);
  return w + a;
}

// do_sin (s_sin.c) for |x| >= taylor_lim: sin(x + dx) from the sin/cos table at k/128.
CLRRT_HD inline double do_sin_tab(double x, double dx) {
  if (x <= 0) dx = -dx;
  double ax = fabs(x);
  double u = ax + big;
  int k = lo_word(u) << 2;
  double xr = ax - (u - big);
  double xx = xr * xr;
  double s = xr + fma_(xr * xx, fma_(xx, sn5, sn3), dx);
  double c = fma_(xr, dx, xx * fma_(xx, fma_(xx, cs6, cs4), cs2));
  const double* T = sincostab();
  double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
  double cor = fma_(s, ccs, ssn);
  cor = fma_(-c, sn, cor);
  cor = fma_(s, cs, cor);
  return copysign_(sn + cor, x);
}

CLRRT_HD inline double do_sin(double x, double dx) {
  if (fabs(x) < taylor_lim) return taylor_sin(x, dx);
  return do_sin_tab(x, dx);
}

// do_cos (s_sin.c): cos(x + dx) from the sin/cos table at k/128.
CLRRT_HD inline double do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  double ax = fabs(x);
  double u = ax + big;
  int k = lo_word(u) << 2;
  double xr = (ax - (u - big)) + dx;
  double xx = xr * xr;
  double s = fma_(xr * xx, fma_(xx, sn5, sn3), xr);
  double c = xx * fma_(xx, fma_(xx, cs6, cs4), cs2);
  const double* T = sincostab();
  double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
  double cor = fma_(-s, ssn, ccs);
  cor = fma_(-c, cs, cor);
  cor = fma_(-s, sn, cor);
  return cs + cor;
}

// reduce_sincos (s_sin.c): x = n*pi/2 + (a + da), |a| <= pi/4.
CLRRT_HD inline int reduce_sincos(double x, double& a, double& da) {
  double t = fma_(x, hpinv, toint);
  double xn = t - toint;
  int n = lo_word(t) & 3;
  double y = fma_(-xn, mp1, x);
  y = fma_(-xn, mp2, y);
  double t2 = fma_(-xn, pp3, y);
  double db = fma_(-pp3, xn, y - t2);
  double b = fma_(-xn, pp4, t2);
  double db2 = fma_(-xn, pp4, t2 - b);
  a = b;
  da = db + db2;
  return n;
}

CLRRT_HD inline double do_sincos(double a, double da, int n) {
  double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}

CLRRT_HD inline double sin(double x) {
  uint32_t k = hi_word(x) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return do_sin(x, 0.0);
  if (k < 0x400368fdu) {
    double t = hp0 - fabs(x);
    return copysign_(do_cos(t, hp1), x);
  }
  if (k < 0x419921fbu) {
    double a, da;
    int n = reduce_sincos(x, a, da);
    return do_sincos(a, da, n);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  return ::sin(x);  // |x| >= 105414350 or non-finite: outside the restated domain
#else
  return std::sin(x);
#endif
}

CLRRT_HD inline double cos(double x) {
  uint32_t k = hi_word(x) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return do_cos(x, 0.0);
  if (k < 0x400368fdu) {
    double y = hp0 - fabs(x);
    double a = y + hp1;
    double da = (y - a) + hp1;
    return do_sin(a, da);
  }
  if (k < 0x419921fbu) {
    double a, da;
    int n = reduce_sincos(x, a, da);
    return do_sincos(a, da, n + 1);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  return ::cos(x);
#else
  return std::cos(x);
#endif
}

// s_tan.c cases (I) |x| <= g1, (II) |x| < g2 polynomial, (III) |x| <= g3 xfg table.
CLRRT_HD inline double tan(double x) {
  double w = (x < 0.0) ? -x : x;
  if (w <= tan_g1) return x;
  if (w <= tan_g2) {
    double x2 = x * x;
    double t = fma_(x2, d11, d9);
    t = fma_(x2, t, d7);
    t = fma_(x2, t, d5);
    t = fma_(x2, t, d3);
    return fma_(x * x2, t, x);
  }
  if (w <= tan_g3) {
    int i = (int)fma_(w, two8, mfftnhf);
    const double* row = xfg() + 4 * i;
    double z = w - row[0];
    double z2 = z * z;
    double pz = fma_(z * z2, fma_(z2, e1, e0), z);
    double fi = row[1], gi = row[2];
    double y = ((fi + gi) * pz) / (gi - pz) + fi;
    return (x >= 0.0 ? 1.0 : -1.0) * y;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  return ::tan(x);  // outside the restated domain (steering angles never get here)
#else
  return std::tan(x);
#endif
}

// ---------------------------------------------------------------------------------------------
// sincos: glibc's __sincos (s_sincos.c) is NOT ifunc-dispatched; libm ships only its generic SSE2
// build, so its do_sin/do_cos/TAYLOR_SIN/reduce_sincos round every product and sum separately.
// GCC merges a sin(x) and a cos(x) of the same argument in one function into a sincos(x) call, which
// is how the reference evaluates the vehicle heading (controller.cpp:56-57,115-132,
// simulation.cpp:14-15, old_collisioncheck.cpp:34) — so the rollouts need this variant.
namespace nofma {
CLRRT_HD inline double taylor_sin(double a, double da) {
  double xx = a * a;
  double p = ((((s5 * xx + s4) * xx + s3) * xx + s2) * xx) + s1;
  double t = ((p * a - 0.5 * da) * xx + da);
  return a + t;
}
CLRRT_HD inline double do_sin(double x, double dx) {
  double xold = x;
  if (fabs(x) < taylor_lim) return taylor_sin(x, dx);
  if (x <= 0) dx = -dx;
  double u = big + fabs(x);
  int k = lo_word(u) << 2;
  x = fabs(x) - (u - big);
  double xx = x * x;
  double s = x + (dx + x * xx * (sn3 + xx * sn5));
  double c = x * dx + xx * (cs2 + xx * (cs4 + xx * cs6));
  const double* T = sincostab();
  double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
  double cor = (ssn + s * ccs - sn * c) + cs * s;
  return copysign_(sn + cor, xold);
}
CLRRT_HD inline double do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  double u = big + fabs(x);
  int k = lo_word(u) << 2;
  x = fabs(x) - (u - big) + dx;
  double xx = x * x;
  double s = x + x * xx * (sn3 + xx * sn5);
  double c = xx * (cs2 + xx * (cs4 + xx * cs6));
  const double* T = sincostab();
  double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
  double cor = (ccs - s * ssn - cs * c) - sn * s;
  return cs + cor;
}
CLRRT_HD inline int reduce_sincos(double x, double& a, double& da) {
  double t = (x * hpinv + toint);
  double xn = t - toint;
  int n = lo_word(t) & 3;
  double y = (x - xn * mp1) - xn * mp2;
  double t1 = xn * pp3;
  double t2 = y - t1;
  double db = (y - t2) - t1;
  t1 = xn * pp4;
  double b = t2 - t1;
  db += (t2 - b) - t1;
  a = b;
  da = db;
  return n;
}
CLRRT_HD inline double do_sincos(double a, double da, int n) {
  double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}
}  // namespace nofma

CLRRT_HD inline void sincos(double x, double& sx, double& cx) {
  uint32_t k = hi_word(x) & 0x7fffffffu;
  if (k < 0x400368fdu) {
    if (k < 0x3e400000u) { sx = x; cx = 1.0; return; }
    if (k < 0x3feb6000u) { sx = nofma::do_sin(x, 0); cx = nofma::do_cos(x, 0); return; }
    double y = hp0 - fabs(x);
    double a = y + hp1;
    double da = (y - a) + hp1;
    sx = copysign_(nofma::do_cos(a, da), x);
    cx = nofma::do_sin(a, da);
    return;
  }
  if (k < 0x419921fbu) {
    double a, da;
    int n = nofma::reduce_sincos(x, a, da);
    sx = nofma::do_sincos(a, da, n);
    cx = nofma::do_sincos(a, da, n + 1);
    return;
  }
  sx = sin(x);  // outside the restated domain
  cx = cos(x);
}

// The same functions with the range cases selected per lane instead of branched on (the rollout step;
// a wave's lanes hold different headings).  Every case of glibc's sin, cos and sincos below the
// Payne-Hanek range is one do_sin and one do_cos evaluation on per-case arguments, so computing each
// once on the selected arguments (and the cheap Cody-Waite reduction for every lane) costs a divergent
// wave one evaluation per function instead of one per case present.  Values are those of the branched
// functions: the same do_sin / do_cos on the same arguments.  |x| >= 105414350 or non-finite lanes take
// the branched functions.
//   sincos_sel:     sincos (generic build, GCC's merged sin/cos of one argument)
//   sin_cos_fma_sel: sin(x) and cos(x) as two separate FMA-build calls
CLRRT_HD inline void sincos_sel(double x, double& sx, double& cx) {
  const uint32_t k = hi_word(x) & 0x7fffffffu;
  if (!(k < 0x419921fbu)) {
    sincos(x, sx, cx);
    return;
  }
  const bool cA = k < 0x3feb6000u, cB = !cA && k < 0x400368fdu;
  const double y = hp0 - fabs(x);
  const double aB = y + hp1, daB = (y - aB) + hp1;
  double aC, daC;
  const int n = nofma::reduce_sincos(x, aC, daC);
  const double a = cA ? x : (cB ? aB : aC), da = cA ? 0.0 : (cB ? daB : daC);
  const double rs = nofma::do_sin(a, da), rc = nofma::do_cos(a, da);
  if (k < 0x3e400000u) {
    sx = x;
    cx = 1.0;
  } else if (cA) {
    sx = rs;
    cx = rc;
  } else if (cB) {
    sx = copysign_(rc, x);
    cx = rs;
  } else {
    const double s0 = (n & 1) ? rc : rs, c0 = ((n + 1) & 1) ? rc : rs;
    sx = (n & 2) ? -s0 : s0;
    cx = ((n + 1) & 2) ? -c0 : c0;
  }
}

CLRRT_HD inline void sin_cos_fma_sel(double x, double& sx, double& cx) {
  const uint32_t k = hi_word(x) & 0x7fffffffu;
  if (!(k < 0x419921fbu)) {
    sx = sin(x);
    cx = cos(x);
    return;
  }
  const bool cA = k < 0x3feb6000u, cB = !cA && k < 0x400368fdu;
  const double y = hp0 - fabs(x);
  const double aB = y + hp1, daB = (y - aB) + hp1;  // cos, case B: do_sin
  double aC, daC;
  const int n = reduce_sincos(x, aC, daC);
  const double as = cA ? x : (cB ? aB : aC), das = cA ? 0.0 : (cB ? daB : daC);
  const double ac = cA ? x : (cB ? y : aC), dac = cA ? 0.0 : (cB ? hp1 : daC);  // sin, case B: do_cos(y, hp1)
  const double rs = do_sin(as, das), rc = do_cos(ac, dac);
  if (k < 0x3e500000u) sx = x;
  else if (cA) sx = rs;
  else if (cB) sx = copysign_(rc, x);
  else {
    const double s0 = (n & 1) ? rc : rs;
    sx = (n & 2) ? -s0 : s0;
  }
  if (k < 0x3e400000u) cx = 1.0;
  else if (cA) cx = rc;
  else if (cB) cx = rs;
  else {
    const double c0 = ((n + 1) & 1) ? rc : rs;
    cx = ((n + 1) & 2) ? -c0 : c0;
  }
}

// The rollout step's trigonometry -- sincos(x2) (generic build), sin(x2) and cos(x2) (FMA build), tan(x3) --
// as one branch-free block, so the five independent evaluation chains (two reductions, four table-driven
// do_sin/do_cos, tan's polynomial or xfg row) interleave instead of running one basic block after another.
// Every branch of the functions above becomes a select between values computed on both sides (the side
// not taken reads valid table rows: the reduced arguments stay below pi/4, tan's row index is clamped), so
// the results are theirs bit for bit.  Returns false (nothing written) outside the block's domain:
// |x2| >= 105414350, |x3| > tan_g3 or non-finite arguments; the caller then takes the branched functions.
namespace bf {
CLRRT_HD inline double do_sin_fma(double x, double dx) {
  const double t = taylor_sin(x, dx), tab = do_sin_tab(x, dx);
  return fabs(x) < taylor_lim ? t : tab;
}
CLRRT_HD inline double do_sin_nofma(double x, double dx) {
  const double t = nofma::taylor_sin(x, dx);
  const double ddx = x <= 0 ? -dx : dx;
  const double u = big + fabs(x);
  const int k = lo_word(u) << 2;
  const double xr = fabs(x) - (u - big);
  const double xx = xr * xr;
  const double s = xr + (ddx + xr * xx * (sn3 + xx * sn5));
  const double c = xr * ddx + xx * (cs2 + xx * (cs4 + xx * cs6));
  const double* T = sincostab();
  const double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
  const double tab = copysign_(sn + cor, x);
  return fabs(x) < taylor_lim ? t : tab;
}
CLRRT_HD inline double tan_core(double x) {
  const double w = (x < 0.0) ? -x : x;
  const double x2 = x * x;
  double t = fma_(x2, d11, d9);
  t = fma_(x2, t, d7);
  t = fma_(x2, t, d5);
  t = fma_(x2, t, d3);
  const double poly = fma_(x * x2, t, x);
  int i = (int)fma_(w, two8, mfftnhf);
  i = i < 0 ? 0 : i;  // (rows below the table serve only the unselected side)
  const double* row = xfg() + 4 * i;
  const double z = w - row[0];
  const double z2 = z * z;
  const double pz = fma_(z * z2, fma_(z2, e1, e0), z);
  const double fi = row[1], gi = row[2];
  const double y = ((fi + gi) * pz) / (gi - pz) + fi;
  const double tab = (x >= 0.0 ? 1.0 : -1.0) * y;
  return w <= tan_g1 ? x : (w <= tan_g2 ? poly : tab);
}
}  // namespace bf

CLRRT_HD inline bool step_trig(double x2, double x3, double& s2, double& c2, double& swp, double& cwp, double& t3) {
  const uint32_t k = hi_word(x2) & 0x7fffffffu;
  if (!(k < 0x419921fbu) || !(fabs(x3) <= tan_g3)) return false;
  const bool cA = k < 0x3feb6000u, cB = !cA && k < 0x400368fdu;
  const double y = hp0 - fabs(x2);
  const double aB = y + hp1, daB = (y - aB) + hp1;
  // sincos (generic build): one do_sin and one do_cos on the case's arguments
  double aCn, daCn;
  const int nn = nofma::reduce_sincos(x2, aCn, daCn);
  const double an = cA ? x2 : (cB ? aB : aCn), dan = cA ? 0.0 : (cB ? daB : daCn);
  // sin, cos (FMA build): cos's case B is do_sin(aB, daB), sin's is do_cos(y, hp1)
  double aCf, daCf;
  const int nf = reduce_sincos(x2, aCf, daCf);
  const double as = cA ? x2 : (cB ? aB : aCf), das = cA ? 0.0 : (cB ? daB : daCf);
  const double ac = cA ? x2 : (cB ? y : aCf), dac = cA ? 0.0 : (cB ? hp1 : daCf);
  const double rsn = bf::do_sin_nofma(an, dan), rcn = nofma::do_cos(an, dan);
  const double rsf = bf::do_sin_fma(as, das), rcf = do_cos(ac, dac);
  const double tn = bf::tan_core(x3);
  // sincos_sel's selection
  {
    const double s0 = (nn & 1) ? rcn : rsn, c0 = ((nn + 1) & 1) ? rcn : rsn;
    const double sC = (nn & 2) ? -s0 : s0, cC = ((nn + 1) & 2) ? -c0 : c0;
    s2 = k < 0x3e400000u ? x2 : (cA ? rsn : (cB ? copysign_(rcn, x2) : sC));
    c2 = k < 0x3e400000u ? 1.0 : (cA ? rcn : (cB ? rsn : cC));
  }
  // sin_cos_fma_sel's selection
  {
    const double s0 = (nf & 1) ? rcf : rsf, c0 = ((nf + 1) & 1) ? rcf : rsf;
    const double sC = (nf & 2) ? -s0 : s0, cC = ((nf + 1) & 2) ? -c0 : c0;
    swp = k < 0x3e500000u ? x2 : (cA ? rsf : (cB ? copysign_(rcf, x2) : sC));
    cwp = k < 0x3e400000u ? 1.0 : (cA ? rcf : (cB ? rsf : cC));
  }
  t3 = tn;
  return true;
}

// ------------------------------------------------------------------------------- float sincosf
// glibc 2.35 sincosf (sysdeps/ieee754/flt-32/s_sincosf.c + sincosf.h; the FMA variant libm's ifunc
// selects on FMA+AVX2 hosts): the float argument is widened to double, reduced by a Cody-Waite step
// (|y| < 120) or the Payne-Hanek reduce_large (2/pi bits __inv_pio4), and sin/cos come from two
// double polynomials rounded once to float.  The reference's OBB::setVertices calls cos(o) and
// sin(o) of its float angle, which GCC merges into sincosf (rrt/src/old_collisioncheck.cpp:56-65).
// The second table of glibc (quadrants 2 and 3) is the first with c0..c4 negated; as every rounding
// is symmetric, the cos polynomial is evaluated with the first table and negated.  Checked against
// the host libm on all 2^32 floats (tests/native/sincosf_check.cpp).
constexpr double kSincosf[28] = CLRRT_GLIBC_SINCOSF_TAB;
constexpr double sf_hpi_inv = kSincosf[4], sf_hpi = kSincosf[5];
constexpr double sf_c0 = kSincosf[6], sf_c1 = kSincosf[7], sf_s1 = kSincosf[8], sf_c2 = kSincosf[9];
constexpr double sf_s2 = kSincosf[10], sf_c3 = kSincosf[11], sf_s3 = kSincosf[12], sf_c4 = kSincosf[13];

CLRRT_HD inline uint32_t fbits(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return u;
}
CLRRT_HD inline uint32_t abstop12f(float x) { return (fbits(x) >> 20) & 0x7ff; }

// sincosf_poly (sincosf.h) with x the reduced argument times the quadrant sign; negc: table 1
CLRRT_HD inline void sincosf_poly(double x, double x2, int n, bool negc, float& sinp, float& cosp) {
  const double x4 = x2 * x2;
  const double x3 = x2 * x;
  const double c2 = fma_(x2, sf_c4, sf_c3);
  const double s1 = fma_(x2, sf_s3, sf_s2);
  const double c1 = fma_(x2, sf_c1, sf_c0);
  const double x5 = x3 * x2;
  const double x6 = x4 * x2;
  const double s = fma_(x3, sf_s1, x);
  const double c = fma_(x4, sf_c2, c1);
  const float sv = (float)fma_(x5, s1, s);
  float cv = (float)fma_(x6, c2, c);
  if (negc) cv = -cv;
  if (n & 1) { sinp = cv; cosp = sv; }
  else { sinp = sv; cosp = cv; }
}

CLRRT_HD inline void sincosf(float y, float& sinp, float& cosp) {
  double x = y;
  const uint32_t t = abstop12f(y);
  if (t < abstop12f(0x1.921FB6p-1f)) {  // |y| < pi/4
    const double x2 = x * x;
    if (t < abstop12f(0x1p-12f)) { sinp = y; cosp = 1.0f; return; }
    sincosf_poly(x, x2, 0, false, sinp, cosp);
  } else if (t < abstop12f(120.0f)) {
    // reduce_fast (no TOINT intrinsics on x86-64): the quadrant lands in bits 24..31 of r
    const double r = x * sf_hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = fma_(-(double)n, sf_hpi, x);
    const double sg = (((n >> 1) ^ n) & 1) ? -1.0 : 1.0;  // sign[n & 3] = {1, -1, -1, 1}
    sincosf_poly(x * sg, x * x, n, (n & 2) != 0, sinp, cosp);
  } else if (t < abstop12f(__builtin_inff())) {
    // reduce_large: Payne-Hanek with 96 bits of 2/pi selected by the exponent
    constexpr uint32_t inv_pio4[24] = CLRRT_GLIBC_INV_PIO4;
    uint32_t xi = fbits(y);
    const int sign = xi >> 31;
    const int k = (xi >> 26) & 15;
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint32_t)(xi * inv_pio4[k]);
    const uint64_t res1 = (uint64_t)xi * inv_pio4[k + 4];
    const uint64_t res2 = (uint64_t)xi * inv_pio4[k + 8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t nn = (res0 + (1ULL << 61)) >> 62;
    res0 -= nn << 62;
    const int n = (int)nn;
    x = (double)(int64_t)res0 * 0x1.921FB54442D18p-62;
    const int q = n + sign;
    const double sg = (((q >> 1) ^ q) & 1) ? -1.0 : 1.0;
    sincosf_poly(x * sg, x * x, n, (q & 2) != 0, sinp, cosp);
  } else {
    sinp = cosp = y - y;
  }
}

// glibc sinf (s_sinf.c): the same reduction and sin polynomial as sincosf (checked bit for bit on all
// floats by tests/native/sincosf_check.cpp)
CLRRT_HD inline float sinf(float y) {
  float s, c;
  sincosf(y, s, c);
  return s;
}

// --------------------------------------------------------------------------------- double atan2
// glibc 2.35 atan2 (sysdeps/ieee754/dbl-64/e_atan2.c, IBM Accurate Mathematical Library; the FMA variant
// libm's ifunc selects on FMA+AVX2 hosts, whose build contracts the EMULV product error and the
// polynomials into fused multiply-adds): special cases, de = exponent difference cut-offs, 2^+-500
// scaling, then u = min/max of |x|, |y| with its division residual du, and atan(u) either from an odd
// polynomial (u < 1/16) or from the cij table row of the 1/256 grid point nearest u (uatan2.tbl), in the
// quadrant form (i) x > 0, |y| < |x|; (ii) x > 0, |x| <= |y|; (iii) x < 0, |x| < |y|; (iv) x < 0,
// |y| <= |x|, with EADD / ESUB double-double corrections.  The reference's feasibleNode angles
// (rrtplanner.cpp:273-274), feasibleGoalBias' angleRef (:305) and sampleAroundVehicle's goal heading
// (:189) call it; restated so that every decision compares the reference's own angles.  Checked bit for
// bit against the host libm (tests/native/atan2_check.cpp).  The default rounding mode is assumed (the
// library's SET_RESTORE_ROUND is a no-op then).
#if defined(__HIPCC__)
static __device__ __constant__ double d_atan2_cij[ATAN2_CIJ_ROWS * 7] = CLRRT_GLIBC_ATAN2_CIJ;
#endif
static const double h_atan2_cij[ATAN2_CIJ_ROWS * 7] = CLRRT_GLIBC_ATAN2_CIJ;

// the cij row of u in [1/16, 1]: i = (TWO52 + TWO8 * u) - TWO52 (one rounding), minus 16
CLRRT_HD inline __attribute__((always_inline)) const double* atan2_row(double u) {
  const int i = (int)(fma_(u, at_two8, at_two52) - at_two52) - 16;
#if defined(__HIP_DEVICE_COMPILE__)
  return d_atan2_cij + 7 * i;
#else
  return h_atan2_cij + 7 * i;
#endif
}
// d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13)))), contracted
CLRRT_HD inline __attribute__((always_inline)) double atan2_poly(double v) {
  double p = fma_(v, at_d13, at_d11);
  p = fma_(v, p, at_d9);
  p = fma_(v, p, at_d7);
  p = fma_(v, p, at_d5);
  return fma_(v, p, at_d3);
}
// cij[2] + v (cij[3] + v (cij[4] + v (cij[5] + v cij[6]))), contracted
CLRRT_HD inline __attribute__((always_inline)) double atan2_tpoly(const double* c, double v) {
  double p = fma_(v, c[6], c[5]);
  p = fma_(v, p, c[4]);
  p = fma_(v, p, c[3]);
  return fma_(v, p, c[2]);
}

CLRRT_HD inline __attribute__((always_inline)) double atan2(double y, double x) {
  const uint32_t ux = hi_word(x), dx = (uint32_t)lo_word(x);
  const uint32_t uy = hi_word(y), dy = (uint32_t)lo_word(y);
  if ((ux & 0x7ff00000u) == 0x7ff00000u && ((ux & 0xfffffu) | dx) != 0) return x + y;  // x NaN
  if ((uy & 0x7ff00000u) == 0x7ff00000u && ((uy & 0xfffffu) | dy) != 0) return y + y;  // y NaN
  const bool xneg = (int32_t)ux < 0, yneg = (int32_t)uy < 0;
  if (uy == 0 && dy == 0) return xneg ? at_opi : 0.0;                   // y = +0
  if (uy == 0x80000000u && dy == 0) return xneg ? at_mopi : -0.0;       // y = -0
  if (x == 0) return yneg ? at_mhpi : at_hpi;
  if (dx == 0 && ux == 0x7ff00000u) {                                    // x = +inf
    if (dy == 0 && uy == 0x7ff00000u) return at_qpi;
    if (dy == 0 && uy == 0xfff00000u) return at_mqpi;
    return yneg ? -0.0 : 0.0;
  }
  if (dx == 0 && ux == 0xfff00000u) {                                    // x = -inf
    if (dy == 0 && uy == 0x7ff00000u) return at_tqpi;
    if (dy == 0 && uy == 0xfff00000u) return at_mtqpi;
    return yneg ? at_mopi : at_opi;
  }
  if (dy == 0 && uy == 0x7ff00000u) return at_hpi;                       // y = +inf
  if (dy == 0 && uy == 0xfff00000u) return at_mhpi;                      // y = -inf
  double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int32_t de = (int32_t)(uy & 0x7ff00000u) - (int32_t)(ux & 0x7ff00000u);
  if (de >= 59768832) return (0 < y) ? at_hpi : at_mhpi;                 // 57 * 16^5
  if (de <= -59768832) {
    if (x > 0) return copysign_(ay / ax, y);
    return (0 < y) ? at_opi : at_mopi;
  }
  if (ax < at_twom500 || ay < at_twom500) { ax *= at_two500; ay *= at_two500; }
  if (ax > at_two500 || ay > at_two500) { ax *= at_twom500; ay *= at_twom500; }
  double u, du;
  if (ay < ax) {
    u = ay / ax;
    const double v = ax * u, vv = fma_(ax, u, -v);
    du = ((ay - v) - vv) / ax;
  } else {
    u = ax / ay;
    const double v = ay * u, vv = fma_(ay, u, -v);
    du = ((ax - v) - vv) / ay;
  }
  double z;
  if (x > 0) {
    if (ay < ax) {  // (i) atan(ay / ax)
      if (u < at_inv16) {
        const double v = u * u;
        z = u + fma_(u * v, atan2_poly(v), du);
      } else {
        const double* c = atan2_row(u);
        const double t3 = u - c[0];
        const double v = t3 + du;  // EADD (t3, du, v, dv)
        const double dv = (fabs(t3) > fabs(du)) ? (t3 - v) + du : (du - v) + t3;
        double p = fma_(v, c[6], c[5]);
        p = fma_(v, p, c[4]);
        p = fma_(v, p, c[3]);
        double q = fma_(dv, c[2], (v * v) * p);
        z = fma_(v, c[2], q) + c[1];
      }
    } else {  // (ii) pi/2 - atan(ax / ay)
      if (u < at_inv16) {
        const double v = u * u;
        const double zz = (u * v) * atan2_poly(v);
        const double t2 = at_hpi - u;  // ESUB (hpi, u, t2, cor)
        const double cor = (at_hpi > fabs(u)) ? (at_hpi - t2) - u : at_hpi - (u + t2);
        z = (((cor + at_hpi1) - du) - zz) + t2;
      } else {
        const double* c = atan2_row(u);
        const double v = (u - c[0]) + du;
        z = (at_hpi - c[1]) + fma_(-v, atan2_tpoly(c, v), at_hpi1);
      }
    }
  } else if (ax < ay) {  // (iii) pi/2 + atan(ax / ay)
    if (u < at_inv16) {
      const double v = u * u;
      const double zz = (v * u) * atan2_poly(v);
      const double t2 = u + at_hpi;  // EADD (hpi, u, t2, cor)
      const double cor = (at_hpi > fabs(u)) ? (at_hpi - t2) + u : (u - t2) + at_hpi;
      z = (((cor + at_hpi1) + du) + zz) + t2;
    } else {
      const double* c = atan2_row(u);
      const double v = (u - c[0]) + du;
      z = (at_hpi + c[1]) + fma_(v, atan2_tpoly(c, v), at_hpi1);
    }
  } else {  // (iv) pi - atan(ay / ax)
    if (u < at_inv16) {
      const double v = u * u;
      const double zz = (v * u) * atan2_poly(v);
      const double t2 = at_opi - u;  // ESUB (opi, u, t2, cor)
      const double cor = (at_opi > fabs(u)) ? (at_opi - t2) - u : at_opi - (t2 + u);
      z = (((cor + at_opi1) - du) - zz) + t2;
    } else {
      const double* c = atan2_row(u);
      const double v = (u - c[0]) + du;
      z = (at_opi - c[1]) + fma_(-v, atan2_tpoly(c, v), at_opi1);
    }
  }
  return copysign_(z, y);
}

// exp (sysdeps/ieee754/dbl-64/e_exp.c, glibc 2.35, as its FMA ifunc variant __exp_fma evaluates it): x =
// k ln2/128 + r, exp(x) = 2^(k/128) exp(r) with 2^(k/128) = scale (1 + tail) from __exp_data.tab and a degree-5
// polynomial; the FMA build contracts the reduction, the polynomial and the final scale + scale * tmp, not the
// out-of-line specialcase (|x| >= 512).  Checked against the host libm bit for bit on 4e7 arguments
// (development check) and on the device by tests/test_gpu_math.py.  Used by the W2 obstacle-cost term
// Wcost[2] exp(-Wcost[3] Dobs) (simulation.cpp:91, rrtplanner.cpp:112).
#if defined(__HIPCC__)
static __device__ __constant__ uint64_t d_exp_tab[256] = CLRRT_GLIBC_EXP_TAB;
#endif
static const uint64_t h_exp_tab[256] = CLRRT_GLIBC_EXP_TAB;
CLRRT_HD inline double from_bits(uint64_t u) {
  double r;
  memcpy(&r, &u, 8);
  return r;
}
CLRRT_HD inline uint64_t exp_tab(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return d_exp_tab[i];
#else
  return h_exp_tab[i];
#endif
}
CLRRT_HD inline double exp_specialcase(double tmp, uint64_t sbits, uint64_t ki) {
  double scale, y;
  if ((ki & 0x80000000) == 0) {  // k > 0: the exponent of scale might have overflowed by <= 460
    sbits -= 1009ull << 52;
    scale = from_bits(sbits);
    y = 0x1p1009 * (scale + scale * tmp);
    return y;
  }
  // k < 0: the result may be subnormal; avoid double rounding
  sbits += 1022ull << 52;
  scale = from_bits(sbits);
  y = scale + scale * tmp;
  if (y < 1.0) {
    double lo = scale - y + scale * tmp;
    const double hi = 1.0 + y;
    lo = 1.0 - hi + y + lo;
    y = (hi + lo) - 1.0;
    if (y == 0) y = 0.0;  // -0 -> +0
  }
  return 0x1p-1022 * y;
}
CLRRT_HD inline double exp(double x) {
  uint32_t abstop = (uint32_t)(bits(x) >> 52) & 0x7ff;
  const uint32_t t_tiny = 0x3c9, t_512 = 0x408, t_1024 = 0x409;  // top12 of 2^-54, 512, 1024
  if (abstop - t_tiny >= t_512 - t_tiny) {
    if ((int32_t)(abstop - t_tiny) < 0) return 1.0 + x;  // tiny x (0 included)
    if (abstop >= t_1024) {
      if (bits(x) == 0xfff0000000000000ull) return 0.0;  // -inf
      if (abstop >= 0x7ff) return 1.0 + x;               // +inf, NaN
      return (bits(x) >> 63) ? 0.0 : from_bits(0x7ff0000000000000ull);  // underflow / overflow
    }
    abstop = 0;  // large |x|: specialcase below
  }
  const double z = exp_invln2N * x;
  double kd = z + exp_shift;
  const uint64_t ki = bits(kd);
  kd -= exp_shift;
  const double r = fma_(kd, exp_negln2loN, fma_(kd, exp_negln2hiN, x));
  const int idx = 2 * (int)(ki % 128);
  const uint64_t top = ki << 45;
  const double tail = from_bits(exp_tab(idx));
  const uint64_t sbits = exp_tab(idx + 1) + top;
  const double r2 = r * r;
  const double tmp = fma_(r2 * r2, fma_(r, exp_C5, exp_C4), fma_(r2, fma_(r, exp_C3, exp_C2), tail + r));
  if (abstop == 0) return exp_specialcase(tmp, sbits, ki);
  const double scale = from_bits(sbits);
  return fma_(scale, tmp, scale);
}

}  // namespace glibc
}  // namespace clrrt
