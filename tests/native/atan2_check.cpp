// Bit-exactness of clrrt::glibc::atan2 (clrrt_glibc.hpp, the GPU restatement of glibc 2.35's double
// atan2) against the system libm on this host (FMA variant).  Prints mismatch counts; exit 1 on any.
#include <math.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>

#include "../../cl-rrt_amd/csrc/clrrt_glibc.hpp"

static uint64_t b(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
__attribute__((noinline)) static double latan2(double y, double x) { return ::atan2(y, x); }

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 4000000;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  long bad = 0;
  auto check = [&](double y, double x) {
    double g = clrrt::glibc::atan2(y, x), w = latan2(y, x);
    bool same = b(g) == b(w) || (std::isnan(g) && std::isnan(w));
    if (!same) { if (bad < 8) printf("atan2(%a, %a): %a vs %a\n", y, x, g, w); bad++; }
  };
  const double sp[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, 1e-310, -1e-310, 1e300, -1e300, 5e-324,
                       2.2250738585072014e-308, 0.0625, 1e-160, 1e160};
  for (double y : sp)
    for (double x : sp) check(y, x);
  const double scales[] = {1e-300, 1e-160, 1e-20, 1e-3, 0.1, 1.0, 3.0, 50.0, 1e6, 1e20, 1e160, 1e300};
  for (long i = 0; i < n; i++) {
    double s1 = scales[i % 12], s2 = scales[(i / 12) % 12];
    double y = (u01(rng) * 2 - 1) * s1, x = (u01(rng) * 2 - 1) * s2;
    if (i % 5 == 0) x = (u01(rng) * 2 - 1) * s1;  // similar magnitudes (|u| near 1, the table's end)
    if (i % 7 == 0) { double a = (u01(rng) * 2 - 1) * 3.2; double r = u01(rng) * 50; y = r * std::sin(a); x = r * std::cos(a); }
    if (i % 11 == 0) { double r = 0.2 + u01(rng) * 40; double a = (i & 1 ? 1 : -1) * 0.7853981633974483 + (u01(rng) - 0.5) * 1e-12;
                       y = r * std::sin(a); x = r * std::cos(a); }  // near the pi/4 limit of feasibleNode
    check(y, x);
  }
  printf("atan2 %ld args: mismatches %ld\n", n, bad);
  return bad ? 1 : 0;
}
