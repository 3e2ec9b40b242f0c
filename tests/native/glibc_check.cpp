// Bit-exactness of clrrt_glibc.hpp (the GPU restatement of glibc's double sin/cos/tan) against the
// system libm on this host (glibc 2.35, FMA variants).  Prints mismatch counts; exit 1 on any.
#define _GNU_SOURCE 1
#include <math.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../cl-rrt_amd/csrc/clrrt_glibc.hpp"

static uint64_t b(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
// one libm call per non-inlinable wrapper: GCC cannot merge them into sincos here
__attribute__((noinline)) static double lsin(double x) { return ::sin(x); }
__attribute__((noinline)) static double lcos(double x) { return ::cos(x); }
__attribute__((noinline)) static double ltan(double x) { return ::tan(x); }
__attribute__((noinline)) static void lsincos(double x, double* s, double* c) { ::sincos(x, s, c); }

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 rng(42);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  long bs = 0, bc = 0, bt = 0, bsc = 0, ns = 0, nt = 0;
  double ranges[] = {1e-9, 1e-3, 0.126, 0.5, 0.855, 1.0, 2.4, 3.2, 6.3, 30.0, 1e4, 1e8};
  for (long i = 0; i < n; i++) {
    double r = ranges[i % 12];
    double x = (u01(rng) * 2 - 1) * r;
    if (i % 97 == 0) x = std::nextafter(0.85546875, (i & 1) ? 0.0 : 1.0) * ((i & 2) ? -1 : 1);
    if (i % 89 == 0) x = (double)(i % 1000) * 0.001;  // headings / steering on a grid
    ns++;
    if (b(clrrt::glibc::sin(x)) != b(lsin(x))) { if (bs < 5) printf("sin %.17g: %a vs %a\n", x, clrrt::glibc::sin(x), lsin(x)); bs++; }
    if (b(clrrt::glibc::cos(x)) != b(lcos(x))) { if (bc < 5) printf("cos %.17g: %a vs %a\n", x, clrrt::glibc::cos(x), lcos(x)); bc++; }
    double ss, cc, gs, gc;
    lsincos(x, &ss, &cc);
    clrrt::glibc::sincos(x, gs, gc);
    if (b(ss) != b(gs) || b(cc) != b(gc)) { if (bsc < 5) printf("sincos %.17g: %a %a vs %a %a\n", x, gs, gc, ss, cc); bsc++; }
    double xt = (u01(rng) * 2 - 1) * 0.786;
    nt++;
    if (b(clrrt::glibc::tan(xt)) != b(ltan(xt))) { if (bt < 5) printf("tan %.17g: %a vs %a\n", xt, clrrt::glibc::tan(xt), ltan(xt)); bt++; }
  }
  printf("sin/cos %ld args: sin mismatches %ld, cos mismatches %ld, sincos mismatches %ld; tan %ld args: mismatches %ld\n", ns, bs, bc, bsc, nt, bt);
  return (bs || bc || bt || bsc) ? 1 : 0;
}
