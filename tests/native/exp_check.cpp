// clrrt::glibc::exp (cl-rrt_amd/csrc/clrrt_glibc.hpp, the restatement of glibc 2.35's __exp_fma) against the
// host libm's exp, bit for bit: uniform arguments over [-750, 10] (normal, subnormal and underflowing
// results), the -W3 * Dobs range of the obstacle cost term, [-1, 1], and random bit patterns.  CPU only.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../cl-rrt_amd/csrc/clrrt_glibc_data.hpp"
#include "../../cl-rrt_amd/csrc/clrrt_glibc.hpp"

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4000000;
  uint64_t s = 88172645463325252ull;
  long bad = 0;
  const double specials[] = {0.0, -0.0, 1e-300, -1e-300, 709.78, 709.79, -708.39, -745.13, -745.14, -1e4, 1e4,
                             INFINITY, -INFINITY, NAN, 512.0, -512.0, 1024.0, -1024.0};
  for (double x : specials) {
    const double a = std::exp(x), g = clrrt::glibc::exp(x);
    uint64_t ua, ug;
    memcpy(&ua, &a, 8);
    memcpy(&ug, &g, 8);
    if (ua != ug && !(a != a && g != g)) { printf("special %a: libm %a restated %a\n", x, a, g); bad++; }
  }
  for (long i = 0; i < n; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    double x;
    if (i % 4 == 0) x = ((s >> 11) * 0x1p-53) * (-760.0) + 10.0;
    else if (i % 4 == 1) x = -((s >> 11) * 0x1p-53) * 260.0;
    else if (i % 4 == 2) x = ((s >> 11) * 0x1p-53 - 0.5) * 2.0;
    else {
      const uint64_t u = ((s & 0x7fefffffffffffffull) >> 1) | (s & 0x8000000000000000ull);
      memcpy(&x, &u, 8);
    }
    const double a = std::exp(x), g = clrrt::glibc::exp(x);
    uint64_t ua, ug;
    memcpy(&ua, &a, 8);
    memcpy(&ug, &g, 8);
    if (ua != ug && !(a != a && g != g)) {
      if (bad < 5) printf("%a: libm %a restated %a\n", x, a, g);
      bad++;
    }
  }
  printf("exp mismatches %ld of %ld\n", bad, n);
  return bad != 0;
}
