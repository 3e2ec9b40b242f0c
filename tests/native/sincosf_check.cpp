// Bit-exactness of clrrt::glibc::sincosf (the device restatement of glibc 2.35's float sincosf) against
// the host libm's sincosf, sinf and cosf over all 2^32 float bit patterns (OpenMP).  Prints mismatch counts; exit 1 on any.
#define _GNU_SOURCE 1
#include <math.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../cl-rrt_amd/csrc/clrrt_glibc.hpp"

static uint32_t fb(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;  // 1: every float
  long bad = 0, checked = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : bad, checked)
  for (int64_t hi = 0; hi < 65536; hi++) {
    for (uint64_t lo = 0; lo < 65536; lo += stride) {
      uint32_t u = (uint32_t)((hi << 16) | lo);
      float y;
      memcpy(&y, &u, 4);
      float s1, c1, s2, c2;
      ::sincosf(y, &s1, &c1);
      clrrt::glibc::sincosf(y, s2, c2);
      const float s3 = ::sinf(y), c3 = ::cosf(y), s4 = clrrt::glibc::sinf(y);
      checked++;
      bool ok = (fb(s1) == fb(s2) || (s1 != s1 && s2 != s2)) && (fb(c1) == fb(c2) || (c1 != c1 && c2 != c2)) &&
                (fb(s3) == fb(s4) || (s3 != s3 && s4 != s4)) && (fb(c3) == fb(c2) || (c3 != c3 && c2 != c2));
      if (!ok) {
        if (bad < 8) {
#pragma omp critical
          printf("sincosf(%a): libm %a %a, port %a %a\n", (double)y, (double)s1, (double)c1, (double)s2, (double)c2);
        }
        bad++;
      }
    }
  }
  printf("sincosf %ld floats: mismatches %ld\n", checked, bad);
  return bad ? 1 : 0;
}
