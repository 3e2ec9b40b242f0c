// Bit-exactness of clrrt_glibcf.hpp (device restatements of glibc 2.35's float atanf, acosf, asinf and
// atan2f) against the host libm: every float for the one-argument functions (stride argv[1]), and
// argv[2] random + edge-case pairs for atan2f.  Prints mismatch counts; exit 1 on any.
#define _GNU_SOURCE 1
#include <math.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <omp.h>
#include <utility>

#include "../../cl-rrt_amd/csrc/clrrt_glibcf.hpp"

static uint32_t fb(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static bool same(float a, float b) { return fb(a) == fb(b) || (a != a && b != b); }
__attribute__((noinline)) static float l_atanf(float x) { return ::atanf(x); }
__attribute__((noinline)) static float l_acosf(float x) { return ::acosf(x); }
__attribute__((noinline)) static float l_asinf(float x) { return ::asinf(x); }
__attribute__((noinline)) static float l_atan2f(float y, float x) { return ::atan2f(y, x); }

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  const long npairs = argc > 2 ? atol(argv[2]) : 100000000;
  long bad[4] = {0, 0, 0, 0}, checked = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : checked)
  for (int64_t hi = 0; hi < 65536; hi++) {
    long b0 = 0, b1 = 0, b2 = 0;
    for (uint64_t lo = 0; lo < 65536; lo += stride) {
      uint32_t u = (uint32_t)((hi << 16) | lo);
      float x;
      memcpy(&x, &u, 4);
      checked++;
      if (!same(l_atanf(x), clrrt::glibcf::atanf(x))) {
        if (b0++ < 1 && hi % 4096 == 0) printf("atanf(%a): libm %a port %a\n", (double)x, (double)l_atanf(x), (double)clrrt::glibcf::atanf(x));
      }
      if (!same(l_acosf(x), clrrt::glibcf::acosf(x))) {
        if (b1++ < 1 && hi % 4096 == 0) printf("acosf(%a): libm %a port %a\n", (double)x, (double)l_acosf(x), (double)clrrt::glibcf::acosf(x));
      }
      if (!same(l_asinf(x), clrrt::glibcf::asinf(x))) {
        if (b2++ < 1 && hi % 4096 == 0) printf("asinf(%a): libm %a port %a\n", (double)x, (double)l_asinf(x), (double)clrrt::glibcf::asinf(x));
      }
    }
#pragma omp atomic
    bad[0] += b0;
#pragma omp atomic
    bad[1] += b1;
#pragma omp atomic
    bad[2] += b2;
  }
  const float edge[] = {0.0f, -0.0f, 1.0f, -1.0f, 4.77f, -4.77f, 1e-30f, -1e-30f, 1e30f, -1e30f,
                        INFINITY, -INFINITY, NAN, 1e-45f, 3.0f, 0.5f};
#pragma omp parallel
  {
    std::mt19937_64 rng(1234 + 17 * (uint64_t)omp_get_thread_num());
    long b3 = 0;
#pragma omp for
    for (long i = 0; i < npairs; i++) {
      float y, x;
      const uint64_t r = rng();
      switch (i % 4) {
        case 0: { uint32_t a = (uint32_t)r, b = (uint32_t)(r >> 32); memcpy(&y, &a, 4); memcpy(&x, &b, 4); } break;
        case 1: y = (float)((double)(r & 0xffffffff) / 4294967296.0 * 120 - 60);
                x = (float)((double)(r >> 32) / 4294967296.0 * 120 - 60); break;
        case 2: y = edge[r % 16]; x = (float)((double)(r >> 32) / 4294967296.0 * 20 - 10); if (r & 16) std::swap(x, y); break;
        default: y = (float)((double)(r & 0xffffffff) / 4294967296.0 * 40 - 20); x = 4.77f - (float)((double)(r >> 32) / 4294967296.0 * 60); break;
      }
      if (!same(l_atan2f(y, x), clrrt::glibcf::atan2f(y, x))) {
        if (b3++ < 3) printf("atan2f(%a, %a): libm %a port %a\n", (double)y, (double)x, (double)l_atan2f(y, x), (double)clrrt::glibcf::atan2f(y, x));
      }
    }
#pragma omp atomic
    bad[3] += b3;
  }
  printf("%ld floats: atanf mismatches %ld, acosf mismatches %ld, asinf mismatches %ld; %ld pairs: atan2f mismatches %ld\n",
         checked, bad[0], bad[1], bad[2], npairs, bad[3]);
  return (bad[0] || bad[1] || bad[2] || bad[3]) ? 1 : 0;
}
