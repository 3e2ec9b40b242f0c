// The partition argument of wave_std_sort (cl-rrt_amd/csrc/clrrt_kernels.hip) checked on the host: its
// algorithm -- both scans' stop positions found 64 at a time on the range as it was, paired, swapped
// after the crossing, the cut at L_k or R_{k-1} -- with the 64 lanes written as loops, against the
// sequential std_sort replay (clrrt_stdsort.hpp, itself checked against libstdc++ by stdsort_check.cpp)
// on 20000 tie-heavy, presorted and reversed sequences.  The device kernel's own output is checked by
// the EXACT-mode tree and candidate-list parity tests.
#include <cstdio>
#include <cstdlib>
#include <climits>
#include <vector>
#include <random>
#include <algorithm>
#include "../../cl-rrt_amd/csrc/clrrt_stdsort.hpp"
using namespace clrrt;
struct I2 { int x, y; };
static void wave_sort(KeyId* a, int n, I2* pairs) {
  if (n <= 1) return;
  struct Rg { int lo, hi, depth; };
  Rg stack[64]; int sp = 0; int lo = 0, hi = n; int depth = 2 * ilog2(n);
  int s_l[64], s_r[64];
  for (;;) {
    while (hi - lo > 16) {
      if (depth == 0) { heap_sort_(a + lo, hi - lo); break; }
      --depth;
      { KeyId* first = a + lo; KeyId* last = a + hi; median_to_first_(first, first + 1, first + (last - first) / 2, last - 1); }
      const float P = a[lo].key;
      const int f = lo + 1, l = hi;
      int lpos = f, rpos = l - 1, nl = 0, hl = 0, nr = 0, hr = 0, np = 0, prevR = INT_MAX, cut = -1;
      while (cut < 0) {
        if (nl == 0) { int c = 0; for (int ln = 0; ln < 64; ln++) { int i = lpos + ln; if (i < l && !(a[i].key < P)) s_l[c++] = i; } nl = c; hl = 0; lpos += 64; }
        if (nr == 0) { int c = 0; for (int ln = 0; ln < 64; ln++) { int i = rpos - ln; if (i >= f && !(P < a[i].key)) s_r[c++] = i; } nr = c; hr = 0; rpos -= 64; }
        const bool lend = nl == 0 && lpos >= l, rend = nr == 0 && rpos < f;
        const int m = std::min(nl, nr);
        int kx = m; 
        for (int k = 0; k < m; k++) if (s_l[hl + k] >= s_r[hr + k]) { kx = k; break; }
        for (int k = 0; k < kx; k++) pairs[np + k] = I2{s_l[hl + k], s_r[hr + k]};
        const int prev = kx > 0 ? s_r[hr + kx - 1] : prevR;
        if (kx < m) { const int Lx = s_l[hl + kx]; cut = Lx < prev ? Lx : prev; }
        else if ((nl - m == 0 && lend) || (nr - m == 0 && rend)) {
          if (nl - m > 0) { const int Lx = s_l[hl + m]; cut = Lx < prev ? Lx : prev; }
          else cut = prev == INT_MAX ? l : prev;
        }
        np += kx; prevR = prev; nl -= m; hl += m; nr -= m; hr += m;
      }
      for (int k = 0; k < np; k++) { KeyId t = a[pairs[k].x]; a[pairs[k].x] = a[pairs[k].y]; a[pairs[k].y] = t; }
      stack[sp++] = Rg{cut, hi, depth}; hi = cut;
    }
    if (sp == 0) break;
    --sp; lo = stack[sp].lo; hi = stack[sp].hi; depth = stack[sp].depth;
  }
  if (n > 16) { insertion_sort_(a, a + 16); for (KeyId* i = a + 16; i != a + n; ++i) unguarded_linear_insert_(i); }
  else insertion_sort_(a, a + n);
}
int main() {
  std::mt19937 rng(1);
  long bad = 0, tot = 0;
  for (int t = 0; t < 20000; t++) {
    int n = 1 + rng() % (t % 10 == 0 ? 5000 : 600);
    int nv = 1 + rng() % (t % 3 == 0 ? 3 : (t % 3 == 1 ? 50 : 100000));
    std::vector<KeyId> a(n);
    for (int i = 0; i < n; i++) { a[i].id = i; a[i].key = (float)(rng() % nv) * 0.25f; }
    if (t % 7 == 0) std::sort(a.begin(), a.end(), [](const KeyId& x, const KeyId& y){ return x.key < y.key; });  // presorted
    if (t % 11 == 0) std::reverse(a.begin(), a.end());
    std::vector<KeyId> b = a;
    std::vector<I2> pr(n / 2 + 64);
    std_sort(a.data(), n);
    wave_sort(b.data(), n, pr.data());
    tot++;
    for (int i = 0; i < n; i++) if (a[i].id != b[i].id) { bad++; if (bad < 5) printf("mismatch t=%d n=%d nv=%d at %d\n", t, n, nv, i); break; }
  }
  printf("arrays %ld mismatches %ld\n", tot, bad);
  return bad != 0;
}
