// clrrt_stdsort.hpp — the exact permutation libstdc++'s std::sort (GCC 11, bits/stl_algo.h:
// __introsort_loop + __final_insertion_sort, with the __partial_sort heapsort fallback) produces
// on a sequence of (node id, key) pairs compared by key only.
//
// Why: sortNodesExplore / sortNodesOptimize (rrtplanner.cpp:227-268) std::sort pairs by a float
// key and then walk the result.  Trees routinely hold nodes with bit-identical keys (e.g. rollouts
// that stop after one step at the root state), so the order of equal keys — which std::sort leaves
// to its algorithm — decides which parent is expanded.  EXACT mode therefore replays the same
// algorithm on samples whose candidate list contains such a tie.  Usable on host (tests) and
// device (one lane per sample).
// Provenance: the algorithm restated is libstdc++'s std::sort (GCC 11, (C) the Free Software Foundation),
// distributed under the GNU General Public License v3 with the GCC Runtime Library Exception.
#pragma once
#include <stdint.h>

#ifndef CLRRT_HD
#if defined(__HIPCC__)
#define CLRRT_HD __host__ __device__
#else
#define CLRRT_HD
#endif
#endif

namespace clrrt {

struct KeyId {
  int32_t id;
  float key;
};

CLRRT_HD inline bool kless(const KeyId& a, const KeyId& b) { return a.key < b.key; }
CLRRT_HD inline void kswap(KeyId* a, KeyId* b) {
  KeyId t = *a;
  *a = *b;
  *b = t;
}
CLRRT_HD inline int ilog2(int64_t n) {
  int k = 0;
  while (n > 1) { n >>= 1; k++; }
  return k;
}

// --- heap (std::__make_heap / __adjust_heap / __push_heap / __pop_heap / __sort_heap)
CLRRT_HD inline void push_heap_(KeyId* f, int64_t hole, int64_t top, KeyId v) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && kless(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
CLRRT_HD inline void adjust_heap_(KeyId* f, int64_t hole, int64_t len, KeyId v) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (kless(f[child], f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  push_heap_(f, hole, top, v);
}
CLRRT_HD inline void heap_sort_(KeyId* f, int64_t n) {
  if (n >= 2) {  // make_heap
    int64_t parent = (n - 2) / 2;
    for (;;) {
      KeyId v = f[parent];
      adjust_heap_(f, parent, n, v);
      if (parent == 0) break;
      parent--;
    }
  }
  for (int64_t last = n; last > 1;) {  // sort_heap
    --last;
    KeyId v = f[last];
    f[last] = f[0];
    adjust_heap_(f, 0, last, v);
  }
}

// --- introsort pieces
CLRRT_HD inline void median_to_first_(KeyId* r, KeyId* a, KeyId* b, KeyId* c) {
  if (kless(*a, *b)) {
    if (kless(*b, *c)) kswap(r, b);
    else if (kless(*a, *c)) kswap(r, c);
    else kswap(r, a);
  } else if (kless(*a, *c)) {
    kswap(r, a);
  } else if (kless(*b, *c)) {
    kswap(r, c);
  } else {
    kswap(r, b);
  }
}
CLRRT_HD inline KeyId* unguarded_partition_(KeyId* first, KeyId* last, KeyId* pivot) {
  for (;;) {
    while (kless(*first, *pivot)) ++first;
    --last;
    while (kless(*pivot, *last)) --last;
    if (!(first < last)) return first;
    kswap(first, last);
    ++first;
  }
}
CLRRT_HD inline void unguarded_linear_insert_(KeyId* last) {
  KeyId v = *last;
  KeyId* next = last - 1;
  while (kless(v, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = v;
}
CLRRT_HD inline void insertion_sort_(KeyId* first, KeyId* last) {
  if (first == last) return;
  for (KeyId* i = first + 1; i != last; ++i) {
    if (kless(*i, *first)) {
      KeyId v = *i;
      for (KeyId* p = i; p != first; --p) *p = *(p - 1);
      *first = v;
    } else {
      unguarded_linear_insert_(i);
    }
  }
}

// std::sort(a, a + n, [](x, y){ return x.key < y.key; })
CLRRT_HD inline void std_sort(KeyId* a, int64_t n) {
  if (n <= 1) return;
  // __introsort_loop with an explicit stack: disjoint ranges are independent, so processing the
  // right part later instead of first does not change the result.
  struct Rg { int64_t lo, hi; int depth; };
  Rg stack[64];
  int sp = 0;
  int64_t lo = 0, hi = n;
  int depth = 2 * ilog2(n);
  for (;;) {
    while (hi - lo > 16) {
      if (depth == 0) {
        heap_sort_(a + lo, hi - lo);
        break;
      }
      --depth;
      KeyId* first = a + lo;
      KeyId* last = a + hi;
      KeyId* mid = first + (last - first) / 2;
      median_to_first_(first, first + 1, mid, last - 1);
      KeyId* cut = unguarded_partition_(first + 1, last, first);
      stack[sp++] = Rg{cut - a, hi, depth};
      hi = cut - a;
    }
    if (sp == 0) break;
    --sp;
    lo = stack[sp].lo;
    hi = stack[sp].hi;
    depth = stack[sp].depth;
  }
  // __final_insertion_sort
  if (n > 16) {
    insertion_sort_(a, a + 16);
    for (KeyId* i = a + 16; i != a + n; ++i) unguarded_linear_insert_(i);
  } else {
    insertion_sort_(a, a + n);
  }
}

}  // namespace clrrt
