// Checks clrrt_stdsort.hpp's replay of std::sort against the real libstdc++ std::sort on
// (id, float key) pairs with heavy ties, as sortNodesExplore (rrtplanner.cpp:227-247) sorts them.
#include <algorithm>
#include <cstdio>
#include <random>
#include <utility>
#include <vector>

#include "../../cl-rrt_amd/csrc/clrrt_stdsort.hpp"

int main() {
  std::mt19937 rng(1234);
  long bad = 0, cases = 0;
  for (int trial = 0; trial < 4000; trial++) {
    int n = 1 + (int)(rng() % (trial < 2000 ? 200 : 5000));
    int distinct = 1 + (int)(rng() % (trial % 3 == 0 ? 4 : 100000));
    std::vector<std::pair<int, float>> ref;
    std::vector<clrrt::KeyId> mine;
    for (int i = 0; i < n; i++) {
      float k = (float)(rng() % distinct) * 0.25f;
      if (trial % 7 == 0) k = (float)(n - i);  // descending runs
      if (trial % 11 == 0) k = 3.0f;           // all equal
      ref.push_back(std::make_pair(i, k));
      mine.push_back(clrrt::KeyId{i, k});
    }
    std::sort(ref.begin(), ref.end(),
              [](const std::pair<int, float>& a, const std::pair<int, float>& b) { return a.second < b.second; });
    clrrt::std_sort(mine.data(), (int64_t)mine.size());
    cases++;
    for (int i = 0; i < n; i++)
      if (ref[i].first != mine[i].id) { bad++; break; }
  }
  // heapsort fallback (__partial_sort(first, last, last) = make_heap + sort_heap)
  for (int trial = 0; trial < 2000; trial++) {
    int n = 1 + (int)(rng() % 3000);
    int distinct = 1 + (int)(rng() % (trial % 2 ? 5 : 100000));
    std::vector<std::pair<int, float>> ref;
    std::vector<clrrt::KeyId> mine;
    for (int i = 0; i < n; i++) {
      float k = (float)(rng() % distinct);
      ref.push_back(std::make_pair(i, k));
      mine.push_back(clrrt::KeyId{i, k});
    }
    auto cmp = [](const std::pair<int, float>& a, const std::pair<int, float>& b) { return a.second < b.second; };
    std::make_heap(ref.begin(), ref.end(), cmp);
    std::sort_heap(ref.begin(), ref.end(), cmp);
    clrrt::heap_sort_(mine.data(), (int64_t)mine.size());
    cases++;
    for (int i = 0; i < n; i++)
      if (ref[i].first != mine[i].id) { bad++; break; }
  }
  printf("cases %ld mismatching %ld\n", cases, bad);
  return bad != 0;
}
