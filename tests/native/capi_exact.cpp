// The C++ drop-in path end to end, linked against libclrrt (no Python, no ctypes): mirror types with the
// reference's field layout (rrt/include/rrt/rrtplanner.h:27-80, vehicle.h, car_msgs/Obstacle2D) go through
// include/clrrt_adapter.hpp exactly as the reference's own types would inside its unity build
// (INTEGRATION.md):
//   * 100 expandTree calls (one iteration each, rrtplanner.cpp:123-174) then the rest of 300 iterations
//     through the Timer-loop form, EXACT mode, 200-obstacle scene, srand(3);
//   * the tree (state bits, parent, float costs, goal flags, trajectory row hashes) and the counters
//     equal the CPU oracle's (tests/golden/capi_exact_obb200_s3.bin, tests/golden/make_capi_fixture.py);
//   * checkObsDistance (collision.h:41) on 48 states equals the oracle's bit for bit;
//   * the process's rand() stream and the engine's clrrt_rng stay equal.
// Usage: capi_exact <fixture.bin>; prints a summary, exit 0 on success.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "../../include/clrrt_adapter.hpp"

using std::vector;
typedef vector<double> state_type;

// ---- mirrors of the reference's types (field names and types as declared there) ----
struct MyReference {  // rrtplanner.h:27-33
  vector<double> x, y, v;
  signed int dir = 1;
  double aend = 0;
};
struct Node {  // rrtplanner.h:35-47
  vector<double> state;
  signed int parentID = -1;
  vector<int> children;
  MyReference ref;
  float costE = 0, costS = 0;
  bool goalReached = false;
  vector<state_type> tra;
};
struct MyRRT {  // rrtplanner.h:51-80 (fields read by the adapter)
  int sortLimit = 10;
  bool bend = false;
  vector<double> goalPose, laneShifts, Cxy;
  double Wcost[5] = {10, 5, 0, 4, 1};  // parameters.launch weights
  vector<Node> tree;
};
struct Vehicle {  // vehicle.h:5-19, values of setPrius (vehicle.h:39-60)
  double dmax = 0.52, ddmax = 0.3294, Td = 0.3, Ta = 0.3, amin = -6, amax = 2, L = 2.7, w = 2, Lrear = 1,
         Lfront = 3.2, b = 1.6132, Vch = 20, rho = 5.95, Kus = ((950.0 + 640.0) / 2.7) * (1.6132 / 22201 - 1.0868 / 22201);
};
struct Obstacle2D {  // car_msgs/Obstacle2D (the fields old_collisioncheck.cpp reads)
  struct { struct { double x, y, theta; } center; double size_x, size_y; } obb;
  struct { struct { double x, y, z; } linear; } vel;
};

static vector<double> LinearSpacedVector(double a, double b, std::size_t N) {  // functions.h:11-21 semantics
  double h = (b - a) / static_cast<double>(N - 1);
  vector<double> xs(N);
  double val = a;
  for (std::size_t k = 0; k < N; ++k, val += h) xs[k] = val;
  return xs;
}

static void addInitialNode(MyRRT& rrt, const vector<double>& state) {  // rrtplanner.cpp:21-37 semantics
  MyReference ref;
  double xend = 1, yend = 0, res = 0.1;
  int N = (int)std::floor(std::sqrt(xend * xend + yend * yend) / res);
  ref.x = LinearSpacedVector(0, xend, N);
  ref.y = LinearSpacedVector(0, yend, N);
  ref.v.assign(N, state[4]);
  Node n;
  n.state = state;
  n.parentID = -1;
  n.ref = ref;
  n.tra = {state};
  rrt.tree.push_back(n);
}

static uint64_t fnv1a(const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}

template <class T>
static T take(const char*& p) {
  T v;
  memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s fixture.bin\n", argv[0]); return 2; }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (buf.size() < 8 || memcmp(buf.data(), "CLRF", 4) != 0) { fprintf(stderr, "bad fixture\n"); return 2; }
  const char* p = buf.data() + 4;
  take<int32_t>(p);
  const int n_obs = take<int32_t>(p);
  vector<Obstacle2D> det(n_obs);
  for (auto& d : det) {
    d.obb.center.x = take<double>(p); d.obb.center.y = take<double>(p); d.obb.center.theta = take<double>(p);
    d.obb.size_x = take<double>(p); d.obb.size_y = take<double>(p);
    d.vel.linear.x = take<double>(p); d.vel.linear.y = take<double>(p); d.vel.linear.z = 0;
  }
  const int n_ref = take<int32_t>(p);
  vector<clrrt_node> want(n_ref);
  memcpy(want.data(), p, sizeof(clrrt_node) * n_ref);
  p += sizeof(clrrt_node) * n_ref;
  vector<uint64_t> row_hash(n_ref);
  for (auto& h : row_hash) h = take<uint64_t>(p);
  int64_t want_cnt[5];
  for (auto& c : want_cnt) c = take<int64_t>(p);
  const int n_st = take<int32_t>(p);
  vector<double> states(10 * (size_t)n_st), dist(n_st);
  memcpy(states.data(), p, sizeof(double) * 10 * n_st);
  p += sizeof(double) * 10 * n_st;
  memcpy(dist.data(), p, sizeof(double) * n_st);

  // MotionPlanner::planMotion's set-up (motionplanner.cpp:8-32) with the mirrors
  Vehicle veh;
  MyRRT rrt;
  rrt.goalPose = {40, 0, 0, 0};
  rrt.laneShifts = {0};
  const clrrt_adapter::Globals g{0.04, 1.4, 3.2, 3.0, 8.0, 0.05, 0.2, 5.0, 0.0, true};
  const clrrt_params prm = clrrt_adapter::params_from(veh, rrt, g, CLRRT_COLLISION_OBB);
  int fails = 0;
  try {
    clrrt_adapter::Engine eng(prm, 1 << 16, 1 << 20, 256, 256);
    eng.set_obstacles(det);
    addInitialNode(rrt, vector<double>(10, 0.0));
    eng.load_tree(rrt);
    srand(3);
    clrrt_rng rng;
    clrrt_rng_seed(&rng, 3);
    int64_t counters[4] = {0, 0, 0, 0};
    const vector<double> Cxy;
    for (int it = 0; it < 100; it++) eng.expandTree(veh, rrt, nullptr, det, Cxy, rng, counters);
    const int64_t more = eng.expandBudget(rrt, rng, 200, 0.0, CLRRT_MODE_EXACT, 256, counters);
    for (int i = 0; i < 3 * 200; i++) (void)rand();  // the budget form does not touch the process's rand()
    if (more != 200) { printf("expandBudget consumed %lld iterations\n", (long long)more); fails++; }
    // the tree
    if ((int)rrt.tree.size() != n_ref) { printf("tree size %zu, oracle %d\n", rrt.tree.size(), n_ref); fails++; }
    int bad_nodes = 0;
    for (int i = 0; i < n_ref && i < (int)rrt.tree.size(); i++) {
      const Node& n = rrt.tree[i];
      const clrrt_node& w = want[i];
      bool ok = n.parentID == w.parent && (int)n.goalReached == w.goal && (int)n.tra.size() == w.nrows &&
                memcmp(n.state.data(), w.state, sizeof(w.state)) == 0 && memcmp(&n.costE, &w.costE, 4) == 0 &&
                memcmp(&n.costS, &w.costS, 4) == 0;
      if (i > 0) {  // rows of the root come from addInitialNode, not the engine
        vector<double> flat;
        for (const auto& r : n.tra) flat.insert(flat.end(), r.begin(), r.end());
        ok = ok && fnv1a(flat.data(), flat.size() * sizeof(double)) == row_hash[i];
      }
      if (!ok) {
        if (bad_nodes < 5) printf("node %d differs (parent %d vs %d, rows %zu vs %d)\n", i, n.parentID, w.parent,
                                  n.tra.size(), w.nrows);
        bad_nodes++;
      }
    }
    fails += bad_nodes;
    for (int k = 0; k < 4; k++)
      if (counters[k] != want_cnt[k]) {
        printf("counter %d: %lld vs oracle %lld\n", k, (long long)counters[k], (long long)want_cnt[k]);
        fails++;
      }
    // the rand() streams
    for (int k = 0; k < 6; k++)
      if (rand() != clrrt_rng_next(&rng)) { printf("rand() stream diverged\n"); fails++; break; }
    // checkObsDistance hook
    int bad_d = 0;
    for (int i = 0; i < n_st; i++) {
      vector<double> x(states.begin() + 10 * i, states.begin() + 10 * i + 10);
      const double d = eng.checkObsDistance(x);
      if (memcmp(&d, &dist[i], 8) != 0) bad_d++;
    }
    if (bad_d) { printf("checkObsDistance: %d of %d differ\n", bad_d, n_st); fails++; }
    printf("capi_exact: %zu nodes (oracle %d), counters sim %lld coll %lld acc %lld iter %lld, "
           "checkObsDistance %d states, failures %d\n",
           rrt.tree.size(), n_ref, (long long)counters[0], (long long)counters[1], (long long)counters[2],
           (long long)counters[3], n_st, fails);
  } catch (const std::exception& e) {
    printf("error: %s\n", e.what());
    return 1;
  }
  return fails ? 1 : 0;
}
