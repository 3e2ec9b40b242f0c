// The reference's unchanged Timer loop through the drop-in expandTree (verdict r04 item 6):
//   Timer timer(200); for (iter; timer.Get(); iter++) expandTree(veh, RRT, pubPtr, det, req.Cxy);
// (motionplanner.cpp:39-43, Timer rrtplanner.h:11-25: clock() CPU time) with clrrt_adapter::dropin::expandTree
// bound to one Engine, the 200-obstacle scene (SURVEY.md §8(d) generator, passed in by the test) and srand(seed).
// The adapter serves the calls from its speculation cache (Engine::set_speculation).  Writes the tree (per node:
// parent, goal, row count, state bits, float cost bits, FNV-1a of the trajectory rows) to <out> and prints the
// iteration count, wall time and nodes/s; tests/test_native_timer_loop.py grows the oracle's tree with the same
// number of iterations and compares.
// Usage: timer_loop <obstacles.bin> <seed> <budget_ms> <out.bin> [width0 width_max | mismatch]
// "mismatch": the caller seeds srand(seed) but the engine with seed + 1 (the drop-in's rand() check must throw
// before the tree changes).
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
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
  double Wcost[5] = {10, 5, 0, 4, 1};
  vector<Node> tree;
};
struct Vehicle {  // vehicle.h:5-19, setPrius values (vehicle.h:39-60)
  double dmax = 0.52, ddmax = 0.3294, Td = 0.3, Ta = 0.3, amin = -6, amax = 2, L = 2.7, w = 2, Lrear = 1,
         Lfront = 3.2, b = 1.6132, Vch = 20, rho = 5.95, Kus = ((950.0 + 640.0) / 2.7) * (1.6132 / 22201 - 1.0868 / 22201);
};
struct Obstacle2D {  // car_msgs/Obstacle2D (the fields old_collisioncheck.cpp reads)
  struct { struct { double x, y, theta; } center; double size_x, size_y; } obb;
  struct { struct { double x, y, z; } linear; } vel;
};
struct Timer {  // rrtplanner.h:11-25 (clock(): CPU time)
  clock_t tstart, tnow;
  double diff, timeLimit;
  Timer(double _timeLimit) : tstart(clock()), timeLimit(_timeLimit) {}
  bool Get() {
    tnow = clock();
    diff = (double)(tnow - tstart) / (CLOCKS_PER_SEC / 1000);
    return 0 + (diff < timeLimit);
  }
};
namespace ros { struct Publisher {}; }

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

int main(int argc, char** argv) {
  if (argc < 5) { fprintf(stderr, "usage: %s obstacles.bin seed budget_ms out.bin [width0 width_max]\n", argv[0]); return 2; }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const int n_obs = (int)(buf.size() / (7 * sizeof(double)));
  vector<Obstacle2D> det(n_obs);
  const double* o = (const double*)buf.data();
  for (int i = 0; i < n_obs; i++, o += 7) {
    det[i].obb.center.x = o[0]; det[i].obb.center.y = o[1]; det[i].obb.center.theta = o[2];
    det[i].obb.size_x = o[3]; det[i].obb.size_y = o[4];
    det[i].vel.linear.x = o[5]; det[i].vel.linear.y = o[6]; det[i].vel.linear.z = 0;
  }
  const unsigned seed = (unsigned)atoi(argv[2]);
  const double budget = atof(argv[3]);
  Vehicle veh;
  MyRRT RRT;
  RRT.goalPose = {40, 0, 0, 0};
  RRT.laneShifts = {0};
  const clrrt_adapter::Globals g{0.04, 1.4, 3.2, 3.0, 8.0, 0.05, 0.2, 5.0, 0.0, true};
  try {
    clrrt_adapter::Engine eng(clrrt_adapter::params_from(veh, RRT, g, CLRRT_COLLISION_OBB), 1 << 18, 1 << 24, 256, 256);
    const bool mismatch = argc >= 6 && strcmp(argv[5], "mismatch") == 0;
    if (argc >= 7) eng.set_speculation(atoll(argv[5]), atoll(argv[6]));
    if (mismatch) {
      RRT.tree.clear();
      addInitialNode(RRT, vector<double>(10, 0.0));
      srand(seed);
      eng.srand(seed + 1);  // a caller that forgot Engine::srand(seed)
      clrrt_adapter::dropin::bind(eng);
      try {
        clrrt_adapter::dropin::expandTree(veh, RRT, (ros::Publisher*)nullptr, det, vector<double>());
      } catch (const clrrt_adapter::Error& e) {
        printf("rand mismatch detected (tree size %zu): %s\n", RRT.tree.size(), e.what());
        return RRT.tree.size() == 1 ? 0 : 4;
      }
      printf("rand mismatch NOT detected\n");
      return 3;
    }
    int sim_count = 0, fail_collision = 0, fail_acclimit = 0, fail_iterlimit = 0;  // rrt_node.cpp:21-24
    eng.bind_counters(&sim_count, &fail_collision, &fail_acclimit, &fail_iterlimit);
    clrrt_adapter::dropin::bind(eng);
    ros::Publisher* pubPtr = nullptr;
    const vector<double> Cxy;
    // warm-up query (module load, first allocations), then the timed one
    for (int q = 0; q < 2; q++) {
      RRT.tree.clear();
      addInitialNode(RRT, vector<double>(10, 0.0));
      sim_count = fail_collision = fail_acclimit = fail_iterlimit = 0;
      srand(seed);
      eng.srand(seed);
      const auto w0 = std::chrono::steady_clock::now();
      // motionplanner.cpp:39-43, unchanged
      Timer timer(q == 0 ? 20 : budget); int iter = 0;
      for (iter; timer.Get(); iter++) {
        using clrrt_adapter::dropin::expandTree;
        expandTree(veh, RRT, pubPtr, det, Cxy);
      };
      const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
      if (q == 0) continue;
      FILE* out = fopen(argv[4], "wb");
      const int32_t n = (int32_t)RRT.tree.size(), it = iter;
      fwrite(&it, 4, 1, out);
      fwrite(&n, 4, 1, out);
      const int32_t cnt[4] = {sim_count, fail_collision, fail_acclimit, fail_iterlimit};
      fwrite(cnt, 4, 4, out);
      for (const Node& nd : RRT.tree) {
        const int32_t hdr[3] = {nd.parentID, nd.goalReached ? 1 : 0, (int32_t)nd.tra.size()};
        fwrite(hdr, 4, 3, out);
        fwrite(nd.state.data(), 8, 10, out);
        fwrite(&nd.costE, 4, 1, out);
        fwrite(&nd.costS, 4, 1, out);
        vector<double> flat;
        for (const auto& r : nd.tra) flat.insert(flat.end(), r.begin(), r.end());
        const uint64_t h = fnv1a(flat.data(), flat.size() * sizeof(double));
        fwrite(&h, 8, 1, out);
      }
      fclose(out);
      printf("timer_loop: Timer(%.0f) CPU ms, %d iterations, %d nodes in %.1f ms wall: %.0f nodes/s "
             "(served %lld of %lld speculated iterations); counters sim %d coll %d acc %d iter %d\n",
             budget, iter, n, wall, (n - 1) / (wall * 1e-3), (long long)eng.served_iterations(),
             (long long)eng.speculated_iterations(), sim_count, fail_collision, fail_acclimit, fail_iterlimit);
    }
  } catch (const std::exception& e) {
    printf("error: %s\n", e.what());
    return 1;
  }
  return 0;
}
