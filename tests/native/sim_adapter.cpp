// The C++ Simulation adapter and the reference-signature drop-ins (include/clrrt_adapter.hpp), linked
// against libclrrt with no Python:
//   * dropin::Simulation(RRT, state, ref, veh, GoalBiased, true, Vstart) (simulation.h:18-19) on the cases of
//     an input file, with references built as getReference / getGoalReference build them
//     (reference.cpp:9-70, mirrored below); writes every stateArray, the costs, the flags and ref.v for the
//     Python side to compare with the CPU oracle (tests/test_native_sim_adapter.py);
//   * dropin::expandTree (rrtplanner.h:87) on a second tree whose size equals the synced one but whose root
//     differs: the engine must reload it (the new nodes grow from the new root);
//   * a reference that is no getReference line is refused;
//   * with <tree.in> <tree.out>: Engine::set_full_reference(true) on trees grown from a root built as
//     addInitialNode builds it (rrtplanner.cpp:22-36), by expandTree iterations (EXACT) or one BATCH
//     expandBudget call; writes every node's parent and full ref.x / ref.y / ref.v for the Python side to
//     compare with the oracle's Node::ref.
// Usage: sim_adapter <in.bin> <out.bin> [<tree.in> <tree.out>]; prints a summary, exit 0 on success.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "../../include/clrrt_adapter.hpp"

using std::vector;
typedef vector<double> state_type;

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
struct Vehicle {  // vehicle.h:5-19, values of setPrius (vehicle.h:39-60)
  double dmax = 0.52, ddmax = 0.3294, Td = 0.3, Ta = 0.3, amin = -6, amax = 2, L = 2.7, w = 2, Lrear = 1,
         Lfront = 3.2, b = 1.6132, Vch = 20, rho = 5.95, Kus = ((950.0 + 640.0) / 2.7) * (1.6132 / 22201 - 1.0868 / 22201);
};
struct Obstacle2D {
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
static MyReference getReference(double sx, double sy, double bx, double by, double ref_res) {  // reference.cpp:9-22
  MyReference ref;
  double L = std::sqrt(std::pow(sx - bx, 2) + std::pow(sy - by, 2));
  int N = (int)std::round(L / ref_res) + 1;
  ref.x = LinearSpacedVector(bx, sx, N);
  ref.y = LinearSpacedVector(by, sy, N);
  ref.dir = 1;
  return ref;
}
static MyReference getGoalReference(double bx, double by, const vector<double>& g, double ref_res) {  // :25-70
  double dla_c = 3.2 - 1.4 * 3.0;
  double dla_end = std::max(3.2, dla_c + 1.4 * std::abs(g[3]));
  double Dextend = dla_end, Dalign = 1;
  MyReference ref;
  double P1x = g[0] + Dalign * std::cos(g[2]), P1y = g[1] + Dalign * std::sin(g[2]);
  double P2x = g[0] - Dalign * std::cos(g[2]), P2y = g[1] - Dalign * std::sin(g[2]);
  double Pcx, Pcy, Pfx, Pfy;
  if (std::sqrt(std::pow(P1x - bx, 2) + std::pow(P1y - by, 2)) < std::sqrt(std::pow(P2x - bx, 2) + std::pow(P2y - by, 2))) {
    Pcx = P1x; Pcy = P1y; Pfx = P1x; Pfy = P1y;
  } else {
    Pcx = P2x; Pcy = P2y; Pfx = P2x; Pfy = P2y;
  }
  Pfx += (Dextend + Dalign) * std::cos(g[2]);
  Pfy += (Dextend + Dalign) * std::sin(g[2]);
  double N1 = std::round(std::sqrt(std::pow(Pcx - bx, 2) + std::pow(Pcy - by, 2)) / ref_res) + 1;
  double N2 = std::round(std::sqrt(std::pow(Pfx - Pcx, 2) + std::pow(Pfy - Pcy, 2)) / ref_res) + 1;
  vector<double> a = LinearSpacedVector(bx, Pcx, (size_t)N1), b = LinearSpacedVector(Pcx, Pfx, (size_t)N2);
  vector<double> c = LinearSpacedVector(by, Pcy, (size_t)N1), d = LinearSpacedVector(Pcy, Pfy, (size_t)N2);
  ref.x = a; ref.x.insert(ref.x.end(), b.begin(), b.end());
  ref.y = c; ref.y.insert(ref.y.end(), d.begin(), d.end());
  ref.dir = 1;
  return ref;
}

template <class T>
static T rd(std::ifstream& f) {
  T v;
  f.read((char*)&v, sizeof(T));
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: sim_adapter <in.bin> <out.bin>\n"); return 2; }
  std::ifstream in(argv[1], std::ios::binary);
  const int coll = rd<int32_t>(in), m = rd<int32_t>(in), n = rd<int32_t>(in);
  vector<double> goal(4);
  for (auto& g : goal) g = rd<double>(in);
  vector<Obstacle2D> det(m);
  for (auto& d : det) {
    d.obb.center.x = rd<double>(in); d.obb.center.y = rd<double>(in); d.obb.center.theta = rd<double>(in);
    d.obb.size_x = rd<double>(in); d.obb.size_y = rd<double>(in); d.vel.linear.x = rd<double>(in);
    d.vel.linear.y = rd<double>(in); d.vel.linear.z = 0;
  }
  Vehicle veh;
  MyRRT rrt;
  rrt.goalPose = goal;
  clrrt_adapter::Globals g{0.04, 1.4, 3.2, 3.0, 8.0, 0.05, 0.2, 5.0, 0.0, true};
  clrrt_params p = clrrt_adapter::params_from(veh, rrt, g, coll);
  clrrt_adapter::Engine eng(p, 1 << 14, 1 << 18, 64, 512);
  eng.set_obstacles(det);
  clrrt_adapter::dropin::bind(eng);
  int failures = 0;
  std::ofstream out(argv[2], std::ios::binary);
  for (int k = 0; k < n; k++) {
    double st[10];
    for (double& v : st) v = rd<double>(in);
    const double bx = rd<double>(in), by = rd<double>(in), sx = rd<double>(in), sy = rd<double>(in);
    const double vstart = rd<double>(in);
    const int gb = rd<int32_t>(in);
    (void)rd<int32_t>(in);
    MyReference ref = gb ? getGoalReference(bx, by, goal, g.ref_res) : getReference(sx, sy, bx, by, g.ref_res);
    state_type state(st, st + 10);
    clrrt_adapter::dropin::Simulation sim(rrt, state, ref, veh, gb != 0, true, vstart);
    const int32_t hdr[4] = {sim.outcome, (int32_t)sim.stateArray.size(), (int32_t)ref.v.size(), sim.endReached + 2 * sim.goalReached};
    out.write((const char*)hdr, sizeof hdr);
    const double costs[2] = {sim.costE, sim.costS};
    out.write((const char*)costs, sizeof costs);
    out.write((const char*)ref.v.data(), sizeof(double) * ref.v.size());
    for (const auto& r : sim.stateArray) out.write((const char*)r.data(), sizeof(double) * 10);
  }
  // a reference that is no getReference line is refused
  {
    MyReference bad = getReference(20, 3, 0.9, 0, g.ref_res);
    bad.x[5] += 1e-3;
    bool threw = false;
    try {
      clrrt_adapter::dropin::Simulation s(rrt, vector<double>(10, 0.0), bad, veh, false, true, 0.0);
    } catch (const clrrt_adapter::Error&) {
      threw = true;
    }
    if (!threw) { printf("FAIL: a non-linspace reference was accepted\n"); failures++; }
  }
  // two trees of equal size with different roots: the second must not expand the first's stale copy
  {
    MyRRT a, b;
    a.goalPose = b.goalPose = goal;
    Node ra, rb;
    ra.state = {0, 0, 0, 0, 2.0, 0, 0, 0, 0, 0};
    rb.state = {1.5, -0.5, 0.1, 0, 3.0, 0, 0, 0, 0, 0};
    for (Node* r : {&ra, &rb}) {
      r->ref.x = LinearSpacedVector(0, 1, 10);
      r->ref.y = LinearSpacedVector(0, 0, 10);
      r->ref.v.assign(10, r->state[4]);
      r->tra = {r->state};
    }
    a.tree = {ra};
    b.tree = {rb};
    eng.load_tree(a);
    eng.srand(7);
    std::srand(7);
    int grown = 0;
    for (int it = 0; it < 40 && grown == 0; it++) {
      clrrt_adapter::dropin::expandTree(veh, b, (void*)nullptr, det, vector<double>{0, 0, 0});
      grown = (int)b.tree.size() - 1;
    }
    bool ok = grown > 0;
    // a child's first row is its parent's state with IDwp in column 7 (simulation.cpp:39-41)
    for (size_t i = 1; i < b.tree.size() && ok; i++)
      if (b.tree[i].parentID == 0)
        for (int c = 0; c < 10; c++)
          if (c != 7 && b.tree[i].tra.front()[c] != rb.state[c]) ok = false;
    if (!ok) { printf("FAIL: expandTree grew a stale tree (grown %d)\n", grown); failures++; }
    if (rand() != clrrt_rng_next(&eng.rng())) { printf("FAIL: rand() streams diverged\n"); failures++; }
  }
  if (argc >= 5) {  // full references of grown trees
    std::ifstream tin(argv[3], std::ios::binary);
    std::ofstream tout(argv[4], std::ios::binary);
    const int ntrees = rd<int32_t>(tin);
    for (int q = 0; q < ntrees; q++) {
      const int seed = rd<int32_t>(tin), iters = rd<int32_t>(tin), batch = rd<int32_t>(tin);
      (void)rd<int32_t>(tin);
      Node root;
      root.state.resize(10);
      for (double& v : root.state) v = rd<double>(tin);
      const int N = (int)std::floor(std::sqrt(std::pow(1.0, 2) + std::pow(0.0, 2)) / 0.1);  // addInitialNode
      root.ref.x = LinearSpacedVector(0, 1, N);
      root.ref.y = LinearSpacedVector(0, 0, N);
      root.ref.v.assign(N, root.state[4]);
      root.ref.dir = 1;
      root.parentID = -1;
      root.tra = {root.state};
      MyRRT t;
      t.goalPose = goal;
      t.tree = {root};
      eng.invalidate();
      eng.set_full_reference(true);
      eng.srand(seed);
      std::srand(seed);
      if (batch == 0) {
        for (int it = 0; it < iters; it++) clrrt_adapter::dropin::expandTree(veh, t, (void*)nullptr, det, vector<double>{0, 0, 0});
      } else {
        eng.expandBudget(t, eng.rng(), iters, 0.0, CLRRT_MODE_BATCH, batch, nullptr);
      }
      eng.set_full_reference(false);
      const int32_t nn = (int32_t)t.tree.size();
      tout.write((const char*)&nn, 4);
      for (const auto& nd : t.tree) {
        const int32_t hdr[2] = {nd.parentID, (int32_t)nd.ref.x.size()};
        tout.write((const char*)hdr, sizeof hdr);
        if (nd.ref.y.size() != nd.ref.x.size() || nd.ref.v.size() != nd.ref.x.size()) {
          printf("FAIL: node reference arrays of unequal length\n");
          failures++;
        }
        tout.write((const char*)nd.ref.x.data(), 8 * nd.ref.x.size());
        tout.write((const char*)nd.ref.y.data(), 8 * nd.ref.x.size());
        tout.write((const char*)nd.ref.v.data(), 8 * nd.ref.x.size());
      }
      printf("full references: tree %d (%s), %d nodes\n", q, batch ? "BATCH" : "EXACT", nn);
    }
  }
  printf("sim_adapter: %d simulations, counters sim_count %lld fail_collision %lld; failures %d\n", n,
         (long long)eng.counters()[0], (long long)eng.counters()[1], failures);
  return failures ? 1 : 0;
}
