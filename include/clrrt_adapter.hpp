/* clrrt_adapter.hpp — header-only C++ drop-in layer over the C-ABI (include/clrrt.h) for the
 * reference's own types (vdBerg93/cl-rrt, rrt/include/rrt/rrtplanner.h:27-80).
 *
 * The reference's hot path is C++ free functions in one unity translation unit
 * (rrt/src/include.cpp:37-43).  The templates below are instantiated with the reference's own
 * MyReference / Node / MyRRT / Vehicle / car_msgs::Obstacle2D types inside that translation unit (see
 * INTEGRATION.md), so the planner keeps its data layout while expansion runs on the GPU:
 *
 *   node_to_c / node_from_c   Node (rrtplanner.h:35-47)  <-> clrrt_node header + trajectory rows
 *   obstacle_to_c             car_msgs::Obstacle2D (old_collisioncheck.cpp:10-16 field use)
 *   Engine::expandTree        void expandTree(Vehicle&, MyRRT&, ros::Publisher*, const vector<Obstacle2D>&,
 *                             const vector<double>&)  (rrtplanner.h:87, rrtplanner.cpp:123-174)
 *   Engine::expandBudget      the Timer(200) loop of MotionPlanner::planMotion (motionplanner.cpp:39-43)
 *   Engine::checkObsDistance  double checkObsDistance(const vector<double>&)  (collision.h:41)
 *
 * A node coming back from the device carries its reference in endpoint form: ref.x = {front, back},
 * ref.y = {front, back}, ref.v = {v.back()} — every field expandTree, feasibleNode, feasibleGoalBias,
 * getReference and Simulation read (rrtplanner.cpp:152,166,273-277,305).  Trajectories (Node::tra) are
 * complete.  The engine consumes the glibc rand() stream through its own restatement (clrrt_rng), so
 * `rng` must be seeded as the reference seeds rand(); Engine::expandTree advances the process's rand()
 * by the same three draws per iteration, keeping both streams equal.
 */
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "clrrt.h"

namespace clrrt_adapter {

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

inline void check(clrrt_ctx* ctx, int rc, const char* what) {
  if (rc != CLRRT_OK) {
    const char* msg = ctx ? clrrt_last_error(ctx) : "";
    throw Error(std::string(what) + " -> " + std::to_string(rc) + ": " + (msg ? msg : ""));
  }
}

/* Node -> header.  ang_par = feasibleNode's angPar (rrtplanner.cpp:273). */
template <class NodeT>
clrrt_node node_to_c(const NodeT& n) {
  clrrt_node h{};
  for (int i = 0; i < 10; i++) h.state[i] = i < (int)n.state.size() ? n.state[i] : 0.0;
  h.ref_front[0] = n.ref.x.front();
  h.ref_front[1] = n.ref.y.front();
  h.ref_back[0] = n.ref.x.back();
  h.ref_back[1] = n.ref.y.back();
  h.ref_vback = n.ref.v.back();
  h.ang_par = std::atan2(n.ref.y.back() - n.ref.y.front(), n.ref.x.back() - n.ref.x.front());
  h.parent = n.parentID;
  h.costE = n.costE;
  h.costS = n.costS;
  h.goal = n.goalReached ? 1 : 0;
  h.nrows = (int32_t)n.tra.size();
  h.owner = 0;
  h.row_offset = 0;
  return h;
}

/* Header + its rows (nrows x 10 doubles) -> Node (reference in endpoint form, see above). */
template <class NodeT>
NodeT node_from_c(const clrrt_node& h, const double* rows) {
  NodeT n;
  n.state.assign(h.state, h.state + 10);
  n.parentID = h.parent;
  n.ref.x = {h.ref_front[0], h.ref_back[0]};
  n.ref.y = {h.ref_front[1], h.ref_back[1]};
  n.ref.v = {h.ref_vback};
  n.ref.dir = 1;
  n.costE = h.costE;
  n.costS = h.costS;
  n.goalReached = h.goal != 0;
  n.tra.resize(h.nrows);
  for (int r = 0; r < h.nrows; r++) n.tra[r].assign(rows + 10 * (size_t)r, rows + 10 * (size_t)r + 10);
  return n;
}

/* car_msgs::Obstacle2D: bounding box centre/size + twist (old_collisioncheck.cpp:10-16). */
template <class ObsT>
clrrt_obstacle obstacle_to_c(const ObsT& d) {
  clrrt_obstacle o;
  o.cx = d.obb.center.x;
  o.cy = d.obb.center.y;
  o.theta = d.obb.center.theta;
  o.size_x = d.obb.size_x;
  o.size_y = d.obb.size_y;
  o.vx = d.vel.linear.x;
  o.vy = d.vel.linear.y;
  return o;
}

/* The planner globals the hot path reads (rrt/src/rrt_node.cpp:15-18, parameters.launch:3-20). */
struct Globals {
  double sim_dt, ctrl_tla, ctrl_mindla, ctrl_dlavmin, ctrl_Kp, ctrl_Ki, ref_res, vmax, ay_road_max;
  bool obs_use_pred;
};

/* clrrt_params from the reference's Vehicle (vehicle.h:5-19), MyRRT (goalPose, Wcost, bend,
 * laneShifts, Cxy, sortLimit: rrtplanner.h:51-66) and globals. */
template <class VehicleT, class RRTT>
clrrt_params params_from(const VehicleT& veh, const RRTT& rrt, const Globals& g, int collision_mode) {
  clrrt_params p;
  const double goal[4] = {rrt.goalPose[0], rrt.goalPose[1], rrt.goalPose[2], rrt.goalPose[3]};
  clrrt_params_default(&p, 0.0, goal, g.vmax);
  p.veh.dmax = veh.dmax; p.veh.ddmax = veh.ddmax; p.veh.Td = veh.Td; p.veh.Ta = veh.Ta;
  p.veh.amin = veh.amin; p.veh.amax = veh.amax; p.veh.L = veh.L; p.veh.Vch = veh.Vch; p.veh.Kus = veh.Kus;
  p.sim_dt = g.sim_dt; p.ctrl_tla = g.ctrl_tla; p.ctrl_mindla = g.ctrl_mindla; p.ctrl_dlavmin = g.ctrl_dlavmin;
  p.ctrl_Kp = g.ctrl_Kp; p.ctrl_Ki = g.ctrl_Ki; p.ref_res = g.ref_res; p.vmax = g.vmax; p.ay_road_max = g.ay_road_max;
  for (int i = 0; i < 5; i++) p.Wcost[i] = rrt.Wcost[i];
  p.bend = rrt.bend ? 1 : 0;
  p.lane_shift0 = rrt.laneShifts.empty() ? 0.0 : rrt.laneShifts[0];
  for (int i = 0; i < 3; i++) p.Cxy[i] = i < (int)rrt.Cxy.size() ? rrt.Cxy[i] : 0.0;
  p.obs_use_pred = g.obs_use_pred ? 1 : 0;
  p.sort_limit = rrt.sortLimit;
  p.collision_mode = collision_mode;
  return p;
}

/* One device context mirroring one MyRRT.  Not thread-safe (neither is the reference). */
class Engine {
 public:
  Engine(const clrrt_params& p, int64_t max_nodes, int64_t max_rows, int32_t max_batch, int32_t max_obstacles,
         int device = 0) {
    clrrt_capacity cap;
    cap.max_nodes = max_nodes;
    cap.max_rows = max_rows;
    cap.max_batch = max_batch;
    cap.max_obstacles = max_obstacles;
    check(nullptr, clrrt_create(&p, &cap, device, &ctx_), "clrrt_create");
  }
  ~Engine() { clrrt_destroy(ctx_); }
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  clrrt_ctx* ctx() { return ctx_; }
  void set_params(const clrrt_params& p) { check(ctx_, clrrt_set_params(ctx_, &p), "clrrt_set_params"); }

  template <class ObsVec>
  void set_obstacles(const ObsVec& det) {
    std::vector<clrrt_obstacle> o;
    o.reserve(det.size());
    for (const auto& d : det) o.push_back(obstacle_to_c(d));
    check(ctx_, clrrt_set_obstacles(ctx_, o.data(), (int32_t)o.size()), "clrrt_set_obstacles");
  }

  /* The device tree := RRT.tree (e.g. after MyRRT::addInitialNode or initializeTree). */
  template <class RRTT>
  void load_tree(const RRTT& rrt) {
    std::vector<clrrt_node> h;
    h.reserve(rrt.tree.size());
    for (const auto& n : rrt.tree) h.push_back(node_to_c(n));
    check(ctx_, clrrt_tree_load(ctx_, h.data(), (int64_t)h.size()), "clrrt_tree_load");
    synced_ = (int64_t)rrt.tree.size();
  }

  /* expandTree: one iteration (exactly three rand() draws), appending 0-2 nodes to RRT.tree and
   * bumping the reference's counters (sim_count, fail_*: rrt_node.cpp:21-24). */
  template <class VehicleT, class RRTT, class ObsVec>
  void expandTree(VehicleT&, RRTT& rrt, void* /*ros::Publisher* (unused)*/, const ObsVec&,
                  const std::vector<double>& /*Cxy (unused)*/, clrrt_rng& rng, int64_t counters[4]) {
    run(rrt, rng, 1, 0.0, CLRRT_MODE_EXACT, 16, counters);
    for (int i = 0; i < 3; i++) (void)rand();
  }

  /* The planMotion Timer loop (motionplanner.cpp:39-43) as one call: EXACT reproduces the reference's
   * tree for the same rand() stream, BATCH is the throughput mode.  Returns the iterations consumed. */
  template <class RRTT>
  int64_t expandBudget(RRTT& rrt, clrrt_rng& rng, int64_t n_iters, double budget_ms, int32_t mode, int32_t batch,
                       int64_t counters[4]) {
    return run(rrt, rng, n_iters, budget_ms, mode, batch, counters);
  }

  /* checkObsDistance(x) (collision.h:41) under the context's collision mode. */
  double checkObsDistance(const std::vector<double>& x) {
    double st[10] = {0};
    for (int i = 0; i < 10 && i < (int)x.size(); i++) st[i] = x[i];
    double out = 0;
    check(ctx_, clrrt_obstacle_distance(ctx_, st, 1, &out), "clrrt_obstacle_distance");
    return out;
  }

 private:
  template <class RRTT>
  int64_t run(RRTT& rrt, clrrt_rng& rng, int64_t n_iters, double budget_ms, int32_t mode, int32_t batch,
              int64_t counters[4]) {
    if ((int64_t)rrt.tree.size() != synced_) load_tree(rrt);
    clrrt_counters c0, c1;
    check(ctx_, clrrt_get_counters(ctx_, &c0), "clrrt_get_counters");
    clrrt_stats st;
    check(ctx_, clrrt_expand(ctx_, &rng, n_iters, budget_ms, mode, batch, &st), "clrrt_expand");
    check(ctx_, clrrt_get_counters(ctx_, &c1), "clrrt_get_counters");
    int64_t n = 0, nr = 0;
    check(ctx_, clrrt_tree_size(ctx_, &n, &nr), "clrrt_tree_size");
    const int64_t first = synced_;
    if (n > first) {
      std::vector<clrrt_node> h((size_t)(n - first));
      check(ctx_, clrrt_tree_download(ctx_, first, n - first, h.data()), "clrrt_tree_download");
      std::vector<double> rows;
      for (const auto& hd : h) {
        rows.resize(10 * (size_t)hd.nrows);
        check(ctx_, clrrt_tree_rows(ctx_, hd.row_offset, hd.nrows, rows.data()), "clrrt_tree_rows");
        rrt.tree.push_back(node_from_c<typename std::decay<decltype(rrt.tree[0])>::type>(hd, rows.data()));
      }
    }
    synced_ = n;
    if (counters) {
      counters[0] += c1.sim_count - c0.sim_count;
      counters[1] += c1.fail_collision - c0.fail_collision;
      counters[2] += c1.fail_acclimit - c0.fail_acclimit;
      counters[3] += c1.fail_iterlimit - c0.fail_iterlimit;
    }
    return st.iterations;
  }

  clrrt_ctx* ctx_ = nullptr;
  int64_t synced_ = 0;
};

}  // namespace clrrt_adapter
