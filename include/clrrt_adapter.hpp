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
#include <algorithm>
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

/* ---------------------------------------------------------------------------------------------
 * MotionPlanner::planMotion (motionplanner.cpp:8-77) without ROS.  The reference's callback reads
 * its state (updateState :89-94), detections (updateObstacles :81-86) and request
 * (car_msgs::MotionRequest) from topics/services and publishes the MPC message and rviz markers;
 * here they are plain arguments and return values, and the whole query runs on the device:
 *
 *   transformStateToLocal(worldState)            transformations.cpp:143-147 (x, y, heading -> 0)
 *   updateReferenceResolution(carPose[4]), vmax  :16-17 (clrrt_params.ref_res / vmax)
 *   transformNodesWorldToCar(bestNodes, world)   :22  clrrt_path_transform(WORLD_TO_CAR)
 *   bestNodes.clear() unless commit_path         :28-30
 *   initializeTree(RRT, veh, bestNodes, carPose) :32  clrrt_tree_init_from_path
 *   Timer(200) loop of expandTree                :39-43 clrrt_expand (budget_ms, or n_iters for tests)
 *   bestNodes = extractBestPath(RRT.tree)        :51  clrrt_extract_best_path + clrrt_path_commit
 *   transformNodesCarToworld(bestNodes, world)   :54  clrrt_path_transform(CAR_TO_WORLD)
 *   generateMPCmessage + filterMPCmessage        :66-70 clrrt_path_mpc_message(filtered = 1)
 *   publish when msg.x.size() >= 3               :71-74 (MPCTrajectory::published)
 *
 * draw_tree (rrtplanner.cpp:322-341, rrt_node.cpp draw flag): the reference builds one rviz marker
 * per node (trajectory + goal flag) inside extractBestPath when the flag is set.  The engine keeps the
 * tree on the device, so the markers' data (every node's rows) is downloaded only when draw_tree is
 * on and a marker sink is passed; with the flag off nothing leaves the device (the default, and what
 * the benchmark runs). */
struct MotionRequest {          /* car_msgs::MotionRequest fields planMotion reads */
  double goal[4] = {0, 0, 0, 0};  /* x, y, heading, velocity (the planner's car frame, used as given) */
  double vmax = 5.0;
  std::vector<double> laneShifts, Cxy;
  bool bend = false;
};

struct MPCTrajectory {          /* car_msgs::Trajectory after filterMPCmessage (no delta: not copied) */
  std::vector<double> x, y, theta, v, a, a_cmd, d_cmd;
  bool published = false;       /* msg.x.size() >= 3 (motionplanner.cpp:71) */
};

struct TreeMarker {             /* createStateMsg(nodeid, tree[nodeid].tra, goalReached) input */
  int32_t id;
  bool goal;
  std::vector<double> rows;     /* nrows x 10 */
};

struct PlanReport {
  int32_t reinit_outcome = -1;  /* CLRRT_REINIT_* of initializeTree */
  int64_t iterations = 0;       /* expandTree iterations of the Timer loop */
  int64_t tree_size = 0;
  std::vector<int32_t> path;    /* bestNodes as tree ids, root -> goal */
  float best_cost = 0;
  int64_t counters[4] = {0, 0, 0, 0};  /* sim_count, fail_collision, fail_acclimit, fail_iterlimit (:9, :45) */
};

class MotionPlanner {
 public:
  struct Config {
    clrrt_params base;          /* vehicle, gains, weights, collision mode (goal/vmax/ref_res set per query) */
    clrrt_capacity cap;
    bool commit_path = true;    /* motionplanner/commit_path */
    int32_t mode = CLRRT_MODE_BATCH;
    int32_t batch = 4096;
    double budget_ms = 200;     /* Timer(200) */
    int64_t n_iters = 0;        /* > 0: a fixed iteration count instead of the budget (reproducible runs) */
    bool draw_tree = false;
  };

  MotionPlanner(const Config& c, uint32_t seed, int device = 0) : cfg_(c) {
    check(nullptr, clrrt_create(&cfg_.base, &cfg_.cap, device, &ctx_), "clrrt_create");
    clrrt_rng_seed(&rng_, seed);
  }
  ~MotionPlanner() { clrrt_destroy(ctx_); }
  MotionPlanner(const MotionPlanner&) = delete;
  MotionPlanner& operator=(const MotionPlanner&) = delete;

  clrrt_ctx* ctx() { return ctx_; }
  clrrt_rng& rng() { return rng_; }

  /* updateState (motionplanner.cpp:89-94): state = [x, y, theta, delta, v, a] in the world frame */
  void updateState(const std::vector<double>& s) {
    if (s.size() != 6) throw Error("updateState: the state has 6 entries (motionplanner.cpp:93)");
    state_ = s;
  }
  /* updateObstacles (motionplanner.cpp:81-86): the detections as the obstacle service returns them */
  void updateObstacles(const std::vector<clrrt_obstacle>& det) { det_ = det; }
  template <class ObsVec>
  void updateObstaclesFrom(const ObsVec& det) {
    det_.clear();
    for (const auto& d : det) det_.push_back(obstacle_to_c(d));
  }

  /* One query.  Returns false when no path was found ("No solution found", :56-58): the committed path
   * is then empty and the next query restarts from the car state. */
  bool planMotion(const MotionRequest& req, MPCTrajectory* msg = nullptr, PlanReport* rep = nullptr,
                  std::vector<TreeMarker>* markers = nullptr) {
    if (state_.size() != 6) throw Error("planMotion before updateState");
    check(ctx_, clrrt_reset_counters(ctx_), "clrrt_reset_counters");  // :9
    const double world[3] = {state_[0], state_[1], state_[2]};
    const double car[6] = {0.0, 0.0, 0.0, state_[3], state_[4], state_[5]};  // transformStateToLocal
    clrrt_params p = cfg_.base;
    p.ref_res = std::max(std::abs(car[4]) * p.ref_int, p.ref_mindist);  // updateReferenceResolution (:16)
    p.vmax = req.vmax;                                                  // :17
    for (int i = 0; i < 4; i++) p.goal[i] = req.goal[i];                // MyRRT RRT(req.goal, ...) (:23)
    p.bend = req.bend ? 1 : 0;
    p.lane_shift0 = req.laneShifts.empty() ? 0.0 : req.laneShifts[0];
    for (int i = 0; i < 3; i++) p.Cxy[i] = i < (int)req.Cxy.size() ? req.Cxy[i] : 0.0;
    check(ctx_, clrrt_set_params(ctx_, &p), "clrrt_set_params");
    check(ctx_, clrrt_set_obstacles(ctx_, det_.data(), (int32_t)det_.size()), "clrrt_set_obstacles");  // RRT.det
    check(ctx_, clrrt_path_transform(ctx_, CLRRT_WORLD_TO_CAR, world), "clrrt_path_transform");          // :22
    if (!cfg_.commit_path) check(ctx_, clrrt_path_commit(ctx_, nullptr, 0, nullptr), "clrrt_path_commit");  // :28-30
    int32_t oc = -1;
    check(ctx_, clrrt_tree_init_from_path(ctx_, car, &oc), "clrrt_tree_init_from_path");                   // :32
    clrrt_stats st;
    check(ctx_, clrrt_expand(ctx_, &rng_, cfg_.n_iters, cfg_.n_iters > 0 ? 0.0 : cfg_.budget_ms, cfg_.mode,
                             cfg_.batch, &st), "clrrt_expand");                                            // :39-43
    int64_t n_nodes = 0, n_rows = 0;
    check(ctx_, clrrt_tree_size(ctx_, &n_nodes, &n_rows), "clrrt_tree_size");
    if (cfg_.draw_tree && markers) draw_tree(n_nodes, *markers);  // extractBestPath's MarkerArray (:322-341)
    // bestNodes = extractBestPath(RRT.tree) (:51)
    int32_t n_path = 0;
    float best = 0;
    std::vector<int32_t> ids(256);
    check(ctx_, clrrt_extract_best_path(ctx_, ids.data(), (int32_t)ids.size(), &n_path, &best, nullptr),
          "clrrt_extract_best_path");
    if (n_path > (int32_t)ids.size()) {
      ids.resize(n_path);
      check(ctx_, clrrt_extract_best_path(ctx_, ids.data(), n_path, &n_path, &best, nullptr), "clrrt_extract_best_path");
    }
    ids.resize(n_path);
    int32_t n_remote = 0;
    check(ctx_, clrrt_path_commit(ctx_, ids.data(), n_path, &n_remote), "clrrt_path_commit");
    check(ctx_, clrrt_path_transform(ctx_, CLRRT_CAR_TO_WORLD, world), "clrrt_path_transform");  // :54
    if (rep) {
      rep->reinit_outcome = oc;
      rep->iterations = st.iterations;
      rep->tree_size = n_nodes;
      rep->path = ids;
      rep->best_cost = best;
      clrrt_counters c;
      check(ctx_, clrrt_get_counters(ctx_, &c), "clrrt_get_counters");
      rep->counters[0] = c.sim_count; rep->counters[1] = c.fail_collision;
      rep->counters[2] = c.fail_acclimit; rep->counters[3] = c.fail_iterlimit;
    }
    if (n_path == 0) return false;  // :56-58
    if (msg) {
      int32_t np = 0;
      check(ctx_, clrrt_path_mpc_message(ctx_, 1, nullptr, 0, &np), "clrrt_path_mpc_message");
      std::vector<double> pts(8 * (size_t)np);
      check(ctx_, clrrt_path_mpc_message(ctx_, 1, pts.data(), np, &np), "clrrt_path_mpc_message");
      *msg = MPCTrajectory{};
      for (int32_t i = 0; i < np; i++) {
        const double* q = &pts[8 * (size_t)i];  // x, y, theta, delta (NaN), v, a, a_cmd, d_cmd
        msg->x.push_back(q[0]); msg->y.push_back(q[1]); msg->theta.push_back(q[2]);
        msg->v.push_back(q[4]); msg->a.push_back(q[5]); msg->a_cmd.push_back(q[6]); msg->d_cmd.push_back(q[7]);
      }
      msg->published = msg->x.size() >= 3;  // :71
    }
    return true;
  }

  /* resetPlanner (motionplanner.cpp:98-100) clears MotionPlanner::motionplan, a ROS-side store the
   * engine does not hold; the committed path (bestNodes) is cleared by clearPath(). */
  void clearPath() { check(ctx_, clrrt_path_commit(ctx_, nullptr, 0, nullptr), "clrrt_path_commit"); }

 private:
  void draw_tree(int64_t n_nodes, std::vector<TreeMarker>& out) {
    std::vector<clrrt_node> h((size_t)n_nodes);
    if (n_nodes) check(ctx_, clrrt_tree_download(ctx_, 0, n_nodes, h.data()), "clrrt_tree_download");
    out.clear();
    out.reserve(h.size());
    for (int64_t i = 0; i < n_nodes; i++) {
      TreeMarker m;
      m.id = (int32_t)i;
      m.goal = h[i].goal != 0;
      m.rows.resize(10 * (size_t)h[i].nrows);
      if (h[i].nrows) check(ctx_, clrrt_tree_rows(ctx_, h[i].row_offset, h[i].nrows, m.rows.data()), "clrrt_tree_rows");
      out.push_back(std::move(m));
    }
  }

  Config cfg_;
  clrrt_ctx* ctx_ = nullptr;
  clrrt_rng rng_;
  std::vector<double> state_;
  std::vector<clrrt_obstacle> det_;
};

}  // namespace clrrt_adapter
