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
 *   Simulation                Simulation::Simulation(const MyRRT&, const vector<double>&, MyReference&,
 *                             const Vehicle&, const bool&, const bool&, const double&)  (simulation.h:18-19)
 *   dropin::expandTree /      the same with the reference's exact signatures, bound to one Engine
 *   dropin::Simulation        (dropin::bind), for the unity build's call sites
 *   Engine::expandBudget      the Timer(200) loop of MotionPlanner::planMotion (motionplanner.cpp:39-43)
 *   Engine::checkObsDistance  double checkObsDistance(const vector<double>&)  (collision.h:41)
 *
 * A node coming back from the device carries its reference in endpoint form: ref.x = {front, back},
 * ref.y = {front, back}, ref.v = {v.back()} — every field expandTree, feasibleNode, feasibleGoalBias,
 * getReference and Simulation read (rrtplanner.cpp:152,166,273-277,305) — unless
 * Engine::set_full_reference(true): then ref.x / ref.y / ref.v hold all N points, as the reference's own
 * Node does (regenerated from the iterations' samples and the device's Simulation).  Trajectories
 * (Node::tra) are complete.  The engine consumes the glibc rand() stream through its own restatement (clrrt_rng), so
 * the engine's rng must be seeded as the reference seeds rand() (Engine::srand); Engine::expandTree
 * advances the process's rand() by the same three draws per iteration, keeping both streams equal.
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
    p_ = p;
  }
  ~Engine() { clrrt_destroy(ctx_); }
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  clrrt_ctx* ctx() { return ctx_; }
  const clrrt_params& params() const { return p_; }
  void set_params(const clrrt_params& p) {
    drop_cache();
    check(ctx_, clrrt_set_params(ctx_, &p), "clrrt_set_params");
    p_ = p;
  }
  /* Node::ref of the nodes an expansion appends: the endpoint form (default) or all N points of ref.x /
   * ref.y / ref.v, so the Node equals the reference's field for field.  The full form is regenerated
   * after each expansion: each iteration's sample is re-drawn from the stream (sampleAroundVehicle), the
   * regular node's reference is getReference's LinearSpacedVector from the parent's ref.back() to the
   * sample (reference.cpp:9-23; a sample whose line does not end at the node's ref.back() bit for bit
   * produced no node), and ref.v -- and the goal-biased node's whole reference (getGoalReference,
   * reference.cpp:27-69) -- come from the device's Simulation of the node (clrrt_simulate), whose end
   * state must equal the node's.  Costs one rollout per appended node. */
  void set_full_reference(bool on) { full_ref_ = on; }

  template <class ObsVec>
  void set_obstacles(const ObsVec& det) {
    drop_cache();
    std::vector<clrrt_obstacle> o;
    o.reserve(det.size());
    for (const auto& d : det) o.push_back(obstacle_to_c(d));
    check(ctx_, clrrt_set_obstacles(ctx_, o.data(), (int32_t)o.size()), "clrrt_set_obstacles");
    det_ = std::move(o);
    det_set_ = true;
  }

  /* The device tree := RRT.tree (e.g. after MyRRT::addInitialNode or initializeTree). */
  template <class RRTT>
  void load_tree(const RRTT& rrt) {
    spec_ = Spec{};
    std::vector<clrrt_node> h;
    h.reserve(rrt.tree.size());
    for (const auto& n : rrt.tree) h.push_back(node_to_c(n));
    check(ctx_, clrrt_tree_load(ctx_, h.data(), (int64_t)h.size()), "clrrt_tree_load");
    synced_ = (int64_t)rrt.tree.size();
    root_ = h.empty() ? clrrt_node{} : h.front();
    last_ = h.empty() ? clrrt_node{} : h.back();
  }
  /* Forget the synced tree: the next expansion reloads RRT.tree (call after replacing RRT.tree by other
   * means than expansion; a changed root or last synced node is also detected by itself). */
  void invalidate() {
    drop_cache();
    synced_ = -1;
  }

  /* The rand() stream (srand(seed) semantics) the expansion draws from; rng() for the explicit form. */
  void srand(uint32_t seed) { clrrt_rng_seed(&rng_, seed); }
  clrrt_rng& rng() { return rng_; }
  /* The reference's failure counters (rrt_node.cpp:21-24) bumped as its expandTree bumps them, or null. */
  void bind_counters(int* sim_count, int* fail_collision, int* fail_acclimit, int* fail_iterlimit) {
    gc_[0] = sim_count; gc_[1] = fail_collision; gc_[2] = fail_acclimit; gc_[3] = fail_iterlimit;
  }
  const int64_t* counters() const { return counters_; }
  /* One rollout's share of the counters (simulation.cpp:59,85,102,142): steps, then the failure it ended in. */
  void count_rollout(int32_t outcome, int32_t steps) {
    int64_t c[4] = {steps, outcome == CLRRT_ROLL_COLLISION, outcome == CLRRT_ROLL_ACCLIMIT,
                    outcome == CLRRT_ROLL_ITERLIMIT};
    for (int i = 0; i < 4; i++) {
      counters_[i] += c[i];
      if (gc_[i]) *gc_[i] += (int)c[i];
    }
  }

  /* expandTree (rrtplanner.h:87): one iteration (exactly three rand() draws of the engine's stream and of
   * the process's), appending 0-2 nodes to RRT.tree, bumping the counters; the detections `det` are
   * (re)loaded when they differ from the last ones loaded.
   *
   * Served from a speculation cache (set_speculation; on by default): the reference's Timer loop
   * (motionplanner.cpp:39-43) calls expandTree once per iteration, and one GPU round per call would run at
   * the round's latency.  The first call of a query expands the next `width` iterations at once in EXACT mode
   * (the reference's sequential tree, bit for bit) on the device with the per-iteration log on, and each call
   * appends one iteration's nodes (0-2) from the cache and its share of the counters; the cache is re-made,
   * twice as wide up to the cap, when it runs out, and dropped (the device tree truncated back) when anything it
   * was made for changes: RRT.tree (a new query, an edited tree), the stream state, the obstacles, the
   * parameters.  Iterations speculated but never served are discarded. */
  template <class VehicleT, class RRTT, class PubT, class ObsVec>
  void expandTree(VehicleT&, RRTT& RRT, PubT* /*ptrPub (unused)*/, const ObsVec& det,
                  const std::vector<double>& /*Cxy (unused)*/) {
    // The process's rand() stream must be the engine's (srand(seed) and Engine::srand(seed) together): the three
    // values the reference's iteration would take from rand() (rrtplanner.cpp:142, 193-194) are compared with the
    // engine stream's next three before anything changes; a caller that seeded only one of them gets an Error
    // instead of a tree grown from another stream (set_rand_check(false) turns the check off).
    {
      clrrt_rng probe = rng_;
      bool same = true;
      for (int i = 0; i < 3; i++) {
        const int32_t want = clrrt_rng_next(&probe), got = (int32_t)rand();
        same = same && want == got;
      }
      if (rand_check_ && !same)
        throw Error("clrrt_adapter::expandTree: the process's rand() stream differs from the engine's (seed both: "
                    "srand(seed) and Engine::srand(seed))");
    }
    sync_obstacles(det);
    int64_t c[4] = {0, 0, 0, 0};
    one_iteration(RRT, rng_, c);
    for (int i = 0; i < 4; i++) {
      counters_[i] += c[i];
      if (gc_[i]) *gc_[i] += (int)c[i];
    }
  }
  /* expandTree's check that rand() and the engine's stream agree (on by default). */
  void set_rand_check(bool on) { rand_check_ = on; }
  /* The same with an explicit stream and counter sink (no check: the stream is the caller's). */
  template <class VehicleT, class RRTT, class ObsVec>
  void expandTree(VehicleT&, RRTT& rrt, void* /*ros::Publisher* (unused)*/, const ObsVec& det,
                  const std::vector<double>& /*Cxy (unused)*/, clrrt_rng& rng, int64_t counters[4]) {
    sync_obstacles(det);
    one_iteration(rrt, rng, counters);
    for (int i = 0; i < 3; i++) (void)rand();
  }
  /* The speculation of expandTree: the first cache of a query holds `width0` iterations, each next one twice as
   * many up to `width_max` (default 32 / 64: the loop's Timer stops while a cache is partly served, and what is
   * left of it was computed for nothing -- a 256-iteration cache wasted ~60% of a 200 ms query); width0 = 0: no
   * cache (one device round per call). */
  void set_speculation(int64_t width0, int64_t width_max) {
    drop_cache();
    spec_w0_ = std::max<int64_t>(0, width0);
    spec_wmax_ = std::max(spec_w0_, width_max);
  }
  /* Iterations served from caches, and speculated in all (statistics). */
  int64_t served_iterations() const { return spec_served_; }
  int64_t speculated_iterations() const { return spec_made_; }

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
  static bool same_node(const clrrt_node& a, const clrrt_node& b) {
    for (int i = 0; i < 10; i++)
      if (!(a.state[i] == b.state[i]) && !(a.state[i] != a.state[i] && b.state[i] != b.state[i])) return false;
    return a.parent == b.parent && a.costE == b.costE && a.costS == b.costS && a.ref_back[0] == b.ref_back[0] &&
           a.ref_back[1] == b.ref_back[1] && a.ref_front[0] == b.ref_front[0] && a.ref_front[1] == b.ref_front[1] &&
           a.nrows == b.nrows;
  }
  /* RRT.tree is the synced tree plus nodes appended since?  (same length, same root, same last node) */
  template <class RRTT>
  bool tree_synced(const RRTT& rrt) const {
    if (synced_ < 0 || (int64_t)rrt.tree.size() != synced_) return false;
    if (synced_ == 0) return true;
    return same_node(node_to_c(rrt.tree.front()), root_) && same_node(node_to_c(rrt.tree.back()), last_);
  }
  template <class ObsVec>
  void sync_obstacles(const ObsVec& det) {
    bool same = det_set_ && det_.size() == det.size();
    if (same) {
      size_t i = 0;
      for (const auto& d : det) {
        const clrrt_obstacle o = obstacle_to_c(d), &q = det_[i++];
        if (o.cx != q.cx || o.cy != q.cy || o.theta != q.theta || o.size_x != q.size_x || o.size_y != q.size_y ||
            o.vx != q.vx || o.vy != q.vy) { same = false; break; }
      }
    }
    if (!same) set_obstacles(det);
  }

  /* The speculation cache: headers and rows of `count` iterations' nodes expanded past RRT.tree's first
   * tree_size nodes from stream state `rng0`; `next` of them served. */
  struct Spec {
    bool valid = false;
    clrrt_rng next_rng{};         // the stream state before iteration `next`
    int64_t next = 0, count = 0;
    int64_t tree_size = 0;        // RRT.tree.size() expected before serving iteration `next`
    clrrt_node last{};            // and RRT.tree.back()
    int64_t dev_base = 0;         // device tree size before the cache's nodes
    std::vector<clrrt_iteration> its;
    std::vector<int64_t> off;     // first cached node of each iteration
    std::vector<clrrt_node> hdr;
    std::vector<std::vector<double>> rows;
    int64_t width = 0;            // iterations of the next cache
  };
  /* The device tree back to RRT.tree (the served prefix) and no cache. */
  void drop_cache() {
    if (spec_.valid) {
      const int64_t keep = spec_.dev_base + (spec_.next < (int64_t)spec_.off.size() ? spec_.off[spec_.next]
                                                                                     : (int64_t)spec_.hdr.size());
      if (keep >= 1 && clrrt_tree_truncate(ctx_, keep) == CLRRT_OK) {
        synced_ = keep;
        last_ = spec_.last;  // RRT.tree.back() when the last iteration was served = device node keep - 1
      } else {
        synced_ = -1;
      }
    }
    spec_ = Spec{};
  }
  static bool same_rng(const clrrt_rng& a, const clrrt_rng& b) {
    for (int i = 0; i < 34; i++)
      if (a.r[i] != b.r[i]) return false;
    return a.pos == b.pos;
  }
  template <class RRTT>
  bool cache_serves(const RRTT& rrt, const clrrt_rng& rng) const {
    return spec_.valid && spec_.next < spec_.count && (int64_t)rrt.tree.size() == spec_.tree_size &&
           !rrt.tree.empty() && same_node(node_to_c(rrt.tree.back()), spec_.last) && same_rng(rng, spec_.next_rng);
  }
  template <class RRTT>
  void one_iteration(RRTT& rrt, clrrt_rng& rng, int64_t counters[4]) {
    if (spec_w0_ <= 0 || full_ref_) {  // one device round per call
      run(rrt, rng, 1, 0.0, CLRRT_MODE_EXACT, 16, counters);
      return;
    }
    if (!cache_serves(rrt, rng)) speculate(rrt, rng);
    const int64_t i = spec_.next;
    const clrrt_iteration& it = spec_.its[(size_t)i];
    using NodeT = typename std::decay<decltype(rrt.tree[0])>::type;
    for (int64_t k = spec_.off[(size_t)i]; k < spec_.off[(size_t)i] + it.nodes; k++)
      rrt.tree.push_back(node_from_c<NodeT>(spec_.hdr[(size_t)k], spec_.rows[(size_t)k].data()));
    if (counters) {
      counters[0] += it.sim_count;
      counters[1] += it.fail_collision;
      counters[2] += it.fail_acclimit;
      counters[3] += it.fail_iterlimit;
    }
    for (int q = 0; q < 3; q++) clrrt_rng_next(&rng);
    spec_.next_rng = rng;
    spec_.next++;
    spec_.tree_size = (int64_t)rrt.tree.size();
    spec_.last = node_to_c(rrt.tree.back());
    spec_served_++;
  }
  /* A new cache for the iterations that follow RRT.tree and the stream state rng. */
  template <class RRTT>
  void speculate(RRTT& rrt, const clrrt_rng& rng) {
    // the device tree: RRT.tree is the served prefix of the old cache's (truncate), or reload it
    const bool prefix = spec_.valid && (int64_t)rrt.tree.size() == spec_.tree_size && !rrt.tree.empty() &&
                        same_node(node_to_c(rrt.tree.back()), spec_.last);
    const int64_t width = prefix && spec_.width > 0 ? spec_.width : spec_w0_;
    drop_cache();
    if (!prefix || synced_ != (int64_t)rrt.tree.size()) load_tree(rrt);
    Spec s;
    s.dev_base = (int64_t)rrt.tree.size();
    clrrt_rng work = rng;
    // from here on the device tree may hold nodes RRT.tree does not (a failed expansion's rounds, a cache whose
    // download failed): on any error the next call reloads RRT.tree instead of trusting the device tree
    struct Unsync {
      int64_t* synced;
      bool armed = true;
      ~Unsync() { if (armed) *synced = -1; }
    } unsync{&synced_};
    check(ctx_, clrrt_iteration_log(ctx_, 1), "clrrt_iteration_log");
    clrrt_stats st;
    const int rc = clrrt_expand(ctx_, &work, width, 0.0, CLRRT_MODE_EXACT, 256, &st);
    if (rc != CLRRT_OK) clrrt_iteration_log(ctx_, 0);
    check(ctx_, rc, "clrrt_expand");
    s.its.resize((size_t)st.iterations);
    int64_t total = 0;
    if (st.iterations > 0)
      check(ctx_, clrrt_iteration_records(ctx_, 0, st.iterations, s.its.data(), &total), "clrrt_iteration_records");
    check(ctx_, clrrt_iteration_log(ctx_, 0), "clrrt_iteration_log");
    int64_t n = 0, nr = 0;
    check(ctx_, clrrt_tree_size(ctx_, &n, &nr), "clrrt_tree_size");
    s.hdr.resize((size_t)(n - s.dev_base));
    if (n > s.dev_base) check(ctx_, clrrt_tree_download(ctx_, s.dev_base, n - s.dev_base, s.hdr.data()), "clrrt_tree_download");
    s.rows.resize(s.hdr.size());
    if (!s.hdr.empty()) {  // the expansion's rows are one contiguous range of the arena: one download
      int64_t r0 = INT64_MAX, r1 = 0;
      for (const auto& h : s.hdr) {
        r0 = std::min<int64_t>(r0, h.row_offset);
        r1 = std::max<int64_t>(r1, h.row_offset + h.nrows);
      }
      std::vector<double> all(10 * (size_t)(r1 - r0));
      check(ctx_, clrrt_tree_rows(ctx_, r0, r1 - r0, all.data()), "clrrt_tree_rows");
      for (size_t k = 0; k < s.hdr.size(); k++) {
        const double* src = all.data() + 10 * (size_t)(s.hdr[k].row_offset - r0);
        s.rows[k].assign(src, src + 10 * (size_t)s.hdr[k].nrows);
      }
    }
    s.off.resize(s.its.size());
    int64_t o = 0;
    for (size_t i = 0; i < s.its.size(); i++) {
      s.off[i] = o;
      o += s.its[i].nodes;
    }
    if (o != (int64_t)s.hdr.size()) throw Error("expandTree cache: the iteration log does not match the nodes appended");
    unsync.armed = false;
    s.valid = st.iterations > 0;
    s.next_rng = rng;
    s.count = st.iterations;
    s.tree_size = (int64_t)rrt.tree.size();
    s.last = node_to_c(rrt.tree.back());
    s.width = std::min(spec_wmax_, 2 * width);
    spec_ = std::move(s);
    spec_made_ += st.iterations;
    synced_ = -1;  // the device holds the cache's nodes beyond RRT.tree (drop_cache truncates them)
    if (!spec_.valid) throw Error("expandTree cache: the expansion consumed no iteration");
  }

  template <class RRTT>
  int64_t run(RRTT& rrt, clrrt_rng& rng, int64_t n_iters, double budget_ms, int32_t mode, int32_t batch,
              int64_t counters[4]) {
    drop_cache();
    if (!tree_synced(rrt)) load_tree(rrt);
    const clrrt_rng rng0 = rng;
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
      if (full_ref_) full_references(rrt, first, h, rng0, st.iterations);
    }
    synced_ = n;
    if (!rrt.tree.empty()) {
      root_ = node_to_c(rrt.tree.front());
      last_ = node_to_c(rrt.tree.back());
    }
    if (counters) {
      counters[0] += c1.sim_count - c0.sim_count;
      counters[1] += c1.fail_collision - c0.fail_collision;
      counters[2] += c1.fail_acclimit - c0.fail_acclimit;
      counters[3] += c1.fail_iterlimit - c0.fail_iterlimit;
    }
    return st.iterations;
  }

  /* The full references of the appended nodes rrt.tree[first ..] (headers h), see set_full_reference. */
  template <class RRTT>
  void full_references(RRTT& rrt, int64_t first, const std::vector<clrrt_node>& h, clrrt_rng rng0, int64_t iters) {
    std::vector<clrrt_sample> smp((size_t)std::max<int64_t>(iters, 0));
    if (iters > 0) check(ctx_, clrrt_draw_samples(&p_, &rng0, (int32_t)iters, smp.data()), "clrrt_draw_samples");
    std::vector<clrrt_sim_case> q(h.size());
    size_t j = 0;  // next sample
    for (size_t k = 0; k < h.size(); k++) {
      const clrrt_node& n = h[k];
      const auto& par = rrt.tree[(size_t)n.parent];
      clrrt_sim_case& c = q[k];
      c = clrrt_sim_case{};
      for (int i = 0; i < 10; i++) c.state[i] = i < (int)par.state.size() ? par.state[i] : 0.0;
      const double bx = par.ref.x.back(), by = par.ref.y.back();
      c.ax = bx;
      c.ay = by;
      c.vstart = par.ref.v.back();
      // a regular node: the first remaining sample whose getReference line ends at the node's ref.back()
      bool regular = false;
      for (size_t t = j; t < smp.size() && !regular; t++) {
        const double L = std::sqrt(std::pow(smp[t].x - bx, 2) + std::pow(smp[t].y - by, 2));
        const int N = (int)std::round(L / p_.ref_res) + 1;  // reference.cpp:15
        if (N < 2) continue;
        const double hx = (smp[t].x - bx) / static_cast<double>(N - 1), hy = (smp[t].y - by) / static_cast<double>(N - 1);
        double vx = bx, vy = by;
        for (int i = 1; i < N; i++) { vx += hx; vy += hy; }
        if (vx == n.ref_back[0] && vy == n.ref_back[1]) {
          regular = true;
          j = t + 1;
          c.hx = hx; c.hy = hy; c.ref_n = N; c.goal_biased = 0;
        }
      }
      if (!regular) {  // the goal-biased node of the regular node just before it (rrtplanner.cpp:163-173)
        if (k == 0 || n.parent != first + (int64_t)k - 1)
          throw Error("set_full_reference: an appended node matches no sample of the expansion");
        c.goal_biased = 1;
      }
    }
    // the cases are independent (each parent's ref.v.back() is in its header): chunks of 512
    int32_t cap = 2048;
    for (const auto& c : q) cap = std::max(cap, c.ref_n);
    const size_t chunk = 512;
    std::vector<clrrt_rollout_result> res(chunk);
    std::vector<double> ref(3 * (size_t)cap * chunk);
    for (size_t k0 = 0; k0 < q.size(); k0 += chunk) {
      const size_t m = std::min(chunk, q.size() - k0);
      check(ctx_, clrrt_simulate(ctx_, &q[k0], (int32_t)m, res.data(), nullptr, 0, ref.data(), cap), "clrrt_simulate");
      for (size_t i = 0; i < m; i++) {
        const clrrt_rollout_result& r = res[i];
        const clrrt_node& hd = h[k0 + i];
        const double* rx = &ref[3 * (size_t)cap * i];
        if (r.ref_n < 1 || r.ref_n > cap) throw Error("set_full_reference: reference longer than the buffer");
        bool same = r.nrows == hd.nrows && rx[r.ref_n - 1] == hd.ref_back[0] && rx[cap + r.ref_n - 1] == hd.ref_back[1];
        for (int t = 0; t < 10 && same; t++) same = r.final_state[t] == hd.state[t];
        if (!same) throw Error("set_full_reference: the re-simulated node differs from the expansion's");
        auto& node = rrt.tree[(size_t)first + k0 + i];
        node.ref.x.assign(rx, rx + r.ref_n);
        node.ref.y.assign(rx + cap, rx + cap + r.ref_n);
        node.ref.v.assign(rx + 2 * (size_t)cap, rx + 2 * (size_t)cap + r.ref_n);
      }
    }
  }

  clrrt_ctx* ctx_ = nullptr;
  clrrt_params p_{};
  bool full_ref_ = false;
  bool rand_check_ = true;
  int64_t synced_ = -1;  // nodes of RRT.tree the device holds (-1: unknown, reload)
  clrrt_node root_{}, last_{};
  clrrt_rng rng_{};
  int64_t counters_[4] = {0, 0, 0, 0};
  int* gc_[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<clrrt_obstacle> det_;
  bool det_set_ = false;
  Spec spec_;
  int64_t spec_w0_ = 32, spec_wmax_ = 64;
  int64_t spec_served_ = 0, spec_made_ = 0;
};

/* The step h of a reference coordinate built by LinearSpacedVector (functions.h:11-21: val += h from v[0]):
 * an h whose accumulation reproduces every value of v bit for bit (the device regenerates the reference
 * by the same accumulation).  h = v[1] - v[0] is h rounded to the grid of v[0]; the true step lies within
 * half an ulp of v[0] of it. */
inline bool linspace_step(const std::vector<double>& v, double& h) {
  const size_t N = v.size();
  if (N < 2) { h = 0.0; return true; }
  auto reproduces = [&](double c) {
    double val = v[0];
    for (size_t i = 0; i < N; i++, val += c)
      if (!(val == v[i])) return false;
    return true;
  };
  const double h0 = v[1] - v[0];
  if (reproduces(h0)) { h = h0; return true; }
  double up = h0, dn = h0;
  const double span = std::fabs(std::nextafter(v[0], INFINITY) - v[0]) + std::fabs(h0) * 1e-15;
  for (int k = 0; k < 1 << 14 && std::fabs(up - h0) <= span; k++) {
    up = std::nextafter(up, INFINITY);
    dn = std::nextafter(dn, -INFINITY);
    if (reproduces(up)) { h = up; return true; }
    if (reproduces(dn)) { h = dn; return true; }
  }
  return false;
}

/* Simulation (simulation.h:7-21): the constructor runs the closed-loop prediction on the device
 * (clrrt_simulate, the rollout kernels' own code) and fills the members the reference fills: stateArray,
 * costS, costE, goalReached, endReached, and ref.v (generateVelocityProfile, simulation.cpp:42-45).  The
 * reference `ref` must be what getReference (a LinearSpacedVector line) or, with GoalBiased,
 * getGoalReference produced -- the only references expandTree simulates; anything else throws.  The
 * engine's params must be those of RRT (Engine::set_params(params_from(...))); genProfile = false (never
 * used by the reference) throws.  The failure counters move as the reference's propagate moves them. */
class Simulation {
 public:
  std::vector<std::vector<double>> stateArray;
  std::vector<double> curvature;
  std::vector<int> closestPoints;
  std::vector<double> acmd, dcmd;
  double costS = 0, costE = 0;
  bool goalReached = false, endReached = false;
  int32_t outcome = -1;  /* CLRRT_ROLL_* (the counter the reference bumps) */

  template <class RRTT, class RefT, class VehicleT>
  Simulation(Engine& eng, const RRTT& /*RRT (params)*/, const std::vector<double>& state, RefT& ref,
             const VehicleT& /*veh (params)*/, const bool& GoalBiased, const bool& genProfile, const double& Vstart) {
    if (!genProfile) throw Error("Simulation: genProfile = false is not supported (expandTree always passes true)");
    if (ref.x.empty() || ref.x.size() != ref.y.size()) throw Error("Simulation: malformed reference");
    clrrt_sim_case q{};
    for (int i = 0; i < 10; i++) q.state[i] = i < (int)state.size() ? state[i] : 0.0;
    q.ax = ref.x.front();
    q.ay = ref.y.front();
    q.vstart = Vstart;
    q.goal_biased = GoalBiased ? 1 : 0;
    q.ref_n = (int32_t)ref.x.size();
    if (!GoalBiased && !(linspace_step(ref.x, q.hx) && linspace_step(ref.y, q.hy)))
      throw Error("Simulation: the reference is not a getReference line");
    const int32_t cap = (int32_t)std::max<size_t>(ref.x.size(), 1);
    clrrt_rollout_result res;
    /* propagate's loop runs while i < 20/sim_dt (simulation.cpp:58): that many steps + the initial row */
    int32_t n_steps = 0;
    while (n_steps < 20 / eng.params().sim_dt) n_steps++;
    const int32_t rows_cap = n_steps + 1;
    std::vector<double> rows(10 * (size_t)rows_cap), refo(3 * (size_t)cap);
    check(eng.ctx(), clrrt_simulate(eng.ctx(), &q, 1, &res, rows.data(), rows_cap, refo.data(), cap),
          "clrrt_simulate");
    if (res.ref_n != (int32_t)ref.x.size()) throw Error("Simulation: the reference is not the one getGoalReference builds");
    for (int32_t i = 0; i < res.ref_n; i++)
      if (!(refo[i] == ref.x[i]) || !(refo[cap + i] == ref.y[i]))
        throw Error("Simulation: the reference is not the one getReference / getGoalReference builds");
    ref.v.assign(refo.begin() + 2 * (size_t)cap, refo.begin() + 2 * (size_t)cap + res.ref_n);
    stateArray.resize(res.nrows);
    for (int32_t r = 0; r < res.nrows; r++) stateArray[r].assign(&rows[10 * (size_t)r], &rows[10 * (size_t)r] + 10);
    costE = res.costE;
    costS = res.costS;
    outcome = res.outcome;
    eng.count_rollout(res.outcome, res.nrows - 1);
    endReached = res.outcome == CLRRT_ROLL_END;
    goalReached = res.outcome == CLRRT_ROLL_GOAL;
  }
  bool isvalid() { return endReached; }  /* simulation.h:22-25 */
};

/* The reference's own signatures for its call sites, bound to one Engine:
 *   clrrt_adapter::dropin::bind(engine);            once, after the engine is configured
 *   expandTree(veh, RRT, pubPtr, det, Cxy);         rrtplanner.h:87 (motionplanner.cpp:41)
 *   Simulation sim(RRT, state, ref, veh, GB, true, Vstart);   simulation.h:18-19 */
namespace dropin {
inline Engine*& bound() {
  static Engine* e = nullptr;
  return e;
}
inline void bind(Engine& e) { bound() = &e; }
inline Engine& engine() {
  if (!bound()) throw Error("clrrt_adapter::dropin: no Engine bound (dropin::bind)");
  return *bound();
}
template <class VehicleT, class RRTT, class PubT, class ObsVec>
void expandTree(VehicleT& veh, RRTT& RRT, PubT* ptrPub, const ObsVec& det, const std::vector<double>& Cxy) {
  engine().expandTree(veh, RRT, ptrPub, det, Cxy);
}
class Simulation : public clrrt_adapter::Simulation {
 public:
  template <class RRTT, class RefT, class VehicleT>
  Simulation(const RRTT& RRT, const std::vector<double>& state, RefT& ref, const VehicleT& veh, const bool& GoalBiased,
             const bool& genProfile, const double& Vstart)
      : clrrt_adapter::Simulation(engine(), RRT, state, ref, veh, GoalBiased, genProfile, Vstart) {}
};
}  // namespace dropin

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
