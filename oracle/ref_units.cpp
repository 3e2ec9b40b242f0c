// ref_units.cpp — TEST INFRASTRUCTURE ONLY (never linked into, loaded by or called from the product).
//
// Driver around the reference's OWN source text.  `make ref` (oracle/Makefile) copies verbatim line
// ranges out of /root/reference into oracle/_ref/*.inc (git-ignored, never committed) and compiles
// this file against them into oracle/_ref/libref_units_O3.so (CMake's Release flags -O3 -DNDEBUG:
// README.md:59-64 asks for a release build), libref_units_O2.so (the survey's probe flags) and
// libref_units_O0.so (catkin's default empty build type).  Nothing here restates the reference's
// arithmetic: file-scope text (_ref/ref_units.inc) is the reference's own functions, and every
// function below that the reference defines is its own body included as a statement range inside a
// signature of the same name.  The driver supplies only
//   * Pt, the three doubles of geometry_msgs::Point (a ROS message header the image lacks), where a
//     body declares one (Makefile: reference.cpp:37, rrtplanner.cpp:129,192,295);
//   * RRTd, the MyRRT fields the bodies read (rrtplanner.h:51-80 also holds car_msgs detections,
//     which need ROS), with addInitialNode / addNode bodies from the reference;
//   * the class declarations of Controller (controller.h:11-31) and Simulation (simulation.h:7-21)
//     with the reference's member names and types (Pt for geometry_msgs::Point), whose method bodies
//     are the reference's;
//   * checkObsDistance: the shipped stub (collisioncheck.cpp:6-8, what the unity build links) or the
//     OBB form (old_collisioncheck.cpp:24-51: its statements, with getOBBvector's field reads :14-16
//     over plain detections);
//   * extern "C" entry points that marshal inputs and outputs.
// Units (reference file:line):
//   OBB ctor / setVertices / setNorms / findMaxMin / getOBBdist   collision.h:4-35, old_collisioncheck.cpp:56-148
//   checkObsDistance                                              old_collisioncheck.cpp:24-51 / collisioncheck.cpp:6-8
//   VehicleODE / IntegrateEuler / enforceConstraints               simulation.cpp:7-34
//   transformToVehicle / interpolate                               controller.cpp:115-148
//   getReference, LinearSpacedVector                               reference.cpp:9-22, functions.h:11-21
//   generateVelocityProfile                                        reference.cpp:72-170
//   getGoalReference                                               reference.cpp:25-70
//   angleDiff / wrapToPi                                           functions.h:43-57
//   Vehicle::setPrius, updateLookahead, updateReferenceResolution  vehicle.h:39-60, controller.cpp:13-21
//   dubinsDistance, feasibleNode, feasibleGoalBias                 rrtplanner.cpp:371-406, 271-289, 292-315
//   sortNodesExplore / sortNodesOptimize                           rrtplanner.cpp:227-268
//   sampleAroundVehicle + the heuristic draw                       rrtplanner.cpp:187-201, 142
//   Controller (ctor, getControls, commands, updateWaypoint,
//     getLateralError, findClosestPoint)                           controller.cpp:23-113
//   Simulation (ctor, propagate)                                   simulation.cpp:36-143
//   expandTree, addInitialNode                                     rrtplanner.cpp:123-174, 21-37
//   initializeTree, getNodeCost, d2L, extractBestPath              rrtplanner.cpp:39-119, 318-368
//   transformNodesWorldToCar / CarToworld                          transformations.cpp:6-17, 113-120, 289-315
//
// Uninitialised field: getGoalReference declares `MyReference ref;` (reference.cpp:34) and never sets
// ref.dir, which updateWaypoint multiplies into the preview point (controller.cpp:56-57).  The returned
// object lives in the caller's storage (NRVO); in expandTree that is where the loop's `ref` (dir = 1,
// reference.cpp:18) lived, and the full-tree pins (ref_tree_expand, tests/test_ref_tree.py: the
// reference's own expandTree, no driver intervention) agree with dir = 1, as do the survey's probe
// numbers.  The unit drivers below set dir = 1 after the call (the canonical value).
//
// Determinism recipe: a zero-filling global operator new with 256 B of padding, so
// IntegrateEuler's `i<=x.size()` loop (simulation.cpp:28) reads dx[7..10] as 0.0 and its write of
// x[10] lands in padding, and ref.v[i] past the end (controller.cpp:39, simulation.cpp:66) reads 0.0
// within the padding.
#include <algorithm>
#include <array>
#include <cassert>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <iostream>
#include <limits>
#include <new>
#include <vector>

#include "_ref/ref_units.inc"

void* operator new(std::size_t n) {
  void* p = calloc(1, n + 256);
  if (!p) throw std::bad_alloc();
  return p;
}
void* operator new[](std::size_t n) { return operator new(n); }
void operator delete(void* p) noexcept { free(p); }
void operator delete[](void* p) noexcept { free(p); }
void operator delete(void* p, std::size_t) noexcept { free(p); }
void operator delete[](void* p, std::size_t) noexcept { free(p); }

// setNorms leaves normsY[3] unset (old_collisioncheck.cpp:74-75: normsX[3] is written twice).  The
// stack object's slot is indeterminate in the reference; here it is set explicitly per mode:
//   0: the proper edge normal of edge 3->0 (the oracle's and the kernels' canonical axis 3)
//   1: normsX[3] as the reference leaves it, normsY[3] = 0
//   2: normsX[3] as the reference leaves it, normsY[3] = pseudo-random value in [-1000, 1000)
//   3: normsX[3] as the reference leaves it, normsY[3] = NaN
static void set_axis3(OBB& b, int mode, uint64_t key) {
  switch (mode) {
    case 0:
      b.normsX[3] = b.verticesY[0] - b.verticesY[3];
      b.normsY[3] = -(b.verticesX[0] - b.verticesX[3]);
      break;
    case 1: b.normsY[3] = 0.0f; break;
    case 2: {
      uint64_t z = key * 0x9E3779B97F4A7C15ull;
      z ^= z >> 29;
      b.normsY[3] = (float)(std::ldexp((double)(z >> 11), -53) * 2000.0 - 1000.0);
    } break;
    default: b.normsY[3] = std::numeric_limits<float>::quiet_NaN(); break;
  }
}

// ------------------------------------------------------------------------------------ driver types
// geometry_msgs::Point: three doubles, zero-initialised by the message's default constructor.
struct Pt {
  double x = 0, y = 0, z = 0;
};

// The MyRRT fields the reference's bodies read (rrtplanner.h:51-80; the car_msgs detections are the
// driver's g_det below).  Defaults as MyRRT's constructor leaves them (rrtplanner.cpp:12-19).
struct RRTd {
  int sortLimit = 10;
  bool reverseAllowed = false;
  bool goalReached = false;
  bool bend = false;
  vector<double> goalPose = vector<double>(4, 0.0);
  signed int direction = 1;
  vector<double> laneShifts = vector<double>(2, 0.0);
  vector<double> Cxy = vector<double>(3, 0.0);
  vector<int> det;  // RRT.det: only passed through to getNodeCost's unused parameter
  vector<double> carState;
  double Wcost[5] = {0, 0, 0, 0, 0};
  vector<Node> tree;
  void addInitialNode(const vector<double>& state);
  void addNode(Node node);
};
void RRTd::addInitialNode(const vector<double>& state) {
#include "_ref/add_initial_node.inc"
}
void RRTd::addNode(Node node) {
#include "_ref/add_node.inc"
}

// ------------------------------------------------------------------------------------ collision
namespace refstub {
#include "_ref/cc_stub.inc"
}
struct Det {
  double cx, cy, th, sx, sy, vx, vy;  // car_msgs/Obstacle2D: obb.center.{x,y,theta}, obb.size_{x,y}, vel.linear.{x,y}
};
static vector<Det> g_det;
static int g_coll = 0;  // 0: the shipped stub, 1: the OBB form

// getOBBvector old_collisioncheck.cpp:6-22 over the plain detections (the field reads of :14-16)
static vector<OBB> drv_obb_vector(const double& t) {
  vector<OBB> obstacleVector;
  for (size_t i = 0; i != g_det.size(); i++) {
    const Det& d = g_det[i];
    OBB obs(Vector2D(d.cx + d.vx * t, d.cy + d.vy * t), d.sx / 2, d.sy / 2, d.th);
    obstacleVector.push_back(obs);
  }
  return obstacleVector;
}
// checkObsDistance(states, det, carState) old_collisioncheck.cpp:24-51
static double check_obs_obb(const vector<double>& states) {
#include "_ref/cc_time.inc"
  vector<OBB> obstacleVector = drv_obb_vector(t);
#include "_ref/veh_box.inc"
#include "_ref/cc_loop.inc"
}
double checkObsDistance(const vector<double>& x) { return g_coll ? check_obs_obb(x) : refstub::checkObsDistance(x); }

// ------------------------------------------------------------------------------------ rrtplanner.cpp
float dubinsDistance(Pt S, Node N, int dir) {
#include "_ref/dubins.inc"
}
bool feasibleNode(const RRTd& rrt, const Node& node, const Pt& sample) {
#include "_ref/feasible_node.inc"
}
bool feasibleGoalBias(const RRTd& rrt) {
#include "_ref/feasible_goal_bias_a.inc"
  Pt center_l, center_r;
#include "_ref/feasible_goal_bias_b.inc"
}
vector<int> sortNodesExplore(const RRTd& rrt, const Pt& sample) {
#include "_ref/sort_explore.inc"
}
vector<int> sortNodesOptimize(const RRTd& rrt, const Pt& sample) {
#include "_ref/sort_optimize.inc"
}
Pt sampleAroundVehicle(const vector<double> goalPose) {
#include "_ref/sample_a.inc"
  Pt sample;
#include "_ref/sample_b.inc"
}

// ------------------------------------------------------------------------------------ reference.cpp
MyReference getReference(Pt sample, Node node, signed int dir) {
#include "_ref/get_reference_body.inc"
}
MyReference getGoalReference(const Vehicle& veh, Node node, vector<double> goalPose) {
#include "_ref/goal_ref_a.inc"
  Pt P1, P2, Pclose, Pfar;
#include "_ref/goal_ref_b.inc"
}

// ------------------------------------------------------------------------------------ controller.cpp
int findClosestPoint(const MyReference& ref, const Pt& point, int ID) {
#include "_ref/ctrl_closest_point.inc"
}
double getLateralError(const MyReference& ref, const state_type& x, const int& IDwp, const Pt& Ppreview) {
#include "_ref/ctrl_lateral_error.inc"
}
class Controller {  // controller.h:11-31 (declarations; the definitions follow out of class, as there)
 public:
  int IDwp;
  Pt Ppreview;
  double ym;
  double E, iE;
  bool endreached;
  Controller(const MyReference& ref, const state_type& x);
  ControlCommand getControls(const MyReference& ref, const Vehicle& veh, const state_type& x);

 private:
  double getAccelerationCommand(const Vehicle& veh, const MyReference& ref, const state_type& x);
  double getSteerCommand(const MyReference& ref, const state_type& x, const Vehicle& veh);
  void updateWaypoint(const MyReference& ref, const state_type& x);
};
Controller::Controller(const MyReference& ref, const state_type& x) {
#include "_ref/ctrl_ctor.inc"
}
ControlCommand Controller::getControls(const MyReference& ref, const Vehicle& veh, const state_type& x) {
#include "_ref/ctrl_get_controls.inc"
}
double Controller::getAccelerationCommand(const Vehicle& veh, const MyReference& ref, const state_type& x) {
#include "_ref/ctrl_accel.inc"
}
double Controller::getSteerCommand(const MyReference& ref, const state_type& x, const Vehicle& veh) {
#include "_ref/ctrl_steer.inc"
}
void Controller::updateWaypoint(const MyReference& ref, const state_type& x) {
#include "_ref/ctrl_update_waypoint.inc"
}

// ------------------------------------------------------------------------------------ simulation.cpp
class Simulation {  // simulation.h:7-21
 private:
  void propagate(const RRTd& RRT, Controller control, const MyReference& ref, const Vehicle& veh);

 public:
  StateArray stateArray;
  vector<double> curvature;
  vector<int> closestPoints;
  vector<double> acmd, dcmd;
  double costS, costE;
  bool goalReached, endReached;
  Simulation(const RRTd& RRT, const vector<double>& state, MyReference& ref, const Vehicle& veh,
             const bool& GoalBiased, const bool& genProfile, const double& Vstart);
};
Simulation::Simulation(const RRTd& RRT, const vector<double>& state, MyReference& ref, const Vehicle& veh,
                       const bool& GoalBiased, const bool& genProfile, const double& Vstart)
    : costE(0), costS(0), goalReached(false), endReached(false) {
#include "_ref/sim_ctor.inc"
}
void Simulation::propagate(const RRTd& RRT, Controller control, const MyReference& ref, const Vehicle& veh) {
#include "_ref/sim_propagate.inc"
}

// ------------------------------------------------------------------------------------ tree level
void expandTree(Vehicle& veh, RRTd& RRT) {
#include "_ref/expand_a.inc"
  Pt sample;
#include "_ref/expand_b.inc"
}
double getNodeCost(const RRTd& RRT, const Vehicle& veh, const double& parentCost, const Node& node,
                   const vector<int> det) {
#include "_ref/node_cost.inc"
}
void initializeTree(RRTd& RRT, const Vehicle& veh, vector<Node>& nodes, vector<double>& carState) {
#include "_ref/initialize_tree.inc"
}
vector<Node> extractBestPath(vector<Node> tree) {
#include "_ref/best_path.inc"
}

// ------------------------------------------------------------------------------------ driver state
static RRTd g_rrt;         // the planner of the tree-level entry points
static vector<Node> g_best;  // MotionPlanner::bestNodes

static Vehicle prius() {
  Vehicle v;
  v.setPrius();
  return v;
}

// Outcome of a finished Simulation, from its flags and the failure counters it bumped.
static int sim_outcome(const Simulation& s, int col0, int acc0, int it0) {
  if (s.endReached) return 1;       // CLRRT_ROLL_END
  if (s.goalReached) return 2;      // CLRRT_ROLL_GOAL
  if (fail_collision != col0) return 3;
  if (fail_acclimit != acc0) return 4;
  (void)it0;
  return 0;                         // CLRRT_ROLL_ITERLIMIT
}

// Node export: state[0..9], parent, costE, costS, goal, nrows, ref N, ref front x/y, ref back x/y,
// ref.v.back() (0 when empty), ref.v.size()
static const int NODE_W = 22;
static void export_node(const Node& n, double* o) {
  for (int i = 0; i < 10; i++) o[i] = i < (int)n.state.size() ? n.state[i] : 0.0;
  o[10] = n.parentID;
  o[11] = n.costE;
  o[12] = n.costS;
  o[13] = n.goalReached;
  o[14] = (double)n.tra.size();
  o[15] = (double)n.ref.x.size();
  o[16] = n.ref.x.empty() ? 0.0 : n.ref.x.front();
  o[17] = n.ref.y.empty() ? 0.0 : n.ref.y.front();
  o[18] = n.ref.x.empty() ? 0.0 : n.ref.x.back();
  o[19] = n.ref.y.empty() ? 0.0 : n.ref.y.back();
  o[20] = n.ref.v.empty() ? 0.0 : n.ref.v.back();
  o[21] = (double)n.ref.v.size();
}
static void export_rows(const Node& n, double* o) {
  for (size_t r = 0; r < n.tra.size(); r++)
    for (int c = 0; c < 10; c++) o[r * 10 + c] = c < (int)n.tra[r].size() ? n.tra[r][c] : 0.0;
}
// A node as a tree loader gives it: state, parent, a 2-point reference [front, back] with
// v = [vback, vback], costs; one trajectory row (the state).
static Node import_node(const double* a) {
  Node n;
  n.state.assign(a, a + 10);
  n.parentID = (int)a[10];
  n.costE = (float)a[11];
  n.costS = (float)a[12];
  n.goalReached = a[13] != 0;
  n.ref.x = {a[16], a[18]};
  n.ref.y = {a[17], a[19]};
  n.ref.v = {a[20], a[20]};
  n.ref.dir = 1;
  n.tra.push_back(n.state);
  return n;
}

extern "C" {

// Parameter globals of rrt_node.cpp:15-18 at the parameters.launch values the oracle uses.
void ref_set_globals(double mindla, double tla, double dlavmin, double dt, double res) {
  ctrl_mindla = mindla; ctrl_tla = tla; ctrl_dlavmin = dlavmin; sim_dt = dt; ref_res = res;
  debug_velocity = 0; debug_mode = 0;
}

// The planner configuration of a query: cfg = sim_dt, tla, mindla, dlavmin, Kp, Ki, ref_res, ref_int,
// ref_mindist, vmax, Wcost[0..4], goal[0..3], collision (0 stub, 1 OBB), obs_use_pred, bend,
// laneShifts[0], Cxy[0..2]  (26 doubles)
void ref_config(const double* c) {
  sim_dt = c[0]; ctrl_tla = c[1]; ctrl_mindla = c[2]; ctrl_dlavmin = c[3]; ctrl_Kp = c[4]; ctrl_Ki = c[5];
  ref_res = c[6]; ref_int = c[7]; ref_mindist = c[8]; vmax = c[9];
  for (int i = 0; i < 5; i++) g_rrt.Wcost[i] = c[10 + i];
  g_rrt.goalPose.assign(c + 15, c + 19);
  g_coll = (int)c[19];
  obs_use_pred = c[20] != 0;
  g_rrt.bend = c[21] != 0;
  g_rrt.laneShifts = {c[22], 0.0};
  g_rrt.Cxy.assign(c + 23, c + 26);
  debug_mode = 0; debug_velocity = 0; debug_sim = 0; draw_states = 0;
}
void ref_set_obstacles(const double* obs7, int m) {
  g_det.clear();
  for (int i = 0; i < m; i++) {
    const double* d = obs7 + 7 * i;
    g_det.push_back(Det{d[0], d[1], d[2], d[3], d[4], d[5], d[6]});
  }
}
void ref_srand(unsigned s) { srand(s); }
int ref_rand(void) { return rand(); }
void ref_counters(long* out4) {
  out4[0] = sim_count; out4[1] = fail_collision; out4[2] = fail_acclimit; out4[3] = fail_iterlimit;
}
void ref_reset_counters(void) { sim_count = fail_collision = fail_acclimit = fail_iterlimit = 0; }

// in: x, y, th, t, cx, cy, oth, size_x, size_y, vx, vy (11 doubles per case) -> getOBBdist.
double ref_obb_one(const double* a, int mode, uint64_t key) {
  vector<double> states(10, 0.0);
  states[0] = a[0]; states[1] = a[1]; states[2] = a[2]; states[6] = a[3];
#include "_ref/veh_box.inc"
  // getOBBvector old_collisioncheck.cpp:14-16 (its car_msgs field accesses, on plain doubles)
  double t = a[3];
  OBB obs(Vector2D(a[4] + a[9] * t, a[5] + a[10] * t), a[7] / 2, a[8] / 2, a[6]);
  set_axis3(vOBB, mode, 2 * key);
  set_axis3(obs, mode, 2 * key + 1);
  return getOBBdist(vOBB, obs);
}
void ref_obb(int n, const double* in, int mode, double* out) {
  for (int k = 0; k < n; k++) out[k] = ref_obb_one(in + 11 * k, mode, (uint64_t)k);
}

// OBB(pos, w, h, o) -> verticesX/Y, normsX[0..3], normsY[0..2] and, in slot 15, normsX[3] again.
void ref_obb_geom(int n, const double* in, float* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 5 * k;
    OBB b(Vector2D(a[0], a[1]), (float)a[2], (float)a[3], (float)a[4]);
    float* o = out + 16 * k;
    for (int i = 0; i < 4; i++) { o[i] = b.verticesX[i]; o[4 + i] = b.verticesY[i]; o[8 + i] = b.normsX[i]; }
    for (int i = 0; i < 3; i++) o[12 + i] = b.normsY[i];
    o[15] = b.normsX[3];
  }
}

// VehicleODE then IntegrateEuler on a 10-element state (Prius, dt = sim_dt).
// in: x0..x6, dc, ac; out: x0..x9 after the step, dx[2] (11 doubles).
void ref_ode(int n, const double* in, double* out) {
  Vehicle veh = prius();
  for (int k = 0; k < n; k++) {
    const double* a = in + 9 * k;
    state_type x(10, 0.0);
    for (int i = 0; i < 7; i++) x[i] = a[i];
    x[7] = 7.0; x[8] = 8.0; x[9] = 9.0;
    ControlCommand ctrl(a[7], a[8]);
    double dt = sim_dt;
    state_type dx = VehicleODE(ctrl, x, veh);
    IntegrateEuler(ctrl, x, dx, dt, veh);
    for (int i = 0; i < 10; i++) out[11 * k + i] = x[i];
    out[11 * k + 10] = dx[2];
  }
}

// in: xval[3], yval[3], X[3] -> interpolate(transformToVehicle(...)).
void ref_lateral(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    double xv[3], yv[3], X[3], Tx[3], Ty[3];
    for (int i = 0; i < 3; i++) { xv[i] = in[9 * k + i]; yv[i] = in[9 * k + 3 + i]; X[i] = in[9 * k + 6 + i]; }
    transformToVehicle(xv, yv, Tx, Ty, X);
    out[k] = interpolate(Tx, Ty);
  }
}

void ref_linspace(double a, double b, long N, double* out) {
  vector<double> v = LinearSpacedVector(a, b, (std::size_t)N);
  for (long i = 0; i < N; i++) out[i] = v[i];
}

// getReference's body (reference.cpp:13-18) toward (sx, sy) from a parent whose ref ends at (ax, ay),
// then generateVelocityProfile.  in: ax, ay, sx, sy, res, v0, vmax, goal[4], GB; out: N, v[0..N).
void ref_profile(int n, const double* in, int nmax, double* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 12 * k;
    struct { double x, y; } sample;
    struct { MyReference ref; } node;
    sample.x = a[2]; sample.y = a[3];
    node.ref.x.assign(1, a[0]);
    node.ref.y.assign(1, a[1]);
    int dir = 1;
    ref_res = a[4];
#include "_ref/get_reference.inc"
    vector<double> goal(a + 7, a + 11);
    generateVelocityProfile(ref, 0, 0, a[5], a[6], goal, a[11] != 0);
    double* row = out + (std::size_t)(1 + nmax) * k;
    row[0] = (double)ref.v.size();
    for (std::size_t i = 0; i < ref.v.size() && (int)i < nmax; i++) row[1 + i] = ref.v[i];
  }
}

// angleDiff(a, b), wrapToPi(a)
void ref_angle(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    out[2 * k] = angleDiff(in[2 * k], in[2 * k + 1]);
    out[2 * k + 1] = wrapToPi(in[2 * k]);
  }
}

// Vehicle::setPrius: dmax, ddmax, Td, Ta, amin, amax, L, w, Lrear, Lfront, b, Vch, rho, Kus
void ref_prius(double* out) {
  Vehicle v = prius();
  const double f[14] = {v.dmax, v.ddmax, v.Td, v.Ta, v.amin, v.amax, v.L, v.w, v.Lrear, v.Lfront, v.b, v.Vch, v.rho, v.Kus};
  for (int i = 0; i < 14; i++) out[i] = f[i];
}

// updateLookahead(v) -> ctrl_dla; updateReferenceResolution(v) -> ref_res (controller.cpp:13-21), with
// the globals of the last ref_config.  out: 2 doubles per v.
void ref_lookahead_res(int n, const double* v, double* out) {
  const double res0 = ref_res;
  for (int k = 0; k < n; k++) {
    updateLookahead(v[k]);
    updateReferenceResolution(v[k]);
    out[2 * k] = ctrl_dla;
    out[2 * k + 1] = ref_res;
  }
  ref_res = res0;
}

// dubinsDistance(S, N, 1).  in: sx, sy, node x, y, heading, costE (6 doubles; costE unused) -> the
// float key.
void ref_dubins(int n, const double* in, float* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 6 * k;
    Pt S;
    S.x = a[0]; S.y = a[1];
    Node N;
    N.state.assign(10, 0.0);
    N.state[0] = a[2]; N.state[1] = a[3]; N.state[2] = a[4];
    out[k] = dubinsDistance(S, N, 1);
  }
}

// feasibleNode(rrt, node, sample).  in: sx, sy, ref front x, y, ref back x, y, ref_res.
void ref_feasible(int n, const double* in, double* out) {
  const double res0 = ref_res;
  for (int k = 0; k < n; k++) {
    const double* a = in + 7 * k;
    ref_res = a[6];
    Pt s;
    s.x = a[0]; s.y = a[1];
    Node N;
    N.ref.x = {a[2], a[4]};
    N.ref.y = {a[3], a[5]};
    out[k] = feasibleNode(g_rrt, N, s) ? 1.0 : 0.0;
  }
  ref_res = res0;
}

// feasibleGoalBias with the new node as tree.back().  in: goal[4], node x, y, ref back x, y.
void ref_goal_bias(int n, const double* in, double* out) {
  RRTd r;
  for (int k = 0; k < n; k++) {
    const double* a = in + 8 * k;
    r.goalPose.assign(a, a + 4);
    Node N;
    N.state.assign(10, 0.0);
    N.state[0] = a[4]; N.state[1] = a[5];
    N.ref.x = {a[6] - 1.0, a[6]};
    N.ref.y = {a[7], a[7]};
    r.tree.assign(1, N);
    out[k] = feasibleGoalBias(r) ? 1.0 : 0.0;
  }
}

// getGoalReference(veh, node, goal) + generateVelocityProfile(GB = true) from v0 at the current vmax.
// in: goal[4], parent ref back x, y, v0, ref_res (8 doubles); out row (1 + 3 nmax): N, v, x, y.
void ref_goal_ref(int n, const double* in, int nmax, double* out) {
  Vehicle veh = prius();
  const double res0 = ref_res;
  for (int k = 0; k < n; k++) {
    const double* a = in + 8 * k;
    ref_res = a[7];
    vector<double> goal(a, a + 4);
    Node N;
    N.ref.x = {a[4]};
    N.ref.y = {a[5]};
    MyReference ref = getGoalReference(veh, N, goal);
    generateVelocityProfile(ref, 0, 0, a[6], vmax, goal, true);
    double* row = out + (std::size_t)(1 + 3 * nmax) * k;
    row[0] = (double)ref.x.size();
    for (std::size_t i = 0; i < ref.x.size() && (int)i < nmax; i++) {
      row[1 + i] = i < ref.v.size() ? ref.v[i] : 0.0;
      row[1 + nmax + i] = ref.x[i];
      row[1 + 2 * nmax + i] = ref.y[i];
    }
  }
  ref_res = res0;
}

// sampleAroundVehicle(goal) + the heuristic draw (:142), n iterations from the current rand() state.
// out: x, y, r per iteration.
void ref_sample(int n, const double* goal4, double* out) {
  vector<double> g(goal4, goal4 + 4);
  for (int k = 0; k < n; k++) {
    Pt s = sampleAroundVehicle(g);
#include "_ref/heuristic_draw.inc"
    out[3 * k] = s.x; out[3 * k + 1] = s.y; out[3 * k + 2] = r;
  }
}

// sortNodesExplore / sortNodesOptimize over a tree of `nn` imported nodes (NODE_W doubles each) for
// `ns` samples (sx, sy, explore).  out_ids[10 * k + j] (-1 padded), out_n[k] = list length.
void ref_sort_nodes(int nn, const double* nodes, int ns, const double* samples, int* out_ids, int* out_n) {
  RRTd r;
  r.tree.clear();
  for (int i = 0; i < nn; i++) r.tree.push_back(import_node(nodes + NODE_W * i));
  for (int k = 0; k < ns; k++) {
    Pt s;
    s.x = samples[3 * k]; s.y = samples[3 * k + 1];
    vector<int> l = samples[3 * k + 2] != 0 ? sortNodesExplore(r, s) : sortNodesOptimize(r, s);
    out_n[k] = (int)l.size();
    for (int j = 0; j < 10; j++) out_ids[10 * k + j] = j < (int)l.size() ? l[j] : -1;
  }
}

// Controller over a state sequence: the Simulation constructor's order (simulation.cpp:39-43: the
// controller on the first state, then the velocity profile), then getControls on each state.
// in (12 + 6 K doubles): kind (0: getReference from (a0, a1) toward (a2, a3); 1: getGoalReference from
// ref back (a0, a1)), a0..a3, goal[4], Vstart, vmax, ref_res, then K states (x, y, heading, delta, v, a).
// out (4 + 8 K): IDwp, endreached, Ppreview after the constructor; per state IDwp, endreached, Px, Py,
// ym, dc, ac, iE.
void ref_controller(int n, const double* in, int K, double* out) {
  Vehicle veh = prius();
  const double vmax0 = vmax, res0 = ref_res;
  for (int k = 0; k < n; k++) {
    const double* a = in + (12 + 6 * K) * (size_t)k;
    ref_res = a[11];
    double* o = out + (4 + 8 * K) * (size_t)k;
    vector<double> goal(a + 5, a + 9);
    Node par;
    par.ref.x = {a[1]};
    par.ref.y = {a[2]};
    MyReference ref;
    const bool GB = a[0] != 0;
    if (GB) {
      ref = getGoalReference(veh, par, goal);
      ref.dir = 1;  // left uninitialised by reference.cpp:34 (see the header): canonical 1
    } else {
      Pt s;
      s.x = a[3]; s.y = a[4];
      ref = getReference(s, par, 1);
    }
    const double* st = a + 12;
    state_type x0(st, st + 6);
    x0.resize(10, 0.0);
    Controller control(ref, x0);
    o[0] = control.IDwp; o[1] = control.endreached; o[2] = control.Ppreview.x; o[3] = control.Ppreview.y;
    vmax = a[10];
    generateVelocityProfile(ref, 0, control.IDwp, a[9], vmax, goal, GB);
    for (int j = 0; j < K; j++) {
      state_type x(st + 6 * j, st + 6 * j + 6);
      x.resize(10, 0.0);
      ControlCommand c = control.getControls(ref, veh, x);
      double* q = o + 4 + 8 * j;
      q[0] = control.IDwp; q[1] = control.endreached; q[2] = control.Ppreview.x; q[3] = control.Ppreview.y;
      q[4] = control.ym; q[5] = c.dc; q[6] = c.ac; q[7] = control.iE;
    }
  }
  vmax = vmax0;
  ref_res = res0;
}

// Simulation(RRT, parent.state, ref, veh, GB, true, parent.ref.v.back()) as expandTree builds it
// (rrtplanner.cpp:151-152, 165-166) from imported parents.  jobs: parent index, gb, sx, sy.
// meta out (10 per job): outcome (CLRRT_ROLL_*), rows, costE, costS, ref N, ref.v.back(), ref back x, y,
// sim_count delta, 0; rows out: rows_cap x 10 per job.
void ref_simulate(int np, const double* parents, int nj, const double* jobs, int rows_cap, double* meta,
                  double* rows) {
  Vehicle veh = prius();
  vector<Node> P;
  for (int i = 0; i < np; i++) P.push_back(import_node(parents + NODE_W * i));
  for (int k = 0; k < nj; k++) {
    const double* j = jobs + 4 * k;
    const Node& par = P[(int)j[0]];
    MyReference ref;
    const bool gb = j[1] != 0;
    if (gb) {
      ref = getGoalReference(veh, par, g_rrt.goalPose);
      ref.dir = 1;  // left uninitialised by reference.cpp:34 (see the header): canonical 1
    } else {
      Pt s;
      s.x = j[2]; s.y = j[3];
      ref = getReference(s, par, 1);
    }
    const int c0 = fail_collision, a0 = fail_acclimit, i0 = fail_iterlimit, s0 = sim_count;
    Simulation sim(g_rrt, par.state, ref, veh, gb, true, par.ref.v.back());
    double* m = meta + 10 * (size_t)k;
    m[0] = sim_outcome(sim, c0, a0, i0);
    m[1] = (double)sim.stateArray.size();
    m[2] = sim.costE; m[3] = sim.costS;
    m[4] = (double)ref.x.size();
    m[5] = ref.v.back();
    m[6] = ref.x.back(); m[7] = ref.y.back();
    m[8] = sim_count - s0;
    m[9] = 0;
    if (rows) {
      double* o = rows + (size_t)rows_cap * 10 * k;
      for (size_t r = 0; r < sim.stateArray.size() && (int)r < rows_cap; r++)
        for (int c = 0; c < 10; c++) o[r * 10 + c] = sim.stateArray[r][c];
    }
  }
}

// ---- the tree (expandTree, addInitialNode, initializeTree, extractBestPath, node transforms)
void ref_tree_init(const double* root10) {
  g_rrt.tree.clear();
  g_rrt.addInitialNode(vector<double>(root10, root10 + 10));
}
void ref_tree_load(int n, const double* nodes) {
  g_rrt.tree.clear();
  for (int i = 0; i < n; i++) g_rrt.tree.push_back(import_node(nodes + NODE_W * i));
}
void ref_tree_expand(long n_iters) {
  Vehicle veh = prius();
  for (long i = 0; i < n_iters; i++) expandTree(veh, g_rrt);
}
long ref_tree_size(void) { return (long)g_rrt.tree.size(); }
void ref_tree_nodes(long first, long count, double* out) {
  for (long k = 0; k < count; k++) export_node(g_rrt.tree[first + k], out + NODE_W * k);
}
void ref_tree_rows(long i, double* out) { export_rows(g_rrt.tree[i], out); }

// bestNodes = extractBestPath(RRT.tree) (motionplanner.cpp:51); returns its size.
long ref_best_path(void) {
  g_best = extractBestPath(g_rrt.tree);
  return (long)g_best.size();
}
long ref_best_size(void) { return (long)g_best.size(); }
void ref_best_clear(void) { g_best.clear(); }
void ref_best_nodes(double* out) {
  for (size_t k = 0; k < g_best.size(); k++) export_node(g_best[k], out + NODE_W * k);
}
void ref_best_rows(long i, double* out) { export_rows(g_best[i], out); }
// transformNodesWorldToCar (to_world 0) / transformNodesCarToworld (1) of bestNodes (pose: x, y, heading)
void ref_best_transform(int to_world, const double* pose3) {
  vector<double> cs(pose3, pose3 + 3);
  cs.resize(6, 0.0);
  if (to_world) transformNodesCarToworld(g_best, cs);
  else transformNodesWorldToCar(g_best, cs);
}
// MyRRT RRT(goal, ...); RRT.carState = carPose; initializeTree(RRT, veh, bestNodes, carPose)
// (motionplanner.cpp:23-32).  car6: x, y, heading, delta, v, a.
void ref_initialize_tree(const double* car6) {
  Vehicle veh = prius();
  RRTd fresh = g_rrt;
  fresh.tree.clear();
  vector<double> carPose(car6, car6 + 6);
  fresh.carState = carPose;
  initializeTree(fresh, veh, g_best, carPose);
  g_rrt.tree = fresh.tree;
}

}  // extern "C"
