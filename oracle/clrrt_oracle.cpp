// clrrt_oracle.cpp — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from
// the product (cl-rrt_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg use it, as the checker / the timed CPU reference.
//
// A plain C++ restatement of the reference's expandTree hot path (vdBerg93/cl-rrt, paths relative
// to the reference root), kept arithmetic-for-arithmetic faithful so that it reproduces the
// reference's outputs bit-for-bit on the same glibc:
//   * float/double typing exactly as the reference declares it (Dubins key and OBB SAT in float,
//     dynamics in double, Node costs narrowed to float);
//   * std::sort over (node id, key) pairs, nodes passed BY VALUE to the Dubins key (the
//     reference's cost profile, rrtplanner.cpp:371);
//   * glibc rand() consumed in the reference order;
//   * canonical semantics for the reference's out-of-bounds reads: every read of
//     ref.x / ref.y / ref.v past the end yields 0.0 — what the reference computes when its heap is
//     zero-filled, which is how the survey pinned it (SURVEY §8(c) "Determinism recipe").
//   * OBB axis 3 (setNorms leaves normsY[3] unset, old_collisioncheck.cpp:74-75): taken as the
//     proper edge normal of edge 3->0.  Decision-neutral (any separating axis proves separation).
//
// Pinned against the survey's golden outputs of the reference (tests/golden/survey_pins.json).
#define _GNU_SOURCE 1
#include <math.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <chrono>
#include <thread>
#include <utility>
#include <vector>

#include "../include/clrrt.h"

namespace orc {

// ---------------------------------------------------------------- libm call sites
// GCC -O2 merges sin(x) and cos(x) of one argument into glibc's sincos() where it can prove the
// argument unchanged between the two calls, and glibc's sincos (generic build) rounds differently
// from its sin/cos (FMA builds) in ~0.1% of arguments.  The reference's goal-biased rollouts are
// ill-conditioned enough for that to matter, so every call site below names its libm entry point
// explicitly (the choice GCC makes for the reference's code structure); the GPU kernels restate
// the same entry point per site (cl-rrt_amd/csrc/clrrt_glibc.hpp).
__attribute__((noinline)) static double lm_sin(double x) { return ::sin(x); }
__attribute__((noinline)) static double lm_cos(double x) { return ::cos(x); }
__attribute__((noinline)) static double lm_tan(double x) { return ::tan(x); }
__attribute__((noinline)) static void lm_sincos(double x, double* s, double* c) { ::sincos(x, s, c); }
__attribute__((noinline)) static void lm_sincosf(float x, float* s, float* c) { ::sincosf(x, s, c); }
__attribute__((noinline)) static float lm_sinf(float x) { return ::sinf(x); }

using std::vector;
using std::pair;
using std::make_pair;
typedef vector<double> Row;

struct Pt { double x = 0, y = 0; };

// MyReference (rrtplanner.h:27-33)
struct Ref {
  vector<double> x, y, v;
  int dir = 1;
};

// Out-of-range reads yield 0.0 (canonical zero-fill semantics).
static inline double at0(const vector<double>& a, long i) {
  return (i >= 0 && (size_t)i < a.size()) ? a[(size_t)i] : 0.0;
}

// Node (rrtplanner.h:35-48)
struct Node {
  vector<double> state;
  int parentID = -1;
  Ref ref;
  float costE = 0, costS = 0;
  bool goalReached = false;
  vector<Row> tra;
};

struct Obs { double cx, cy, th, sx, sy, vx, vy; };

// Controller::dla (controller.h: the lookahead the reference keeps in its global controller object):
// set by updateLookahead at each rollout's start and read by that rollout only; per thread, so that
// orc_eval_iterations' threads do not share it.
static thread_local double g_ctrl_dla = 0;

struct Oracle {
  clrrt_params p;
  int64_t sim_count = 0, fail_collision = 0, fail_acclimit = 0, fail_iterlimit = 0, rollouts = 0;
  vector<Obs> det;
  vector<Node> tree;
  vector<Node> best;  // MotionPlanner::bestNodes (motionplanner.h:23): the committed path
  // test expansions only (orc_expand_batch_defer_mt): keys from cached node rotations without the by-value Node
  // copy, and the stable order's prefix by partial sorts -- the same lists
  bool keys_by_ref = false;
  vector<float> rot;  // (sin, cos) of each node's dubinsDistance rotation angle
};

// ---------------------------------------------------------------- helpers (functions.h)
// LinearSpacedVector functions.h:11-20 — accumulating linspace (val += h)
static vector<double> linspace(double a, double b, size_t N) {
  double h = (b - a) / static_cast<double>(N - 1);
  vector<double> out(N);
  double val = a;
  for (size_t k = 0; k < N; ++k, val += h) out[k] = val;
  return out;
}
template <typename T> static int sgn(T v) { return (T(0) < v) - (v < T(0)); }
// wrapToPi functions.h:43-48
static double wrap_pi(double x) {
  x = std::fmod(x + M_PI, 2 * M_PI);
  if (x < 0) x += 2 * M_PI;
  return x - M_PI;
}
// angleDiff functions.h:50-57
static double angle_diff(double a, double b) {
  double d = std::fmod(b - a + M_PI, 2 * M_PI);
  if (d < 0) d += 2 * M_PI;
  return d - M_PI;
}
// checkSaturation functions.h:61-63 / enforceConstraints simulation.cpp:7-9
static double sat(double lo, double hi, double v) { return std::max(std::min(v, hi), lo); }

// ---------------------------------------------------------------- controller (controller.cpp)
static void update_lookahead(Oracle& o, double v) {  // controller.cpp:13-16
  double dla_c = o.p.ctrl_mindla - o.p.ctrl_tla * o.p.ctrl_dlavmin;
  g_ctrl_dla = std::max(o.p.ctrl_mindla, dla_c + o.p.ctrl_tla * std::abs(v));
}

static int closest_point(const Ref& r, const Pt& q, int from) {  // controller.cpp:96-113
  double best = INFINITY, d;
  int arg = 0;
  for (int i = from; i < (int)r.x.size(); i++) {
    d = (r.x[i] - q.x) * (r.x[i] - q.x) + (r.y[i] - q.y) * (r.y[i] - q.y);
    if (d < best) { best = d; arg = i; }
  }
  return arg;
}

// transformToVehicle controller.cpp:115-132 then interpolate :134-148 (X = preview point + heading)
static double transform_interp(const double xv[3], const double yv[3], double X0, double X1, double X2) {
  double tx[3], ty[3];
  double sX, cX;
  lm_sincos(X2, &sX, &cX);  // transformToVehicle: sin/cos of one argument -> sincos
  for (int i = 0; i < 3; i++) {
    tx[i] = xv[i] * cX - X0 * cX - yv[i] * sX + X1 * sX;
    ty[i] = yv[i] * cX - X1 * cX + xv[i] * sX - X0 * sX;
  }
  double y = 0, L;
  for (int i = 0; i < 3; i++) {
    L = 1;
    for (int j = 0; j < 3; j++)
      if (i != j) L = L * (tx[j]) / (tx[i] - tx[j]);
    y = y + ty[i] * L;
  }
  return y;
}

static double lateral_error(const Ref& r, const Row& x, int wp, const Pt& P) {  // getLateralError :70-93
  int lo, hi;
  if (wp == 0) { lo = wp; hi = wp + 2; }
  else if (wp == (int)r.x.size()) { lo = wp - 2; hi = wp; }
  else { lo = wp - 1; hi = wp + 1; }
  double xv[3] = {at0(r.x, lo), at0(r.x, lo + 1), at0(r.x, hi)};
  double yv[3] = {at0(r.y, lo), at0(r.y, lo + 1), at0(r.y, hi)};
  return transform_interp(xv, yv, P.x, P.y, x[2]);
}

struct Ctrl {  // class Controller controller.h:8-28
  int IDwp = 0;
  Pt P;
  double ym = 0, iE = 0;
  bool endreached = false;

  void update_waypoint(Oracle& o, const Ref& r, const Row& x) {  // controller.cpp:53-68
    update_lookahead(o, x[4]);
    P.x = x[0] + g_ctrl_dla * r.dir * lm_cos(x[2]);  // a store between the two calls: no sincos
    P.y = x[1] + g_ctrl_dla * r.dir * lm_sin(x[2]);
    IDwp = closest_point(r, P, IDwp);
    if ((size_t)IDwp >= r.x.size() - 1 - 2) endreached = true;
    if (at0(r.x, IDwp) == r.x.back() && at0(r.y, IDwp) == r.y.back()) endreached = true;
  }
  Ctrl(Oracle& o, const Ref& r, const Row& x) {  // controller.cpp:23-28
    update_lookahead(o, x[4]);
    IDwp = 0; endreached = false; iE = 0;
    update_waypoint(o, r, x);
  }
  double steer(Oracle& o, const Ref& r, const Row& x) {  // :47-51
    const clrrt_vehicle& veh = o.p.veh;
    ym = lateral_error(r, x, IDwp, P);
    double cmd = 2 * ((veh.L + veh.Kus * x[4] * x[4]) / pow(g_ctrl_dla, 2)) * ym;
    return sat(-veh.dmax, veh.dmax, cmd);
  }
  double accel(Oracle& o, const Ref& r, const Row& x) {  // :37-45 (LAlong = 2, :35)
    double E = at0(r.v, IDwp + 2) - x[4];
    iE = iE + E * o.p.sim_dt;
    return sat(o.p.veh.amin, o.p.veh.amax, o.p.ctrl_Kp * E + o.p.ctrl_Ki * iE);
  }
};

// ---------------------------------------------------------------- references (reference.cpp)
static Ref get_reference(Oracle& o, Pt s, Node node, int dir) {  // reference.cpp:9-22 (node by value)
  Ref r;
  double L = sqrt(pow(s.x - node.ref.x.back(), 2) + pow(s.y - node.ref.y.back(), 2));
  int N = round(L / o.p.ref_res) + 1;
  r.x = linspace(node.ref.x.back(), s.x, N);
  r.y = linspace(node.ref.y.back(), s.y, N);
  r.dir = dir;
  return r;
}

static Ref get_goal_reference(Oracle& o, Node node, vector<double> g) {  // reference.cpp:25-70
  double dla_c = o.p.ctrl_mindla - o.p.ctrl_tla * o.p.ctrl_dlavmin;
  double dla_end = std::max(o.p.ctrl_mindla, dla_c + o.p.ctrl_tla * std::abs(g[3]));
  double Dext = dla_end, Dal = 1;
  Ref r;
  Pt P1, P2, Pc, Pf;
  double sg2, cg2;
  lm_sincos(g[2], &sg2, &cg2);
  P1.x = g[0] + Dal * cg2; P1.y = g[1] + Dal * sg2;
  P2.x = g[0] - Dal * cg2; P2.y = g[1] - Dal * sg2;
  double bx = node.ref.x.back(), by = node.ref.y.back();
  if (sqrt(pow(P1.x - bx, 2) + pow(P1.y - by, 2)) < sqrt(pow(P2.x - bx, 2) + pow(P2.y - by, 2))) {
    Pc = P1; Pf = P1;
  } else {
    Pc = P2; Pf = P2;
  }
  Pf.x += (Dext + Dal) * cg2;
  Pf.y += (Dext + Dal) * sg2;
  double N1 = round(sqrt(pow(Pc.x - bx, 2) + pow(Pc.y - by, 2)) / o.p.ref_res) + 1;
  double N2 = round(sqrt(pow(Pf.x - Pc.x, 2) + pow(Pf.y - Pc.y, 2)) / o.p.ref_res) + 1;
  vector<double> ax = linspace(bx, Pc.x, N1), bxv = linspace(Pc.x, Pf.x, N2);
  vector<double> ay = linspace(by, Pc.y, N1), byv = linspace(Pc.y, Pf.y, N2);
  r.x = ax; r.x.insert(r.x.end(), bxv.begin(), bxv.end());
  r.y = ay; r.y.insert(r.y.end(), byv.begin(), byv.end());
  return r;
}

// generateVelocityProfile reference.cpp:73-170 (a_acc = 1, a_dec = -1, tmin = 1 at :77)
static void velocity_profile(Oracle& o, Ref& r, double v0, double vmax, const vector<double>& g,
                             bool GB) {
  double vend = g[3];
  double aa = 1, ad = -1, tmin = 1;
  double Lp, res;
  if (GB) {
    double Dg = sqrt(pow(g[0] - r.x.front(), 2) + pow(g[1] - r.y.front(), 2));
    Lp = Dg + o.p.ctrl_mindla;
    res = Lp / (r.x.size() - 1);
  } else {
    double Dg = sqrt(pow(g[0] - r.x.back(), 2) + pow(g[1] - r.y.back(), 2));
    double Lref = sqrt(pow(r.x.front() - r.x.back(), 2) + pow(r.y.front() - r.y.back(), 2));
    res = Lref / (r.x.size() - 1);
    Lp = Lref + Dg + o.p.ctrl_mindla;
  }
  double Dacc = (pow(vmax, 2) - pow(v0, 2)) / (2 * aa);
  double Dcst = vmax * tmin;
  double Dbrk = (pow(vend, 2) - pow(vmax, 2)) / (2 * ad);
  bool fits = (Dacc + Dcst + Dbrk) < Lp;
  double Vc;
  if (vend > (v0 + 0.1)) {
    Vc = vend;
  } else if (fits) {
    Vc = vmax;
  } else {
    double D = Lp;
    Vc = (sqrt(pow(aa, 2) * pow(ad, 2) * pow(tmin, 2) - 2 * D * pow(aa, 2) * ad +
               pow(aa, 2) * pow(vend, 2) + 2 * D * aa * pow(ad, 2) - aa * ad * pow(v0, 2) -
               aa * ad * pow(vend, 2) + pow(ad, 2) * pow(v0, 2)) +
          aa * ad * tmin) /
         (aa - ad);
  }
  Dacc = (pow(Vc, 2) - pow(v0, 2)) / (2 * aa);
  if (Dacc < 0) { Dacc = 0; Vc = v0; }
  Dbrk = std::max(double(0), (pow(vend, 2) - pow(Vc, 2)) / (2 * ad));
  Dcst = std::max(double(0), Lp - Dacc - Dbrk);
  double tbrk = (vend - Vc) / ad;
  r.v.clear();
  for (size_t i = 0; i != r.x.size(); i++) {
    double D = i * res;
    if (D < Dacc) {
      double t1 = -(v0 - sqrt(pow(v0, 2) + 2 * aa * D)) / aa;
      double t2 = -(v0 + sqrt(pow(v0, 2) + 2 * aa * D)) / aa;
      double t = (t1 >= 0) * t1 + (t2 >= 0) * t2;
      r.v.push_back(v0 + aa * t);
    } else if (D <= (Dacc + Dcst)) {
      r.v.push_back(Vc);
    } else {
      double q = pow(Vc, 2) + 2 * D * ad - 2 * Dacc * ad - 2 * Dcst * ad;
      double t1 = -(Vc + sqrt(q)) / ad;
      double t2 = -(Vc - sqrt(q)) / ad;
      double dt = (t1 != tbrk) * (t1 >= 0) * (t1 <= tbrk) * t1 + (t2 >= 0) * (t2 <= tbrk) * t2;
      r.v.push_back(std::max(double(0), Vc + ad * dt));
    }
  }
}

// ---------------------------------------------------------------- collision (old_collisioncheck.cpp)
struct Box {  // class OBB collision.h:16-34 (float fields)
  double px, py;
  float w, h, o;
  float vx[4], vy[4], nx[4], ny[4], mm[2];
  Box(double _px, double _py, float _w, float _h, float _o) : px(_px), py(_py), w(_w), h(_h), o(_o) {
    // setVertices old_collisioncheck.cpp:56-65 (float cos/sin of o -> sincosf)
    float so, co;
    lm_sincosf(o, &so, &co);
    vx[0] = px + co * (h / 2) - so * (w / 2);
    vy[0] = py + so * (h / 2) + co * (w / 2);
    vx[1] = px + co * (h / 2) - so * (-w / 2);
    vy[1] = py + so * (h / 2) + co * (-w / 2);
    vx[2] = px + co * (-h / 2) - so * (-w / 2);
    vy[2] = py + so * (-h / 2) + co * (-w / 2);
    vx[3] = px + co * (-h / 2) - so * (w / 2);
    vy[3] = py + so * (-h / 2) + co * (w / 2);
    // setNorms :67-76, axis 3 canonicalised to the proper edge normal
    for (int i = 0; i < 3; i++) {
      nx[i] = vy[i + 1] - vy[i];
      ny[i] = -(vx[i + 1] - vx[i]);
    }
    nx[3] = vy[0] - vy[3];
    ny[3] = -(vx[0] - vx[3]);
  }
  void maxmin(float ax, float ay) {  // findMaxMin :78-95
    mm[0] = vx[0] * ax + vy[0] * ay;
    mm[1] = mm[0];
    for (int i = 1; i <= 3; i++) {
      float pr = vx[i] * ax + vy[i] * ay;
      if (pr > mm[0]) mm[0] = pr;
      else if (pr < mm[1]) mm[1] = pr;
    }
  }
};

static double box_gap(Box a, Box b) {  // getOBBdist :98-148 (first separating gap, 0 = overlap)
  for (int pass = 0; pass < 2; pass++) {
    const Box& src = pass == 0 ? a : b;
    float ax[4], ay[4];
    for (int i = 0; i < 4; i++) { ax[i] = src.nx[i]; ay[i] = src.ny[i]; }
    for (int i = 0; i <= 3; i++) {
      a.maxmin(ax[i], ay[i]);
      float ap[2] = {a.mm[0], a.mm[1]};
      b.maxmin(ax[i], ay[i]);
      float bp[2] = {b.mm[0], b.mm[1]};
      float D1 = bp[1] - ap[0];
      float D2 = ap[1] - bp[0];
      if (D1 > 0) return D1;
      else if (D2 > 0) return D2;
    }
  }
  return 0;
}

// getOBBvector old_collisioncheck.cpp:14-16: one obstacle's OBB at time t
static Box obs_box(const Obs& d, double t) { return Box(d.cx + d.vx * t, d.cy + d.vy * t, d.sx / 2, d.sy / 2, d.th); }

// checkObsDistance :34-36: the vehicle OBB centred 1.424 m ahead of the rear axle
static Box veh_box(const Row& x) {
  double sv, cv;
  lm_sincos(x[2], &sv, &cv);
  return Box(x[0] + 1.424 * cv, x[1] + 1.424 * sv, 2, 4.848, x[2]);
}

// checkObsDistance: stub collisioncheck.cpp:6-8, or the obstacle form old_collisioncheck.cpp:24-51
static double obs_distance(Oracle& o, const Row& x) {
  if (o.p.collision_mode == CLRRT_COLLISION_STUB) return 100;
  double t = o.p.obs_use_pred ? x[6] : 0;
  vector<Box> boxes;  // getOBBvector :6-22 (rebuilt every call, as the reference does)
  for (size_t i = 0; i != o.det.size(); i++) boxes.push_back(obs_box(o.det[i], t));
  Box veh = veh_box(x);
  double best = 10000;
  for (size_t j = 0; j != boxes.size(); j++) {
    double D = box_gap(veh, boxes[j]);
    if (D == 0) return 0;
    else if (D < best) best = D;
  }
  return best;
}

// ---------------------------------------------------------------- simulation (simulation.cpp)
struct Sim {
  vector<Row> rows;
  double costE = 0, costS = 0;
  bool goalReached = false, endReached = false;
  int outcome = CLRRT_ROLL_ITERLIMIT;
};

static double dist_to_lane(double x, double y, double S, const double* C) {  // :49-53
  double Lx = (x - S * C[1] + y * C[1] - C[1] * C[2]) / (pow(C[1], 2) + 1);
  double Ly = S + C[2] + (C[1] * (x - S * C[1] + y * C[1] - C[1] * C[2])) / (pow(C[1], 2) + 1);
  return sqrt(pow(Lx - x, 2) + pow(Ly - y, 2));
}

// VehicleODE simulation.cpp:11-25 then IntegrateEuler :27-34 on x[0..6] (the loop's indices 7..10
// read dx past its 7 elements: zero under the canonical zero-fill, so x[7..9] keep their values and
// are overwritten by propagate).  dx is returned for the lateral-acceleration test (:98).
static void ode_euler(const Oracle& o, Row& x, double dc, double ac, double dx[7]) {
  const clrrt_vehicle& veh = o.p.veh;
  const double dt = o.p.sim_dt;
  double Gss = 1 / (1 + pow((x[4] / veh.Vch), 2));
  // the store to dx[0] may alias x (both are vector<double> storage), so x[2] is reloaded and GCC
  // cannot merge cos and sin into sincos here: glibc cos() then sin() (checked against the
  // reference's own VehicleODE compiled at -O2/-O3, tests/test_ref_units.py)
  dx[0] = x[4] * lm_cos(x[2]);
  dx[1] = x[4] * lm_sin(x[2]);
  dx[2] = (x[4] / veh.L) * lm_tan(x[3]) * Gss;
  dx[3] = (1 / veh.Td) * (dc - x[3]);
  dx[4] = x[5];
  dx[5] = (1 / veh.Ta) * (ac - x[5]);
  dx[6] = 1;
  dx[4] = sat(veh.amin, veh.amax, dx[4]);
  dx[3] = sat(-veh.ddmax, veh.ddmax, dx[3]);
  for (int k = 0; k < 7; k++) x[k] = x[k] + dx[k] * dt;
  x[3] = sat(-veh.dmax, veh.dmax, x[3]);
}

static void propagate(Oracle& o, Sim& s, Ctrl c, const Ref& r) {  // :55-143
  const clrrt_vehicle& veh = o.p.veh;
  const double dt = o.p.sim_dt;
  for (int i = 0; i < (20 / dt); i++) {
    __atomic_fetch_add(&o.sim_count, 1, __ATOMIC_RELAXED);
    Row x = s.rows[i];
    // getControls controller.cpp:30-34 (braced init: steer before accel)
    c.update_waypoint(o, r, x);
    double dc = c.steer(o, r, x);
    double ac = c.accel(o, r, x);
    double dx[7];
    ode_euler(o, x, dc, ac, dx);
    x[7] = c.IDwp;
    x[8] = at0(r.v, c.IDwp + 2);
    x[9] = dc;
    s.rows.push_back(x);
    double Dobs = obs_distance(o, x);
    if (Dobs == 0) { s.endReached = false; __atomic_fetch_add(&o.fail_collision, 1, __ATOMIC_RELAXED); s.outcome = CLRRT_ROLL_COLLISION; return; }
    s.costE += x[4] * dt;
    double kappa = lm_tan(x[3]) / veh.L;
    s.costS += o.p.Wcost[0] * x[4] * dt + o.p.Wcost[1] * std::abs(kappa) +
               o.p.Wcost[2] * exp(-o.p.Wcost[3] * Dobs);
    if (o.p.bend) s.costS += o.p.Wcost[4] * dist_to_lane(x[0], x[1], o.p.lane_shift0, o.p.Cxy);
    double ay = std::abs(x[4] * dx[2]);
    if (ay + o.p.ay_road_max > 3) { s.endReached = false; __atomic_fetch_add(&o.fail_acclimit, 1, __ATOMIC_RELAXED); s.outcome = CLRRT_ROLL_ACCLIMIT; return; }
    double dg = sqrt(pow(x[0] - o.p.goal[0], 2) + pow(x[1] - o.p.goal[1], 2));
    double he = std::abs(angle_diff(x[2], o.p.goal[2]));
    double Ve = (x[4] - r.v.back());
    if (c.endreached && std::abs(Ve < 0.1)) { s.endReached = true; s.outcome = CLRRT_ROLL_END; return; }
    if ((dg <= 1) && (he < 0.05)) { s.goalReached = true; s.outcome = CLRRT_ROLL_GOAL; return; }
  }
  __atomic_fetch_add(&o.fail_iterlimit, 1, __ATOMIC_RELAXED);
}

// Simulation::Simulation :36-47 — mutates ref (fills ref.v)
static Sim simulate(Oracle& o, const vector<double>& state, Ref& r, bool GB, double Vstart) {
  Sim s;
  __atomic_fetch_add(&o.rollouts, 1, __ATOMIC_RELAXED);
  s.rows.push_back(state);
  Ctrl c(o, r, state);
  s.rows.back()[7] = c.IDwp;
  vector<double> g(o.p.goal, o.p.goal + 4);
  velocity_profile(o, r, Vstart, o.p.vmax, g, GB);
  propagate(o, s, c, r);
  return s;
}

// ---------------------------------------------------------------- tree (rrtplanner.cpp)
static Pt sample_around(Oracle& o) {  // :187-201
  const double* g = o.p.goal;
  double dGoal = sqrt(pow(g[0], 2) + pow(g[1], 2));
  double hd = atan2(g[1], g[0]);
  double latMin = -7, latMax = 7;
  Pt s;
  double rLong = static_cast<float>(rand()) / (static_cast<float>(RAND_MAX / (dGoal + 10)));
  double rLat = latMin + static_cast<float>(rand()) / (static_cast<float>(RAND_MAX / (latMax - latMin)));
  double sh, ch, sq, cq;
  lm_sincos(hd, &sh, &ch);
  lm_sincos(hd + M_PI / 2, &sq, &cq);
  s.x = rLong * ch + rLat * cq;
  s.y = rLong * sh + rLat * sq;
  return s;
}

// dubinsDistance :371-406, after the rotation angle's sincosf: the key of offset (qx, qy) from a node whose
// heading rotation is (sa, ca).
static float dubins_rot(float qx, float qy, float sa, float ca) {
  float rho = 4.77;
  float tmp = ca * qx - sa * qy;
  qy = std::abs(sa * qx + ca * qy);
  qx = tmp;
  float dc = std::sqrt(qx * qx + (qy - rho) * (qy - rho));
  float thc = std::atan2(qx, rho - qy);
  while (thc < 0) thc = thc + 2 * M_PI;
  float df = std::sqrt(qx * qx + (qy + rho) * (qy + rho));
  float alpha = 2 * M_PI - std::acos((5 * rho * rho - df * df) / (4 * rho * rho));
  bool inside = (qx * qx + (qy + rho) * (qy + rho) <= rho * rho) |
                (qx * qx + (qy - rho) * (qy - rho) <= rho * rho);
  if (!inside) return std::sqrt(dc * dc - rho * rho) + rho * (thc - std::acos(rho / dc));
  return rho * (alpha + std::asin(qx / df) - std::asin(rho * lm_sinf(alpha) / df));
}

// dubinsDistance :371-406 (Node by value, as the reference: the CPU baseline times that copy)
static float dubins(Pt S, Node N, int dir) {
  float qx = S.x - N.state[0];
  float qy = S.y - N.state[1];
  float ang = -N.state[2] - M_PI * (dir != 1);
  float sa, ca;
  lm_sincosf(ang, &sa, &ca);
  return dubins_rot(qx, qy, sa, ca);
}

// the same key from a node's cached rotation (Oracle::rot, dir = 1): the multi-threaded test expansions
// (orc_expand_batch_defer_mt), without the by-value copy of nodes that hold long trajectories
static float dubins_cached(const Oracle& o, const Pt& S, size_t i) {
  const Node& N = o.tree[i];
  float qx = S.x - N.state[0];
  float qy = S.y - N.state[1];
  return dubins_rot(qx, qy, o.rot[2 * i], o.rot[2 * i + 1]);
}
static void cache_rotations(Oracle& o) {
  for (size_t i = o.rot.size() / 2; i < o.tree.size(); i++) {
    float ang = -o.tree[i].state[2] - M_PI * (1 != 1);
    float sa, ca;
    lm_sincosf(ang, &sa, &ca);
    o.rot.push_back(sa);
    o.rot.push_back(ca);
  }
}

static bool feasible_node(Oracle& o, const Node& n, const Pt& s) {  // :271-289
  double angPar = atan2(n.ref.y.back() - n.ref.y.front(), n.ref.x.back() - n.ref.x.front());
  double angNew = atan2(s.y - n.ref.y.back(), s.x - n.ref.x.back());
  double Lref = sqrt(pow(n.ref.x.back() - s.x, 2) + pow(n.ref.y.back() - s.y, 2));
  if (std::abs(angle_diff(angNew, angPar)) > (M_PI / 4)) return false;
  if (Lref < (2.1 * o.p.ref_res)) return false;
  return true;
}

// sortNodesExplore :227-247 / sortNodesOptimize :250-268 over the first `upto` nodes
// stable = true: ties ordered by node id (std::stable_sort) -- the BATCH-mode semantics of the GPU
// engine; stable = false: std::sort exactly as the reference.
static vector<int> sort_nodes(Oracle& o, const Pt& s, bool explore, size_t upto,
                              vector<float>* keys_out = nullptr, bool stable = false) {
  vector<std::pair<int, float>> dv;
  auto by_key = [](const std::pair<int, float>& a, const std::pair<int, float>& b) { return a.second < b.second; };
  if (o.keys_by_ref && stable && o.rot.size() >= 2 * upto && !keys_out) {
    // test expansions: cached rotations, and the stable order's prefix by partial sorts on (key, id) -- the
    // stable sort of an id-ordered list is the (key, id) order when no key is NaN (else the full sort below)
    dv.reserve(upto);
    bool nan = false;
    for (size_t i = 0; i != upto; i++) {
      const float d = dubins_cached(o, s, i);
      float k = explore ? d : o.tree[i].costE + d;
      nan |= k != k;
      dv.push_back(std::make_pair((int)i, k));
    }
    if (!nan) {
      auto by_key_id = [](const std::pair<int, float>& a, const std::pair<int, float>& b) {
        return a.second < b.second || (a.second == b.second && a.first < b.first);
      };
      size_t K = std::min<size_t>(upto, 64), done = 0;
      vector<int> out;
      for (;;) {
        std::partial_sort(dv.begin() + done, dv.begin() + K, dv.end(), by_key_id);
        for (; done < K; done++) {
          if (feasible_node(o, o.tree[dv[done].first], s)) out.push_back(dv[done].first);
          if ((int)out.size() == o.p.sort_limit) return out;
        }
        if (K == upto) return out;
        K = std::min<size_t>(upto, 8 * K);
      }
    }
    std::stable_sort(dv.begin(), dv.end(), by_key);
  } else {
    for (size_t i = 0; i != upto; i++) {
      float k = explore ? dubins(s, o.tree[i], 1) : o.tree[i].costE + dubins(s, o.tree[i], 1);
      dv.push_back(std::make_pair((int)i, k));
    }
    if (stable) std::stable_sort(dv.begin(), dv.end(), by_key);
    else std::sort(dv.begin(), dv.end(), by_key);
  }
  vector<int> out;
  for (auto it = dv.begin(); it != dv.end(); ++it) {
    if (feasible_node(o, o.tree[it->first], s)) {
      out.push_back(it->first);
      if (keys_out) keys_out->push_back(it->second);
    }
    if ((int)out.size() == o.p.sort_limit) break;
  }
  return out;
}

static bool feasible_goal_bias(Oracle& o, const Node& node) {  // :292-315 (cos for .y kept)
  const double* g = o.p.goal;
  double R1 = 4.77, R2 = R1 - 0.3;
  Pt cl, cr;
  cl.x = g[0] + R1 * lm_cos(g[2] - M_PI_2);
  cl.y = g[1] + R1 * lm_cos(g[2] - M_PI_2);
  cr.x = g[0] + R1 * lm_cos(g[2] + M_PI_2);
  cr.y = g[1] + R1 * lm_cos(g[2] + M_PI_2);
  bool outL = sqrt(pow(node.state[0] - cl.x, 2) + pow(node.state[1] - cl.y, 2)) > R2;
  bool outR = sqrt(pow(node.state[0] - cr.x, 2) + pow(node.state[1] - cr.y, 2)) > R2;
  double aRef = atan2(g[1] - node.ref.y.back(), g[0] - node.ref.x.back());
  double h1 = std::abs(wrap_pi(g[2] - aRef));
  double h2 = std::abs(wrap_pi(g[2] + M_PI - aRef));
  double mn = std::min(h1, h2);
  double sg = sgn(lm_cos(g[2] + M_PI_2 - aRef));
  double ang = sg * mn;
  bool within = std::abs(ang) < (M_PI_4 / 2);
  return outL * outR * within;
}

// Result of one expandTree iteration evaluated against the first `upto` tree nodes.
struct IterResult {
  bool added = false, gb_added = false;
  Node node, gb_node;
  // the longest rollout chain the result depends on, in simulated steps: every candidate tried (a failed
  // one: its steps; the accepted one: its steps + the goal-biased rollout's, when that ran) -- the BATCH
  // engine's deferred-sample rule (defer_steps) commits the sample ceil(chain / T) - 1 rounds late
  long chain = 0;
};

static IterResult evaluate_iteration(Oracle& o, const Pt& s, bool explore, size_t upto, bool stable = false) {
  IterResult res;
  vector<int> cand = sort_nodes(o, s, explore, upto, nullptr, stable);
  for (int id : cand) {
    Ref r = get_reference(o, s, o.tree[id], 1);
    Sim sim = simulate(o, o.tree[id].state, r, false, o.tree[id].ref.v.back());
    res.chain = std::max(res.chain, (long)sim.rows.size() - 1);
    if (sim.endReached || sim.goalReached) {
      Node n;
      n.state = sim.rows.back(); n.parentID = id; n.ref = r; n.tra = sim.rows;
      n.costE = sim.costE + o.tree[id].costE;
      n.costS = sim.costS + o.tree[id].costS;
      n.goalReached = sim.goalReached;
      res.node = n; res.added = true;
      break;
    }
  }
  if (res.added && feasible_goal_bias(o, res.node)) {  // :163-173 on tree.back() == the new node
    vector<double> g(o.p.goal, o.p.goal + 4);
    Ref rg = get_goal_reference(o, res.node, g);
    Sim sg = simulate(o, res.node.state, rg, true, res.node.ref.v.back());
    res.chain = std::max(res.chain, (long)(res.node.tra.size() - 1) + (long)(sg.rows.size() - 1));
    if (sg.endReached || sg.goalReached) {
      Node n;
      n.state = sg.rows.back(); n.parentID = -2 /* set at append */; n.ref = rg; n.tra = sg.rows;
      n.costE = sg.costE + res.node.costE;
      n.costS = sg.costS + res.node.costS;
      n.goalReached = sg.goalReached;
      res.gb_node = n; res.gb_added = true;
    }
  }
  return res;
}

static void append_result(Oracle& o, IterResult& r) {
  if (!r.added) return;
  o.tree.push_back(r.node);
  if (r.gb_added) {
    r.gb_node.parentID = (int)o.tree.size() - 1;
    o.tree.push_back(r.gb_node);
  }
}

// expandTree :123-174 (one iteration, 3 rand() draws)
static void expand_tree(Oracle& o) {
  Pt s = sample_around(o);
  double r = static_cast<double>(rand()) / (static_cast<double>(RAND_MAX / (1)));
  bool explore = r <= ((false * 0.3) + (!false * 0.7));  // RRT.goalReached is never set
  IterResult res = evaluate_iteration(o, s, explore, o.tree.size());
  append_result(o, res);
}

// addInitialNode :21-37
static void add_initial_node(Oracle& o, const vector<double>& state) {
  Ref r;
  double xend = 1, yend = 0, res = 0.1;
  int N = floor(sqrt(pow(xend, 2) + pow(yend, 2)) / res);
  r.x = linspace(0, xend, N);
  r.y = linspace(0, yend, N);
  for (int i = 0; i != N; i++) r.v.push_back(state[4]);
  r.dir = 1;
  Node n;
  n.state = state; n.parentID = -1; n.ref = r; n.tra.push_back(state);
  n.costE = 0; n.costS = 0; n.goalReached = false;
  o.tree.push_back(n);
}

// ---------------------------------------------------------------- tree re-initialisation
// transformPointWorldToCar / CarToWorld transformations.cpp:6-17 (sin and cos of one argument in
// one function: a single sincos call, as for transformToVehicle).
static void point_world_to_car(double& Xw, double& Yw, const double* P) {
  double s, c;
  lm_sincos(P[2], &s, &c);
  double Xc = Xw * c - P[0] * c - P[1] * s + Yw * s;
  double Yc = Yw * c - P[1] * c + P[0] * s - Xw * s;
  Xw = Xc; Yw = Yc;
}
static void point_car_to_world(double& Xc, double& Yc, const double* P) {
  double s, c;
  lm_sincos(P[2], &s, &c);
  double Xw = c * Xc - s * Yc + P[0];
  double Yw = s * Xc + c * Yc + P[1];
  Xc = Xw; Yc = Yw;
}

// transformNodesWorldToCar / CarToworld transformations.cpp:289-315: node state (x, y, heading),
// every reference point, and the (x, y) of every trajectory row (row headings are left alone).
static void transform_nodes(vector<Node>& nodes, int to_world, const double* P) {
  for (auto& n : nodes) {
    if (to_world) { point_car_to_world(n.state[0], n.state[1], P); n.state[2] += P[2]; }
    else { point_world_to_car(n.state[0], n.state[1], P); n.state[2] -= P[2]; }
    for (size_t i = 0; i != n.ref.x.size(); i++)
      to_world ? point_car_to_world(n.ref.x[i], n.ref.y[i], P) : point_world_to_car(n.ref.x[i], n.ref.y[i], P);
    for (size_t j = 0; j != n.tra.size(); j++)
      to_world ? point_car_to_world(n.tra[j][0], n.tra[j][1], P) : point_world_to_car(n.tra[j][0], n.tra[j][1], P);
  }
}

// getNodeCost rrtplanner.cpp:104-119 (checkObsDistance of the row, the commented-out form at :108,
// under the context's collision mode; d2L :97-101 is getDistToLane's formula).
static double node_cost(Oracle& o, const double& parentCost, const Node& node) {
  double cost = parentCost;
  for (auto it = node.tra.begin(); it != node.tra.end(); it++) {
    double Dobs = obs_distance(o, *it);
    double kappa = lm_tan((*it)[3]) / o.p.veh.L;
    cost += o.p.Wcost[0] * (*it)[4] * o.p.sim_dt + o.p.Wcost[1] * std::abs(kappa) +
            o.p.Wcost[2] * exp(-o.p.Wcost[3] * Dobs);
    if (o.p.bend) cost += o.p.Wcost[4] * dist_to_lane((*it)[0], (*it)[1], o.p.lane_shift0, o.p.Cxy);
  }
  return cost;
}

// initializeTree rrtplanner.cpp:39-95 into a fresh tree (MyRRT is constructed per query,
// motionplanner.cpp:23).  Returns CLRRT_REINIT_*:
//   EMPTY      no committed nodes -> addInitialNode(carState)                          (:43-48)
//   ALL_ERASED every node erased (x of its last row < 0); the reference then reads
//              nodes.front() of an empty vector (:90, undefined) -- taken as an empty tree
//   COLLISION  a committed row collides -> empty tree (goto makeEmptyTree, :72-81)
//   KEPT       the surviving nodes as a chain (parent i-1), goal flags and costS recomputed
static int initialize_tree(Oracle& o, vector<Node>& nodes, vector<double> carState) {
  carState.push_back(0); carState.push_back(0); carState.push_back(0); carState.push_back(0);
  o.tree.clear();
  if (nodes.size() == 0) { add_initial_node(o, carState); return CLRRT_REINIT_EMPTY; }
  // :51-57 -- erase(it--) revisits the element moved into the erased slot, i.e. a filter
  vector<Node> kept;
  for (auto& n : nodes) {
    n.goalReached = 0;
    if (!((n.tra.back()[0]) < 0)) kept.push_back(n);
  }
  nodes.swap(kept);
  if (nodes.size() == 0) { add_initial_node(o, carState); return CLRRT_REINIT_ALL_ERASED; }
  // :60-69 (Dgoal uses the row's y, not y - goal y)
  for (auto& n : nodes)
    for (size_t i = 0; i != n.tra.size(); i++) {
      double Dgoal = sqrt(pow(n.tra[i][0] - o.p.goal[0], 2) + pow(n.tra[i][1], 2));
      double Hgoal = std::abs(n.tra[i][2] - o.p.goal[2]);
      double dVgoal = std::abs(n.tra[i][4] - o.p.goal[3]);
      if ((Dgoal <= 1) && (Hgoal <= 0.05) && (dVgoal <= 0.1)) n.goalReached = 1;
    }
  // :72-81
  for (auto& n : nodes)
    for (size_t i = 0; i != n.tra.size(); i++)
      if (obs_distance(o, n.tra[i]) == 0) { add_initial_node(o, carState); return CLRRT_REINIT_COLLISION; }
  // :84-87 (costS is a float; the parent's value is read back through a double)
  nodes.front().costS = node_cost(o, 0, nodes.front());
  for (size_t i = 1; i != nodes.size(); i++) nodes[i].costS = node_cost(o, nodes[i - 1].costS, nodes[i]);
  // :90-93
  for (size_t i = 0; i != nodes.size(); i++) {
    nodes[i].parentID = (int)i - 1;
    o.tree.push_back(nodes[i]);
  }
  return CLRRT_REINIT_KEPT;
}

}  // namespace orc

// ============================================================================ C API (ctypes)
using namespace orc;

extern "C" {

void* orc_create(const clrrt_params* p) {
  Oracle* o = new Oracle();
  o->p = *p;
  return o;
}
void orc_destroy(void* h) { delete (Oracle*)h; }
void orc_srand(unsigned seed) { srand(seed); }
int orc_rand(void) { return rand(); }

void orc_set_params(void* h, const clrrt_params* p) { ((Oracle*)h)->p = *p; }

void orc_set_obstacles(void* h, const double* obs7, int m) {
  Oracle* o = (Oracle*)h;
  o->det.clear();
  for (int i = 0; i < m; i++) {
    const double* d = obs7 + 7 * i;
    o->det.push_back(Obs{d[0], d[1], d[2], d[3], d[4], d[5], d[6]});
  }
}

void orc_init_tree(void* h, const double* root10) {
  Oracle* o = (Oracle*)h;
  o->tree.clear();
  add_initial_node(*o, std::vector<double>(root10, root10 + 10));
}

void orc_expand(void* h, long n_iters) {
  Oracle* o = (Oracle*)h;
  for (long i = 0; i < n_iters; i++) expand_tree(*o);
}

// Budgeted loop (motionplanner.cpp:39-43).  clock_kind 0 = CPU time (the reference's Timer),
// 1 = wall time (steady_clock).  Returns the number of iterations performed.
long orc_expand_budget(void* h, double budget_ms, int clock_kind) {
  Oracle* o = (Oracle*)h;
  long it = 0;
  if (clock_kind == 0) {
    clock_t t0 = clock();
    for (;; it++) {
      double ms = (double)(clock() - t0) / (CLOCKS_PER_SEC / 1000);
      if (!(ms < budget_ms)) break;
      expand_tree(*o);
    }
  } else {
    auto t0 = std::chrono::steady_clock::now();
    for (;; it++) {
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (!(ms < budget_ms)) break;
      expand_tree(*o);
    }
  }
  return it;
}

// BATCH mode restatement: rounds of B iterations; every sample of a round sees only the tree
// as it was at the start of the round; results are appended in sample order; equal keys are
// ordered by node id (stable = 1, the GPU engine's BATCH semantics) or as std::sort (stable = 0).
void orc_expand_batch(void* h, long n_iters, int B, int stable) {
  Oracle* o = (Oracle*)h;
  long done = 0;
  while (done < n_iters) {
    int nb = (int)std::min<long>(B, n_iters - done);
    std::vector<Pt> ss(nb);
    std::vector<char> ex(nb);
    for (int j = 0; j < nb; j++) {
      ss[j] = sample_around(*o);
      double r = static_cast<double>(rand()) / (static_cast<double>(RAND_MAX / (1)));
      ex[j] = r <= 0.7;
    }
    size_t upto = o->tree.size();
    std::vector<IterResult> rs(nb);
    for (int j = 0; j < nb; j++) rs[j] = evaluate_iteration(*o, ss[j], ex[j], upto, stable != 0);
    for (int j = 0; j < nb; j++) append_result(*o, rs[j]);
    done += nb;
  }
}

// BATCH mode with deferred samples (the engine's option "defer_steps" T, clrrt_kernels.hip Carry): every
// sample is evaluated against the tree as it was at the start of its own round, exactly as above, but it is
// appended by the commit of round r + D, D = ceil(chain / T) - 1 (its longest rollout chain, IterResult::chain,
// runs T steps per round's launch); a commit appends the samples of earlier rounds that come due (oldest
// round first, each round's in sample order), then the round's own samples with D = 0; after the last round
// every sample still pending is appended in the same order.  T = 0: plain BATCH rounds.
void orc_expand_batch_defer(void* h, long n_iters, int B, int stable, int T, long* deferred) {
  Oracle* o = (Oracle*)h;
  struct Pend { long due; IterResult r; };
  std::vector<Pend> pend;  // (origin round, sample) order
  long done = 0, round = 0, ndef = 0;
  while (done < n_iters) {
    int nb = (int)std::min<long>(B, n_iters - done);
    std::vector<Pt> ss(nb);
    std::vector<char> ex(nb);
    for (int j = 0; j < nb; j++) {
      ss[j] = sample_around(*o);
      double r = static_cast<double>(rand()) / (static_cast<double>(RAND_MAX / (1)));
      ex[j] = r <= 0.7;
    }
    size_t upto = o->tree.size();
    std::vector<IterResult> rs(nb);
    for (int j = 0; j < nb; j++) rs[j] = evaluate_iteration(*o, ss[j], ex[j], upto, stable != 0);
    std::vector<Pend> keep;
    for (auto& p : pend) {
      if (p.due == round) append_result(*o, p.r);
      else keep.push_back(std::move(p));
    }
    for (int j = 0; j < nb; j++) {
      const long D = (T > 0 && rs[j].chain > 0) ? (rs[j].chain + T - 1) / T - 1 : 0;
      if (D == 0) {
        append_result(*o, rs[j]);
      } else {
        keep.push_back(Pend{round + D, std::move(rs[j])});
        ndef++;
      }
    }
    pend.swap(keep);
    done += nb;
    round++;
  }
  for (auto& p : pend) append_result(*o, p.r);
  if (deferred) *deferred = ndef;
}

// orc_expand_batch_defer with each round's samples evaluated on `threads` host threads (the frozen tree is
// only read; counters are atomic; results are appended in the same order), so that whole trees at the
// benchmarked sizes (16384 samples per round) can be checked.  Test infrastructure.
void orc_expand_batch_defer_mt(void* h, long n_iters, int B, int stable, int T, int threads, long* deferred) {
  Oracle* o = (Oracle*)h;
  struct Pend { long due; IterResult r; };
  std::vector<Pend> pend;
  long done = 0, round = 0, ndef = 0;
  const bool by_ref = o->keys_by_ref;
  o->keys_by_ref = true;
  while (done < n_iters) {
    int nb = (int)std::min<long>(B, n_iters - done);
    std::vector<Pt> ss(nb);
    std::vector<char> ex(nb);
    for (int j = 0; j < nb; j++) {
      ss[j] = sample_around(*o);
      double r = static_cast<double>(rand()) / (static_cast<double>(RAND_MAX / (1)));
      ex[j] = r <= 0.7;
    }
    const size_t upto = o->tree.size();
    cache_rotations(*o);
    std::vector<IterResult> rs(nb);
    std::atomic<int> next{0};
    std::vector<std::thread> pool;
    const int nt = std::max(1, std::min(threads, nb));
    for (int t = 0; t < nt; t++)
      pool.emplace_back([&]() {
        for (int j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nb;)
          rs[j] = evaluate_iteration(*o, ss[j], ex[j], upto, stable != 0);
      });
    for (auto& th : pool) th.join();
    std::vector<Pend> keep;
    for (auto& p : pend) {
      if (p.due == round) append_result(*o, p.r);
      else keep.push_back(std::move(p));
    }
    for (int j = 0; j < nb; j++) {
      const long D = (T > 0 && rs[j].chain > 0) ? (rs[j].chain + T - 1) / T - 1 : 0;
      if (D == 0) {
        append_result(*o, rs[j]);
      } else {
        keep.push_back(Pend{round + D, std::move(rs[j])});
        ndef++;
      }
    }
    pend.swap(keep);
    done += nb;
    round++;
  }
  for (auto& p : pend) append_result(*o, p.r);
  o->keys_by_ref = by_ref;
  o->rot.clear();
  if (deferred) *deferred = ndef;
}

long orc_tree_size(void* h) { return (long)((Oracle*)h)->tree.size(); }

// Export node headers in the clrrt_node layout.
void orc_get_nodes(void* h, long first, long count, clrrt_node* out) {
  Oracle* o = (Oracle*)h;
  for (long k = 0; k < count; k++) {
    const Node& n = o->tree[first + k];
    clrrt_node& d = out[k];
    memset(&d, 0, sizeof(d));
    for (int i = 0; i < 10; i++) d.state[i] = at0(n.state, i);
    d.ref_front[0] = n.ref.x.front(); d.ref_front[1] = n.ref.y.front();
    d.ref_back[0] = n.ref.x.back(); d.ref_back[1] = n.ref.y.back();
    d.ref_vback = n.ref.v.back();
    d.ang_par = atan2(n.ref.y.back() - n.ref.y.front(), n.ref.x.back() - n.ref.x.front());
    d.parent = n.parentID;
    d.costE = n.costE; d.costS = n.costS;
    d.goal = n.goalReached;
    d.nrows = (int)n.tra.size();
    d.owner = 0; d.row_offset = 0;
  }
}

long orc_node_ref_len(void* h, long i) { return (long)((Oracle*)h)->tree[i].ref.x.size(); }

void orc_get_ref(void* h, long i, double* x, double* y, double* v) {
  const Node& n = ((Oracle*)h)->tree[i];
  for (size_t k = 0; k < n.ref.x.size(); k++) {
    x[k] = n.ref.x[k]; y[k] = n.ref.y[k]; v[k] = at0(n.ref.v, (long)k);
  }
}

void orc_get_rows(void* h, long i, double* out) {
  const Node& n = ((Oracle*)h)->tree[i];
  for (size_t r = 0; r < n.tra.size(); r++)
    for (int c = 0; c < 10; c++) out[r * 10 + c] = at0(n.tra[r], c);
}

void orc_counters(void* h, long* out5) {
  Oracle* o = (Oracle*)h;
  out5[0] = o->sim_count; out5[1] = o->fail_collision; out5[2] = o->fail_acclimit;
  out5[3] = o->fail_iterlimit; out5[4] = o->rollouts;
}
void orc_reset_counters(void* h) {
  Oracle* o = (Oracle*)h;
  o->sim_count = o->fail_collision = o->fail_acclimit = o->fail_iterlimit = o->rollouts = 0;
}

// Load a tree from node headers (refs rebuilt as 2-point references carrying front/back/vback —
// all the expansion reads from a node's ref).  Trajectories are 1 row (the node state).
void orc_load_tree(void* h, const clrrt_node* nodes, long n) {
  Oracle* o = (Oracle*)h;
  o->tree.clear();
  for (long k = 0; k < n; k++) {
    const clrrt_node& d = nodes[k];
    Node nd;
    nd.state.assign(d.state, d.state + 10);
    nd.parentID = d.parent;
    nd.ref.x = {d.ref_front[0], d.ref_back[0]};
    nd.ref.y = {d.ref_front[1], d.ref_back[1]};
    nd.ref.v = {d.ref_vback, d.ref_vback};
    nd.costE = d.costE; nd.costS = d.costS; nd.goalReached = d.goal;
    nd.tra.push_back(nd.state);
    o->tree.push_back(nd);
  }
}

// One Simulation from tree node `parent` (gb=0: toward sample; gb=1: goal-biased).
// rows_out may be null; returns the number of rows.
int orc_simulate(void* h, int parent, int gb, double sx, double sy, int* outcome, double* costs2,
                 double* final10, double* ref_back3, int* ref_n, double* rows_out, int rows_cap) {
  Oracle* o = (Oracle*)h;
  Node par = o->tree[parent];
  Ref r;
  if (gb) {
    std::vector<double> g(o->p.goal, o->p.goal + 4);
    r = get_goal_reference(*o, par, g);
  } else {
    Pt s; s.x = sx; s.y = sy;
    r = get_reference(*o, s, par, 1);
  }
  Sim sim = simulate(*o, par.state, r, gb != 0, par.ref.v.back());
  *outcome = sim.outcome;
  costs2[0] = sim.costE; costs2[1] = sim.costS;
  for (int i = 0; i < 10; i++) final10[i] = at0(sim.rows.back(), i);
  ref_back3[0] = r.x.back(); ref_back3[1] = r.y.back(); ref_back3[2] = r.v.back();
  *ref_n = (int)r.x.size();
  if (rows_out) {
    for (size_t k = 0; k < sim.rows.size() && (int)k < rows_cap; k++)
      for (int c = 0; c < 10; c++) rows_out[k * 10 + c] = at0(sim.rows[k], c);
  }
  return (int)sim.rows.size();
}

int orc_feasible_goal_bias(void* h, long node) {
  Oracle* o = (Oracle*)h;
  return feasible_goal_bias(*o, o->tree[node]) ? 1 : 0;
}

// Candidate list of the nearest-node search (ids + keys), count returned.
int orc_sort_nodes(void* h, double sx, double sy, int explore, int stable, int* ids, float* keys) {
  Oracle* o = (Oracle*)h;
  Pt s; s.x = sx; s.y = sy;
  std::vector<float> k;
  std::vector<int> c = sort_nodes(*o, s, explore != 0, o->tree.size(), &k, stable != 0);
  for (size_t i = 0; i < c.size(); i++) { ids[i] = c[i]; keys[i] = k[i]; }
  return (int)c.size();
}

float orc_dubins(void* h, double sx, double sy, long node) {
  Oracle* o = (Oracle*)h;
  Pt s; s.x = sx; s.y = sy;
  return dubins(s, o->tree[node], 1);
}

// getOBBdist known-answer hook: boxes given as (px, py, w, h, o) with float w/h/o.
double orc_obb_dist(double apx, double apy, float aw, float ah, float ao, double bpx, double bpy,
                    float bw, float bh, float bo) {
  Box a(apx, apy, aw, ah, ao), b(bpx, bpy, bw, bh, bo);
  return box_gap(a, b);
}

double orc_check_obs(void* h, const double* x10) {
  Oracle* o = (Oracle*)h;
  std::vector<double> x(x10, x10 + 10);
  return obs_distance(*o, x);
}

// Draw `n` iterations' samples from glibc rand() in the reference order (rLong, rLat, r).
void orc_draw_samples(void* h, int n, double* xy, int* explore) {
  Oracle* o = (Oracle*)h;
  for (int j = 0; j < n; j++) {
    Pt s = sample_around(*o);
    double r = static_cast<double>(rand()) / (static_cast<double>(RAND_MAX / (1)));
    xy[2 * j] = s.x; xy[2 * j + 1] = s.y;
    explore[j] = r <= 0.7;
  }
}

// Evaluate one iteration for a given sample against the whole tree without appending.
// Returns the number of nodes it would append (0..2); fills headers (parent of the GB node = -2).
int orc_eval_iteration(void* h, double sx, double sy, int explore, int stable, clrrt_node* out2) {
  Oracle* o = (Oracle*)h;
  Pt s; s.x = sx; s.y = sy;
  IterResult r = evaluate_iteration(*o, s, explore != 0, o->tree.size(), stable != 0);
  int n = 0;
  Oracle tmp;
  if (r.added) { tmp.tree.push_back(r.node); n++; }
  if (r.gb_added) { tmp.tree.push_back(r.gb_node); n++; }
  if (n) orc_get_nodes(&tmp, 0, n, out2);
  return n;
}


// n independent eval_iteration calls against the same frozen tree on `threads` host threads (the
// tree is only read; the counters are updated atomically).  out: 2 records per sample, counts[k] of
// them valid.  Test infrastructure for bench-size trees, where one call sorts millions of keys.
void orc_eval_iterations(void* h, int n, const double* sx, const double* sy, const int* explore, int stable,
                         int threads, clrrt_node* out, int* counts) {
  std::vector<std::thread> pool;
  const int T = std::max(1, std::min(threads, n));
  for (int t = 0; t < T; t++)
    pool.emplace_back([=]() {
      for (int k = t; k < n; k += T) counts[k] = orc_eval_iteration(h, sx[k], sy[k], explore[k], stable, out + 2 * k);
    });
  for (auto& th : pool) th.join();
}

// orc_eval_iterations against the first `upto` nodes of the loaded tree (the frozen tree of an earlier round inside
// a larger one), keys from cached rotations (the stable order), with each sample's deciding chain in steps
// (IterResult::chain: the engine's deferred-sample rule commits it ceil(chain / T) - 1 rounds late).  Test
// infrastructure (tests/test_full_size_parity.py, late-query deferred rounds).
void orc_eval_iterations_upto(void* h, int n, const double* sx, const double* sy, const int* explore, int stable,
                              int threads, long upto, clrrt_node* out, int* counts, long* chains) {
  Oracle* o = (Oracle*)h;
  const bool by_ref = o->keys_by_ref;
  o->keys_by_ref = true;
  cache_rotations(*o);
  const size_t up = std::min<size_t>((size_t)std::max(0L, upto), o->tree.size());
  std::vector<std::thread> pool;
  const int T = std::max(1, std::min(threads, n));
  for (int t = 0; t < T; t++)
    pool.emplace_back([=]() {
      for (int k = t; k < n; k += T) {
        Pt s;
        s.x = sx[k];
        s.y = sy[k];
        IterResult r = evaluate_iteration(*o, s, explore[k] != 0, up, stable != 0);
        int m = 0;
        Oracle tmp;
        if (r.added) { tmp.tree.push_back(r.node); m++; }
        if (r.gb_added) { tmp.tree.push_back(r.gb_node); m++; }
        if (m) orc_get_nodes(&tmp, 0, m, out + 2 * k);
        counts[k] = m;
        chains[k] = r.chain;
      }
    });
  for (auto& th : pool) th.join();
  o->keys_by_ref = by_ref;
}

// ---- unit hooks (tests/test_ref_units.py): the same functions the tree path runs, one case per row.
// OBB gap of the vehicle box at (x, y, th) against one obstacle at time t.
// in: x, y, th, t, cx, cy, oth, size_x, size_y, vx, vy (11 doubles per case).
void orc_unit_obb(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 11 * k;
    Row x(10, 0.0);
    x[0] = a[0]; x[1] = a[1]; x[2] = a[2]; x[6] = a[3];
    Obs d{a[4], a[5], a[6], a[7], a[8], a[9], a[10]};
    out[k] = box_gap(veh_box(x), obs_box(d, a[3]));
  }
}
// OBB geometry (px, py, w, h, o) -> vertices x4, y4, normals x4, y4 (floats, axis 3 canonical).
void orc_unit_obb_geom(int n, const double* in, float* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 5 * k;
    Box b(a[0], a[1], (float)a[2], (float)a[3], (float)a[4]);
    float* o = out + 16 * k;
    for (int i = 0; i < 4; i++) { o[i] = b.vx[i]; o[4 + i] = b.vy[i]; o[8 + i] = b.nx[i]; o[12 + i] = b.ny[i]; }
  }
}
// VehicleODE + IntegrateEuler. in: x0..x6, dc, ac; out: x0..x6, dx[2].
void orc_unit_ode(void* h, int n, const double* in, double* out) {
  Oracle* o = (Oracle*)h;
  for (int k = 0; k < n; k++) {
    Row x(in + 9 * k, in + 9 * k + 7);
    x.resize(10, 0.0);
    double dx[7];
    ode_euler(*o, x, in[9 * k + 7], in[9 * k + 8], dx);
    for (int i = 0; i < 7; i++) out[8 * k + i] = x[i];
    out[8 * k + 7] = dx[2];
  }
}
// transformToVehicle + interpolate. in: xval[3], yval[3], X[3].
void orc_unit_lateral(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 9 * k;
    out[k] = transform_interp(a, a + 3, a[6], a[7], a[8]);
  }
}
void orc_unit_linspace(double a, double b, long N, double* out) {
  vector<double> v = linspace(a, b, (size_t)N);
  for (long i = 0; i < N; i++) out[i] = v[i];
}
// getReference's straight line from (ax, ay) to (sx, sy) at resolution res, then its velocity profile.
// in: ax, ay, sx, sy, res, v0, vmax, goal[4], GB (12 doubles); out row (stride 1 + nmax): N, v[0..N).
void orc_unit_profile(void* h, int n, const double* in, int nmax, double* out) {
  Oracle o = *(Oracle*)h;
  for (int k = 0; k < n; k++) {
    const double* a = in + 12 * k;
    o.p.ref_res = a[4];
    Node par;
    par.ref.x.assign(1, a[0]);
    par.ref.y.assign(1, a[1]);
    Pt s; s.x = a[2]; s.y = a[3];
    Ref r = get_reference(o, s, par, 1);
    vector<double> g(a + 7, a + 11);
    velocity_profile(o, r, a[5], a[6], g, a[11] != 0);
    double* row = out + (size_t)(1 + nmax) * k;
    row[0] = (double)r.v.size();
    for (size_t i = 0; i < r.v.size() && (int)i < nmax; i++) row[1 + i] = r.v[i];
  }
}
// angleDiff(a, b), wrapToPi(a)
void orc_unit_angle(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    out[2 * k] = angle_diff(in[2 * k], in[2 * k + 1]);
    out[2 * k + 1] = wrap_pi(in[2 * k]);
  }
}
// dubinsDistance (explore key) and costE + dubinsDistance (optimize key).
// in: sx, sy, node x, y, heading, costE.
void orc_unit_dubins(int n, const double* in, double* out) {
  for (int k = 0; k < n; k++) {
    const double* a = in + 6 * k;
    Pt s; s.x = a[0]; s.y = a[1];
    Node nd;
    nd.state.assign(10, 0.0);
    nd.state[0] = a[2]; nd.state[1] = a[3]; nd.state[2] = a[4];
    nd.costE = (float)a[5];
    const float key = dubins(s, nd, 1);
    out[2 * k] = key;
    out[2 * k + 1] = (float)(nd.costE + key);
  }
}
// feasibleNode.  in: sx, sy, ref front x, y, ref back x, y, ref_res.
void orc_unit_feasible(void* h, int n, const double* in, double* out) {
  Oracle o = *(Oracle*)h;
  for (int k = 0; k < n; k++) {
    const double* a = in + 7 * k;
    o.p.ref_res = a[6];
    Pt s; s.x = a[0]; s.y = a[1];
    Node nd;
    nd.ref.x = {a[2], a[4]};
    nd.ref.y = {a[3], a[5]};
    out[k] = feasible_node(o, nd, s) ? 1.0 : 0.0;
  }
}
// feasibleGoalBias of a new node.  in: goal[4], node x, y, ref back x, y.
void orc_unit_goal_bias(void* h, int n, const double* in, double* out) {
  Oracle o = *(Oracle*)h;
  for (int k = 0; k < n; k++) {
    const double* a = in + 8 * k;
    for (int i = 0; i < 4; i++) o.p.goal[i] = a[i];
    Node nd;
    nd.state.assign(10, 0.0);
    nd.state[0] = a[4]; nd.state[1] = a[5];
    nd.ref.x = {a[6]};
    nd.ref.y = {a[7]};
    out[k] = feasible_goal_bias(o, nd) ? 1.0 : 0.0;
  }
}
// getGoalReference + the goal-biased velocity profile.  in: goal[4], parent ref back x, y, v0, ref_res;
// out row (1 + 3 nmax): N, v, x, y.
void orc_unit_goal_ref(void* h, int n, const double* in, int nmax, double* out) {
  Oracle o = *(Oracle*)h;
  for (int k = 0; k < n; k++) {
    const double* a = in + 8 * k;
    vector<double> g(a, a + 4);
    for (int i = 0; i < 4; i++) o.p.goal[i] = a[i];
    o.p.ref_res = a[7];
    Node par;
    par.ref.x = {a[4]};
    par.ref.y = {a[5]};
    Ref r = get_goal_reference(o, par, g);
    velocity_profile(o, r, a[6], o.p.vmax, g, true);
    double* row = out + (size_t)(1 + 3 * nmax) * k;
    row[0] = (double)r.x.size();
    for (size_t i = 0; i < r.x.size() && (int)i < nmax; i++) {
      row[1 + i] = at0(r.v, (long)i);
      row[1 + nmax + i] = r.x[i];
      row[1 + 2 * nmax + i] = r.y[i];
    }
  }
}
// The Controller of a Simulation over a state sequence (CLRRT_UNIT_CTRL layout, include/clrrt.h).
void orc_unit_ctrl(void* h, int n, const double* in, int K, double* out) {
  Oracle o = *(Oracle*)h;
  for (int k = 0; k < n; k++) {
    const double* a = in + (size_t)(12 + 6 * K) * k;
    double* w = out + (size_t)(4 + 8 * K) * k;
    for (int i = 0; i < 4; i++) o.p.goal[i] = a[5 + i];
    o.p.vmax = a[10];
    o.p.ref_res = a[11];
    vector<double> g(a + 5, a + 9);
    const bool GB = a[0] != 0;
    Node par;
    par.ref.x = {a[1]};
    par.ref.y = {a[2]};
    Ref r;
    if (GB) {
      r = get_goal_reference(o, par, g);
    } else {
      Pt s; s.x = a[3]; s.y = a[4];
      r = get_reference(o, s, par, 1);
    }
    const double* st = a + 12;
    Row x0(st, st + 6);
    x0.resize(10, 0.0);
    Ctrl c(o, r, x0);
    w[0] = c.IDwp; w[1] = c.endreached; w[2] = c.P.x; w[3] = c.P.y;
    velocity_profile(o, r, a[9], o.p.vmax, g, GB);
    for (int j = 0; j < K; j++) {
      Row x(st + 6 * j, st + 6 * j + 6);
      x.resize(10, 0.0);
      c.update_waypoint(o, r, x);
      const double dc = c.steer(o, r, x);
      const double ac = c.accel(o, r, x);
      double* q = w + 4 + 8 * j;
      q[0] = c.IDwp; q[1] = c.endreached; q[2] = c.P.x; q[3] = c.P.y;
      q[4] = c.ym; q[5] = dc; q[6] = ac; q[7] = c.iE;
    }
  }
}

}  // extern "C"

// extractBestPath rrtplanner.cpp:318-368: goal nodes as (id, costS) pairs in tree order, std::sort
// ascending by cost (the reference's lambda; not stable), the front's ancestors by backtracking.
// Writes the path root -> goal into ids (at most cap) and returns its length (0: no solution).
extern "C" int orc_extract_best_path(void* h, int* ids, int cap) {
  Oracle* o = (Oracle*)h;
  vector<pair<int, double>> pv;
  for (int nodeid = 0; nodeid != (int)o->tree.size(); nodeid++)
    if (o->tree[nodeid].goalReached) pv.push_back(make_pair(nodeid, (double)o->tree[nodeid].costS));
  if (pv.empty()) return 0;
  sort(pv.begin(), pv.end(), [](const pair<int, double>& a, const pair<int, double>& b) { return a.second < b.second; });
  vector<int> path{pv.front().first};
  int parent = o->tree[pv.front().first].parentID;
  while (parent != -1) {
    path.insert(path.begin(), parent);
    parent = o->tree[parent].parentID;
  }
  int n = (int)path.size();
  for (int i = 0; i < n && i < cap; i++) ids[i] = path[i];
  return n;
}

// bestNodes = tree nodes `ids` (what extractBestPath returns, motionplanner.cpp:51).
extern "C" void orc_path_commit(void* h, const int* ids, int n) {
  Oracle* o = (Oracle*)h;
  o->best.clear();
  for (int i = 0; i < n; i++) o->best.push_back(o->tree[ids[i]]);
}
extern "C" long orc_path_size(void* h) { return (long)((Oracle*)h)->best.size(); }
// to_world 0: transformNodesWorldToCar (motionplanner.cpp:22); 1: transformNodesCarToworld (:54).
extern "C" void orc_path_transform(void* h, int to_world, const double* pose3) {
  orc::transform_nodes(((Oracle*)h)->best, to_world, pose3);
}
extern "C" void orc_path_get_nodes(void* h, clrrt_node* out) {
  Oracle tmp;
  tmp.tree = ((Oracle*)h)->best;
  if (!tmp.tree.empty()) orc_get_nodes(&tmp, 0, (long)tmp.tree.size(), out);
}
extern "C" void orc_path_get_rows(void* h, long i, double* out) {
  Oracle tmp;
  tmp.tree.push_back(((Oracle*)h)->best[i]);
  orc_get_rows(&tmp, 0, out);
}
// initializeTree(RRT, veh, bestNodes, carPose) with carPose = 6 doubles (x, y, theta, delta, v, a).
extern "C" int orc_initialize_tree(void* h, const double* car6) {
  Oracle* o = (Oracle*)h;
  return orc::initialize_tree(*o, o->best, vector<double>(car6, car6 + 6));
}

// convertNodesToPath motionplanner.cpp:264-275 + generateMPCmessage :103-128 (+ filterMPCmessage
// :130-151 when `filtered`) over bestNodes; the message's fields as in car_msgs::Trajectory.
// Points are written as 8 doubles (x, y, theta, delta, v, a, a_cmd, d_cmd; delta NaN when filtered,
// the reference leaves it out).  Returns the point count.  Empty messages stay empty (the
// reference's size()-1 loop and i = 1 loop are undefined there).
namespace orc {
struct Traj { vector<double> x, y, theta, delta, v, a, a_cmd, d_cmd; };
}
extern "C" int orc_path_mpc_message(void* h, int filtered, double* out, int cap) {
  using orc::Traj;
  Oracle* o = (Oracle*)h;
  Traj tra;
  for (auto it = o->best.begin(); it != o->best.end(); ++it)
    for (size_t i = 1; i < it->tra.size(); i++) {
      tra.x.push_back(it->tra[i][0]); tra.y.push_back(it->tra[i][1]); tra.theta.push_back(it->tra[i][2]);
      tra.delta.push_back(it->tra[i][3]); tra.v.push_back(it->tra[i][4]); tra.a.push_back(it->tra[i][5]);
      tra.a_cmd.push_back(it->tra[i][8]); tra.d_cmd.push_back(it->tra[i][9]);
    }
  if (filtered && !tra.x.empty()) {
    Traj f;
    double interval = 5;
    double d = 0;
    for (size_t i = 1; i != tra.x.size(); i++) {
      if (d == 0) {
        f.x.push_back(tra.x[i]); f.y.push_back(tra.y[i]); f.theta.push_back(tra.theta[i]);
        f.v.push_back(tra.v[i]); f.a.push_back(tra.a[i]); f.a_cmd.push_back(tra.a_cmd[i]);
        f.d_cmd.push_back(tra.d_cmd[i]);
      }
      d += sqrt(pow(tra.x[i] - tra.x[i - 1], 2) + pow(tra.y[i] - tra.y[i - 1], 2));
      if (d >= interval) d = 0;
    }
    tra = f;
  }
  int n = (int)tra.x.size();
  for (int i = 0; i < n && i < cap; i++) {
    double* p = out + 8 * i;
    p[0] = tra.x[i]; p[1] = tra.y[i]; p[2] = tra.theta[i];
    p[3] = filtered ? NAN : tra.delta[i];
    p[4] = tra.v[i]; p[5] = tra.a[i]; p[6] = tra.a_cmd[i]; p[7] = tra.d_cmd[i];
  }
  return n;
}
