// MotionPlanner::planMotion (motionplanner.cpp:8-77) end to end through include/clrrt_adapter.hpp's
// ROS-free MotionPlanner, linked against libclrrt (no Python): a sequence of 5 Hz queries whose inputs
// (world state, goal and detections in the car frame) come from tests/test_native_plan_motion.py, which
// runs the same sequence on the CPU oracle and compares what this program writes: the re-init outcome,
// iterations, tree size, committed path ids, the filtered MPC message bit for bit, and (draw_tree on)
// every node's goal flag and trajectory hash (the rviz marker data of extractBestPath :322-341).
// Usage: plan_motion <inputs.bin> <outputs.bin> <seed> <iters> [draw_tree]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "../../include/clrrt_adapter.hpp"

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

template <class T>
static void put(std::vector<char>& o, const T& v) {
  const char* b = (const char*)&v;
  o.insert(o.end(), b, b + sizeof(T));
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s inputs.bin outputs.bin seed iters [draw_tree]\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (buf.size() < 12 || memcmp(buf.data(), "CLPM", 4) != 0) { fprintf(stderr, "bad inputs\n"); return 2; }
  const char* p = buf.data() + 4;
  const int32_t mode_coll = take<int32_t>(p);
  const int32_t nq = take<int32_t>(p);
  const uint32_t seed = (uint32_t)atoi(argv[3]);
  const int64_t iters = atoll(argv[4]);
  const bool draw = argc > 5 && atoi(argv[5]) != 0;

  clrrt_adapter::MotionPlanner::Config cfg;
  const double goal0[4] = {0, 0, 0, 0};
  clrrt_params_default(&cfg.base, 0.0, goal0, 5.0);
  cfg.base.collision_mode = mode_coll;
  cfg.cap.max_nodes = 1 << 16;
  cfg.cap.max_rows = 1 << 21;
  cfg.cap.max_batch = 256;
  cfg.cap.max_obstacles = 256;
  cfg.commit_path = true;
  cfg.mode = CLRRT_MODE_EXACT;
  cfg.batch = 256;
  cfg.n_iters = iters;
  cfg.draw_tree = draw;
  std::vector<char> out;
  out.insert(out.end(), {'C', 'L', 'P', 'O'});
  put(out, nq);
  try {
    clrrt_adapter::MotionPlanner mp(cfg, seed);
    for (int q = 0; q < nq; q++) {
      std::vector<double> st(6);
      for (auto& v : st) v = take<double>(p);
      clrrt_adapter::MotionRequest req;
      for (auto& g : req.goal) g = take<double>(p);
      req.vmax = 5.0;
      const int32_t m = take<int32_t>(p);
      std::vector<clrrt_obstacle> det(m);
      for (auto& o : det) {
        o.cx = take<double>(p); o.cy = take<double>(p); o.theta = take<double>(p);
        o.size_x = take<double>(p); o.size_y = take<double>(p); o.vx = take<double>(p); o.vy = take<double>(p);
      }
      mp.updateState(st);
      mp.updateObstacles(det);
      clrrt_adapter::MPCTrajectory msg;
      clrrt_adapter::PlanReport rep;
      std::vector<clrrt_adapter::TreeMarker> markers;
      const bool found = mp.planMotion(req, &msg, &rep, &markers);
      put(out, (int32_t)found);
      put(out, rep.reinit_outcome);
      put(out, rep.iterations);
      put(out, rep.tree_size);
      put(out, (int32_t)rep.path.size());
      for (int32_t id : rep.path) put(out, id);
      put(out, (int32_t)msg.published);
      put(out, (int32_t)msg.x.size());
      for (size_t i = 0; i < msg.x.size(); i++) {
        put(out, msg.x[i]); put(out, msg.y[i]); put(out, msg.theta[i]); put(out, msg.v[i]);
        put(out, msg.a[i]); put(out, msg.a_cmd[i]); put(out, msg.d_cmd[i]);
      }
      for (int k = 0; k < 4; k++) put(out, rep.counters[k]);
      put(out, (int32_t)markers.size());
      for (const auto& mk : markers) {
        put(out, (int32_t)mk.goal);
        put(out, fnv1a(mk.rows.data(), mk.rows.size() * sizeof(double)));
      }
      printf("query %d: outcome %d, %lld iterations, tree %lld, path %zu, message %zu points%s, markers %zu\n", q,
             rep.reinit_outcome, (long long)rep.iterations, (long long)rep.tree_size, rep.path.size(), msg.x.size(),
             msg.published ? " (published)" : "", markers.size());
    }
  } catch (const std::exception& e) {
    printf("error: %s\n", e.what());
    return 1;
  }
  std::ofstream o(argv[2], std::ios::binary);
  o.write(out.data(), (std::streamsize)out.size());
  return o ? 0 : 1;
}
