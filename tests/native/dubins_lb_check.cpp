// Validates clrrt::dubins_lb <= the float Dubins key (restated as dubinsDistance computes it,
// rrtplanner.cpp:371-406, with glibc's float functions) on random points in the node frame.
// Prints the number of violations and the median slack; exit 1 on any violation.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include <algorithm>

#include "../../cl-rrt_amd/csrc/clrrt_dubins_lb.hpp"

static float key(float qx, float qy) {
  const float rho = 4.77f;
  qy = std::fabs(qy);
  float dc = std::sqrt(qx * qx + (qy - rho) * (qy - rho));
  float thc = std::atan2(qx, rho - qy);
  while (thc < 0) thc = (float)((double)thc + 2 * M_PI);
  float df = std::sqrt(qx * qx + (qy + rho) * (qy + rho));
  bool inside = (qx * qx + (qy + rho) * (qy + rho) <= rho * rho) | (qx * qx + (qy - rho) * (qy - rho) <= rho * rho);
  if (!inside) return std::sqrt(dc * dc - rho * rho) + rho * (thc - std::acos(rho / dc));
  float alpha = (float)(2 * M_PI - (double)std::acos((5 * rho * rho - df * df) / (4 * rho * rho)));
  return rho * (alpha + std::asin(qx / df) - std::asin(rho * std::sin(alpha) / df));
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<float> u(-30.f, 30.f), v(0.f, 30.f), small(-0.05f, 0.05f);
  long bad = 0;
  std::vector<float> slack;
  for (long i = 0; i < n; i++) {
    float qx, qy;
    switch (i % 4) {
      case 0: qx = u(g); qy = v(g); break;
      case 1: qx = u(g) / 10; qy = v(g) / 10; break;
      case 2: {  // near the turning circle boundary (ill-conditioned acos)
        float t = u(g) / 30 * 3.14159265f;
        float rr = 4.77f + small(g);
        qx = rr * std::sin(t); qy = std::fabs(4.77f - rr * std::cos(t));
      } break;
      default: qx = small(g) * 20; qy = v(g); break;
    }
    float k = key(qx, qy);
    float lb = clrrt::dubins_lb(qx, std::fabs(qy));
    if (std::isnan(k)) continue;  // NaN keys never enter a list
    if (lb > k) {
      if (bad < 10) printf("violation q=(%.9g, %.9g) key %.9g lb %.9g\n", qx, qy, k, lb);
      bad++;
    }
    if (i % 97 == 0) slack.push_back(k - lb);
  }
  std::sort(slack.begin(), slack.end());
  printf("points %ld violations %ld median slack %.4f p10 %.4f\n", n, bad, slack[slack.size() / 2],
         slack[slack.size() / 10]);
  return bad ? 1 : 0;
}
