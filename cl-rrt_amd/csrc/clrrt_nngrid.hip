// clrrt_nngrid.hip — spatial index for the nearest-node search (sortNodesExplore/Optimize,
// rrtplanner.cpp:227-268) of large trees.
//
// The reference sorts every node by its Dubins key (explore) or cost + Dubins key (optimize) and
// walks the sorted list for the first sortLimit feasible nodes.  The result is the sortLimit
// smallest (key, index) pairs among the feasible nodes (+ one more to reveal a boundary tie), which
// the brute-force kernels find by scanning all N nodes per sample.
//
// Index (rebuilt every round, counting sort): a uniform grid of cells of size cs, grouped in 8x8
// super-cells; cells are numbered super-cell-major so a super-cell's nodes are contiguous.  Per cell
// the minimum cost, per super-cell the minimum cost and the fixed-point bounds of its nodes'
// ref.back() points and ang_par values.
//
// Search (k_nn_tile): samples are bucketed by super-cell so that a wave holds spatially close
// samples; the wave walks rings of super-cells around its centre with WAVE-UNIFORM control flow and
// node loads (each lane keeps its own top-11 list), skipping a super-cell or cell when no lane can
// take a node from it:
//   key(node) >= |q| * (1 - 1e-5) - 1e-4          (Dubins length >= Euclidean, float rounding)
//   |q| >= distance from the sample to the cell rectangle;  optimize: + minimum cost of the cell
//   feasibleNode (rrtplanner.cpp:271-289) impossible: the directions from the box of the nodes'
//   ref.back() points to the sample stay more than pi/4 (+ margin) away from their ang_par arc.
// A skipped cell holds no pair that could enter the list, so each list equals the brute-force one
// bit for bit (ties included: pairs are ordered by (key, node index) in both).  A wave that has read
// more than `cap` nodes stops; its lanes whose search was not complete are handed to the chunked
// brute-force kernels, so no sample costs more than a brute-force search.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "clrrt_dev.hpp"
#include "clrrt_internal.hpp"

namespace clrrt {

#define CAND_K 10
#define NN_K (CAND_K + 1)
#define SUPER 8

// Order-preserving float <-> uint32 (for atomicMin over signed floats).
__device__ __forceinline__ uint32_t ord_enc(float f) {
  uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Cells are numbered in Morton (Z) order on a square power-of-two grid, so any aligned 2^k x 2^k
// block -- in particular an 8x8 super-cell -- is a contiguous range, and consecutive records of the
// place-ordered array are close in the plane.
__device__ __forceinline__ uint32_t spread2(uint32_t v) {  // bits of v to the even positions
  v &= 0xffff;
  v = (v | (v << 8)) & 0x00ff00ff;
  v = (v | (v << 4)) & 0x0f0f0f0f;
  v = (v | (v << 2)) & 0x33333333;
  v = (v | (v << 1)) & 0x55555555;
  return v;
}
__device__ __forceinline__ int morton(int x, int y) { return (int)(spread2((uint32_t)x) | (spread2((uint32_t)y) << 1)); }
__device__ __forceinline__ int cell_of(const NnGrid& g, int gx, int gy) { return morton(gx, gy); }
// super-cell (X, Y) holds cells [64 morton(X, Y), 64 morton(X, Y) + 64)
__device__ __forceinline__ int super_of(int X, int Y) { return morton(X, Y); }

__device__ __forceinline__ int node_cell(const NnGrid& g, double x, double y) {
  double fx = (x - g.x0) * g.inv, fy = (y - g.y0) * g.inv;
  if (!(fx >= 0.0 && fx < (double)g.gw && fy >= 0.0 && fy < (double)g.gh)) return g.ncell;  // overflow
  return cell_of(g, (int)fx, (int)fy);
}

__global__ void __launch_bounds__(256) k_nng_count(const NnRec* __restrict__ nodes, int N, NnGrid g,
                                                   int* __restrict__ cellid, uint32_t* __restrict__ count,
                                                   uint32_t* __restrict__ cmin, uint32_t* __restrict__ smin,
                                                   uint32_t* __restrict__ fmin, uint32_t* __restrict__ fmax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const NnRec& r = nodes[i];
  int c = node_cell(g, r.x, r.y);
  // non-finite costs / feasibility inputs, or ref.back() beyond +-2000 km, go to the always-scanned
  // cell (keeps every bound finite and representable)
  const bool ok = isfinite(r.costE) && fabs(r.bx) < 2e6 && fabs(r.by) < 2e6 && fabs(r.ang_par) < 4.0;
  if (!ok) c = g.ncell;
  cellid[i] = c;
  atomicAdd(&count[c], 1u);
  if (c < g.ncell) {
    const uint32_t e = ord_enc(r.costE);
    atomicMin(&cmin[c], e);
    const int sc = c >> 6;
    atomicMin(&smin[sc], e);
    // feasibility bounds in fixed point, rounded outward: ref.back() in mm, ang_par in microradians
    const double ap2 = r.ang_par < 0.0 ? r.ang_par + 2 * M_PI : r.ang_par;
    int* mn = (int*)fmin + 4 * sc;
    int* mx = (int*)fmax + 4 * sc;
    atomicMin(&mn[0], (int)floor(r.bx * 1e3));
    atomicMin(&mn[1], (int)floor(r.by * 1e3));
    atomicMin(&mn[2], (int)floor(r.ang_par * 1e6));
    atomicMin(&mn[3], (int)floor(ap2 * 1e6));
    atomicMax(&mx[0], (int)ceil(r.bx * 1e3));
    atomicMax(&mx[1], (int)ceil(r.by * 1e3));
    atomicMax(&mx[2], (int)ceil(r.ang_par * 1e6));
    atomicMax(&mx[3], (int)ceil(ap2 * 1e6));
  }
}

// Exclusive scan of count[0..n) into start[0..n] (one block, sequential chunks + block scan).
__global__ void __launch_bounds__(1024) k_nng_scan(const uint32_t* __restrict__ count, int n,
                                                   uint32_t* __restrict__ start) {
  __shared__ uint32_t s_sum[1024];
  const int t = threadIdx.x;
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int b0 = min(n, t * per), b1 = min(n, b0 + per);
  uint32_t acc = 0;
  for (int i = b0; i < b1; i++) acc += count[i];
  s_sum[t] = acc;
  __syncthreads();
  for (int off = 1; off < (int)blockDim.x; off <<= 1) {
    uint32_t v = t >= off ? s_sum[t - off] : 0;
    __syncthreads();
    s_sum[t] += v;
    __syncthreads();
  }
  uint32_t run = s_sum[t] - acc;
  for (int i = b0; i < b1; i++) {
    start[i] = run;
    run += count[i];
  }
  if (t == (int)blockDim.x - 1) start[n] = s_sum[t];
}

__global__ void __launch_bounds__(256) k_nng_scatter(const NnRec* __restrict__ nodes, int N,
                                                     const int* __restrict__ cellid,
                                                     const uint32_t* __restrict__ start,
                                                     uint32_t* __restrict__ fill, NnRec* __restrict__ sorted) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int c = cellid[i];
  const uint32_t pos = start[c] + atomicAdd(&fill[c], 1u);
  sorted[pos] = nodes[i];
}

// ------------------------------------------------------------------------------------ samples
// Bucket samples by super-cell (explore buckets first, then optimize; non-finite samples last).
__device__ __forceinline__ int sample_bucket(const NnGrid& g, const clrrt_sample& s) {
  const int SG = g.sw * g.sh;
  const double fx = (s.x - g.x0) * g.inv / SUPER, fy = (s.y - g.y0) * g.inv / SUPER;
  if (!(isfinite(fx) && isfinite(fy))) return 2 * SG;
  const int X = (int)fmin((double)(g.sw - 1), fmax(0.0, floor(fx)));
  const int Y = (int)fmin((double)(g.sh - 1), fmax(0.0, floor(fy)));
  return (s.explore ? 0 : SG) + super_of(X, Y);
}

__global__ void __launch_bounds__(256) k_smp_count(const clrrt_sample* __restrict__ S, int B, NnGrid g,
                                                   uint32_t* __restrict__ count) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < B) atomicAdd(&count[sample_bucket(g, S[t])], 1u);
}

// order[pos] = sample; home[pos] = first place-ordered node record of the sample's grid cell (or of
// the nearest cell inside the grid), where its nearest-node search starts.
__global__ void __launch_bounds__(256) k_smp_scatter(const clrrt_sample* __restrict__ S, int B, NnGrid g,
                                                     const uint32_t* __restrict__ start, uint32_t* __restrict__ fill,
                                                     int* __restrict__ order, int* __restrict__ home) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B) return;
  const int b = sample_bucket(g, S[t]);
  const uint32_t pos = start[b] + atomicAdd(&fill[b], 1u);
  order[pos] = t;
  const double fx = (S[t].x - g.x0) * g.inv, fy = (S[t].y - g.y0) * g.inv;
  int h = 0;
  if (isfinite(fx) && isfinite(fy)) {
    const int gx = (int)fmin((double)(g.gw - 1), fmax(0.0, floor(fx)));
    const int gy = (int)fmin((double)(g.gh - 1), fmax(0.0, floor(fy)));
    h = (int)g.start[cell_of(g, gx, gy)];
  }
  home[pos] = h;
}

// ------------------------------------------------------------------------------------ search
__device__ __forceinline__ bool lex_less2(float ka, int ia, float kb, int ib) {
  return (ka < kb) || (ka == kb && ia < ib);
}

__device__ __forceinline__ void topk_insert2(float (&keys)[NN_K], int (&ids)[NN_K], float k, int i) {
#pragma unroll
  for (int j = 0; j < NN_K; j++) {
    bool sw = lex_less2(k, i, keys[j], ids[j]);
    float tk = keys[j];
    int ti = ids[j];
    keys[j] = sw ? k : tk;
    ids[j] = sw ? i : ti;
    k = sw ? tk : k;
    i = sw ? ti : i;
  }
}

// Lower bound on a float key for an exact Euclidean distance lower bound d >= 0.
__device__ __forceinline__ float key_lb(double d) { return (float)(d * 0.99998 - 2e-4); }

// Distance from (sx, sy) to the rectangle of grid cells [cx0, cx1) x [cy0, cy1), minus a slack.
__device__ __forceinline__ double rect_dist(const NnGrid& g, double sx, double sy, int cx0, int cy0, int cx1,
                                            int cy1) {
  const double rx0 = g.x0 + cx0 * g.cs, rx1 = g.x0 + cx1 * g.cs;
  const double ry0 = g.y0 + cy0 * g.cs, ry1 = g.y0 + cy1 * g.cs;
  const double dx = fmax(0.0, fmax(rx0 - sx, sx - rx1));
  const double dy = fmax(0.0, fmax(ry0 - sy, sy - ry1));
  return fmax(0.0, sqrt(dx * dx + dy * dy) - g.slack);
}

__device__ __forceinline__ float wrapf(float a) {  // into [-pi, pi)
  const float tp = (float)(2 * M_PI), pi = (float)M_PI;
  return a - tp * floorf((a + pi) / tp);
}

// True when no node of super-cell sc can be feasible for the sample (see the header).
__device__ __forceinline__ bool super_infeasible(const NnGrid& g, int sc, double sx, double sy) {
  const int* mn = (const int*)g.fmin + 4 * sc;
  const int* mx = (const int*)g.fmax + 4 * sc;
  const double m = 1e-3;  // metres: rounding of the bounds and of the sample
  const double x0 = mn[0] * 1e-3 - m, y0 = mn[1] * 1e-3 - m;
  const double x1 = mx[0] * 1e-3 + m, y1 = mx[1] * 1e-3 + m;
  // the sample must lie clearly outside the box: float rounding of the direction vectors below then
  // moves the arc by far less than the 1e-3 rad margin
  const double out = fmax(fmax(x0 - sx, sx - x1), fmax(y0 - sy, sy - y1));  // > 0: outside the box
  if (!(out > 0.05)) return false;
  // arc of directions from the box to the sample (the box is convex and excludes the sample)
  const float t0 = atan2f((float)(sy - y0), (float)(sx - x0));
  const float d1 = wrapf(atan2f((float)(sy - y0), (float)(sx - x1)) - t0);
  const float d2 = wrapf(atan2f((float)(sy - y1), (float)(sx - x0)) - t0);
  const float d3 = wrapf(atan2f((float)(sy - y1), (float)(sx - x1)) - t0);
  const float dlo = fminf(0.f, fminf(d1, fminf(d2, d3)));
  const float dhi = fmaxf(0.f, fmaxf(d1, fmaxf(d2, d3)));
  const float cI = t0 + 0.5f * (dlo + dhi), wI = 0.5f * (dhi - dlo);
  // the ang_par values lie in both arcs [a1, b1] (atan2 range) and [a2, b2] (shifted to [0, 2pi)):
  // either arc far enough from the direction arc proves infeasibility
  const float a1 = (float)mn[2] * 1e-6f, b1 = (float)mx[2] * 1e-6f;
  const float a2 = (float)mn[3] * 1e-6f, b2 = (float)mx[3] * 1e-6f;
  const float gap1 = fabsf(wrapf(cI - 0.5f * (a1 + b1))) - wI - 0.5f * (b1 - a1);
  const float gap2 = fabsf(wrapf(cI - 0.5f * (a2 + b2))) - wI - 0.5f * (b2 - a2);
  return fmaxf(gap1, gap2) > (float)(M_PI / 4) + 1e-3f;
}

struct Lane {
  double sx, sy;
  int ex;
  bool act;
  float keys[NN_K];
  int ids[NN_K];
};

// Nodes recs[a .. b) (wave-uniform range) offered to the lanes with `take` set.
__device__ __forceinline__ void scan_nodes(Lane& L, const NnRec* __restrict__ recs, uint32_t a, uint32_t b,
                                           bool take, double feas_len) {
  const float feas2 = nn_feas2(feas_len);
  for (uint32_t k = a; k < b; k++) {
    const NnRec rec = recs[k];
    if (!take) continue;
    float qx = (float)(L.sx - rec.x), qy = (float)(L.sy - rec.y);
    float lb = sqrtf(qx * qx + qy * qy) * 0.99999f - 1e-4f;
    if (!L.ex) lb = rec.costE + lb;
    if (lb <= L.keys[NN_K - 1] &&
        nn_prefilter(L.sx, L.sy, qx, qy, rec.c, rec.s, rec.ca, rec.sa, rec.bx, rec.by, rec.costE, L.ex,
                     L.keys[NN_K - 1], feas2)) {
      float key = dubins_key(L.sx, L.sy, rec.x, rec.y, rec.c, rec.s);
      if (!L.ex) key = rec.costE + key;
      if (lex_less2(key, rec.id, L.keys[NN_K - 1], L.ids[NN_K - 1]) &&
          feasible_search(L.sx, L.sy, rec.bx, rec.by, rec.ca, rec.sa, rec.ang_par, feas_len))
        topk_insert2(L.keys, L.ids, key, rec.id);
    }
  }
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// One super-cell (wave-uniform SX, SY) for the whole wave.
__device__ __forceinline__ void visit_super(Lane& L, const NnGrid& g, int SX, int SY, double feas_len,
                                            int& budget, bool& truncated) {
  if (budget <= 0) {  // out of budget: this super-cell is not searched
    truncated = true;
    return;
  }
  const int sc = super_of(SX, SY);
  const uint32_t sm = g.smin[sc];
  if (sm == 0xffffffffu) return;  // empty
  bool need = false;
  if (L.act) {
    float lb = key_lb(rect_dist(g, L.sx, L.sy, SX * SUPER, SY * SUPER, SX * SUPER + SUPER, SY * SUPER + SUPER));
    if (!L.ex) lb = ord_dec(sm) + lb;
    need = !(lb > L.keys[NN_K - 1]) && !super_infeasible(g, sc, L.sx, L.sy);
  }
  if (__ballot(need) == 0) return;
  const int base = sc * 64;
  for (int c = 0; c < 64; c++) {
    const uint32_t a = g.start[base + c], b = g.start[base + c + 1];
    if (a == b) continue;
    bool take = false;
    if (need) {
      const int gx = SX * SUPER + (c & 1) + ((c >> 1) & 2) + ((c >> 2) & 4);
      const int gy = SY * SUPER + ((c >> 1) & 1) + ((c >> 2) & 2) + ((c >> 3) & 4);
      float lb = key_lb(rect_dist(g, L.sx, L.sy, gx, gy, gx + 1, gy + 1));
      if (!L.ex) lb = ord_dec(g.cmin[base + c]) + lb;
      take = !(lb > L.keys[NN_K - 1]);
    }
    if (__ballot(take) == 0) continue;
    budget -= (int)(b - a);
    scan_nodes(L, g.recs, a, b, take, feas_len);
  }
}

__global__ void __launch_bounds__(256) k_nn_tile(const clrrt_sample* __restrict__ S, int B, const int* __restrict__ order,
                                                 NnGrid g, DevParams p, int* __restrict__ cand,
                                                 float* __restrict__ ckey, int* __restrict__ ncand,
                                                 int* __restrict__ ctie, int cap, int* __restrict__ fb_list,
                                                 int* __restrict__ fb_count, unsigned long long* __restrict__ stats) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x + (threadIdx.x & ~63)) >= B) return;  // whole wave past the end
  Lane L;
  L.act = t < B;
  const int s = L.act ? order[t] : 0;
  L.sx = L.act ? S[s].x : 0.0;
  L.sy = L.act ? S[s].y : 0.0;
  L.ex = L.act ? S[s].explore : 1;
#pragma unroll
  for (int j = 0; j < NN_K; j++) { L.keys[j] = __builtin_inff(); L.ids[j] = 0x7fffffff; }
  const double fx = (L.sx - g.x0) * g.inv / SUPER, fy = (L.sy - g.y0) * g.inv / SUPER;
  // non-finite samples and samples of modes not searched through the grid go to brute force
  bool fallback = L.act && (!(isfinite(fx) && isfinite(fy)) || !(g.modes & (L.ex ? 1 : 2)));
  if (fallback) L.act = false;
  int budget = cap;
  // nodes outside the grid (or with non-finite bounds) are offered to every lane
  {
    const uint32_t a = g.start[g.ncell], b = g.start[g.ncell + 1];
    if ((int)(b - a) > budget) {
      budget = -1;
    } else {
      budget -= (int)(b - a);
      scan_nodes(L, g.recs, a, b, L.act, p.feas_len);
    }
  }
  // the lane's super-cell and the wave's centre
  const int X = L.act ? (int)fmin((double)(g.sw - 1), fmax(0.0, floor(fx))) : 0;
  const int Y = L.act ? (int)fmin((double)(g.sh - 1), fmax(0.0, floor(fy))) : 0;
  const int any = __ballot(L.act) != 0;
  const int x0 = wave_min(L.act ? X : 0x7fffffff), x1 = wave_max(L.act ? X : -1);
  const int y0 = wave_min(L.act ? Y : 0x7fffffff), y1 = wave_max(L.act ? Y : -1);
  const int CX = __builtin_amdgcn_readfirstlane(any ? (x0 + x1) / 2 : 0);
  const int CY = __builtin_amdgcn_readfirstlane(any ? (y0 + y1) / 2 : 0);
  const int dl = max(abs(X - CX), abs(Y - CY));  // lane's super-cell distance from the centre
  const int maxr = max(max(CX, g.sw - 1 - CX), max(CY, g.sh - 1 - CY));
  const float cmin_all = ord_dec(g.gmin[0]);
  const double scs = g.cs * SUPER;
  bool done = !L.act;
  bool truncated = budget <= 0;
  int r = 0;
  if (any && !truncated) {
    for (; r <= maxr; r++) {
      // ring r lies >= (r - dl - 1) super-cells from the lane's sample; the bound covers every later
      // ring, but only while no super-cell has been skipped for the budget
      if (!done && !truncated && r - dl - 1 >= 1) {
        float lb = key_lb(fmax(0.0, (r - dl - 1) * scs - g.slack));
        if (!L.ex) lb = cmin_all + lb;
        done = lb > L.keys[NN_K - 1];
      }
      if (__ballot(!done) == 0 || truncated) break;
      for (int dy = -r; dy <= r; dy++) {
        const int cy = CY + dy;
        if (cy < 0 || cy >= g.sh) continue;
        const int step = (dy == -r || dy == r) ? 1 : 2 * r;
        for (int dx = -r; dx <= r; dx += step) {
          const int cx = CX + dx;
          if (cx >= 0 && cx < g.sw) visit_super(L, g, cx, cy, p.feas_len, budget, truncated);
        }
      }
    }
    if (r > maxr && !truncated) done = true;  // every ring visited in full
  }
  if (stats && (threadIdx.x & 63) == 0) {  // search statistics: waves, nodes read, rings, truncated waves
    atomicAdd(&stats[0], 1ull);
    atomicAdd(&stats[1], (unsigned long long)(cap - budget));
    atomicAdd(&stats[2], (unsigned long long)r);
    atomicAdd(&stats[3], (unsigned long long)truncated);
  }
  if (!L.act) {
    if (fallback) fb_list[atomicAdd(fb_count, 1)] = s;
    return;
  }
  if (!done) {  // budget spent before this lane's search completed: brute force
    fb_list[atomicAdd(fb_count, 1)] = s;
    return;
  }
  int valid = 0, n = 0, tie = 0;
#pragma unroll
  for (int j = 0; j < NN_K; j++) valid += L.ids[j] != 0x7fffffff;
  const int sel = min(p.sort_limit, valid);
#pragma unroll
  for (int j = 0; j < CAND_K; j++) {
    bool v = j < sel;
    cand[s * CAND_K + j] = v ? L.ids[j] : -1;
    ckey[s * CAND_K + j] = L.keys[j];
    n += v;
    tie |= (j < sel && j + 1 < valid && L.keys[j] == L.keys[j + 1]);
  }
  ncand[s] = n;
  ctie[s] = tie;
}

__global__ void k_nng_gmin(const uint32_t* __restrict__ smin, int n, uint32_t* __restrict__ gmin) {
  uint32_t m = 0xffffffffu;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = min(m, smin[i]);
  atomicMin(gmin, m);
}

#define LAUNCH_CHECK2()                          \
  do {                                           \
    hipError_t e_ = hipGetLastError();           \
    if (e_ != hipSuccess) return e_;             \
  } while (0)

hipError_t launch_nn_grid_build(hipStream_t st, const NnRec* nodes, int N, NnGrid& g, NnGridBufs& b) {
  const int G = g.ncell;
  const int SG = g.sw * g.sh;
  hipError_t e;
  if ((e = hipMemsetAsync(b.fmin, 0x7f, sizeof(uint32_t) * 4 * SG, st)) != hipSuccess) return e;  // ~INT_MAX
  if ((e = hipMemsetAsync(b.fmax, 0x80, sizeof(uint32_t) * 4 * SG, st)) != hipSuccess) return e;  // ~INT_MIN
  if ((e = hipMemsetAsync(b.count, 0, sizeof(uint32_t) * (G + 1), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.fill, 0, sizeof(uint32_t) * (G + 1), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.cmin, 0xff, sizeof(uint32_t) * G, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.smin, 0xff, sizeof(uint32_t) * (SG + 1), st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_nng_count, dim3((N + 255) / 256), dim3(256), 0, st, nodes, N, g, b.cellid, b.count, b.cmin,
                     b.smin, b.fmin, b.fmax);
  LAUNCH_CHECK2();
  hipLaunchKernelGGL(k_nng_scan, dim3(1), dim3(1024), 0, st, b.count, G + 1, b.start);
  LAUNCH_CHECK2();
  hipLaunchKernelGGL(k_nng_scatter, dim3((N + 255) / 256), dim3(256), 0, st, nodes, N, b.cellid, b.start, b.fill,
                     b.sorted);
  LAUNCH_CHECK2();
  hipLaunchKernelGGL(k_nng_gmin, dim3(1), dim3(1024), 0, st, b.smin, SG, b.smin + SG);
  LAUNCH_CHECK2();
  g.start = b.start;
  g.recs = b.sorted;
  g.cmin = b.cmin;
  g.smin = b.smin;
  g.gmin = b.smin + SG;
  g.fmin = b.fmin;
  g.fmax = b.fmax;
  return hipSuccess;
}

hipError_t launch_sample_order(hipStream_t st, const clrrt_sample* S, int B, const NnGrid& g, NnGridBufs& b) {
  const int nb = 2 * g.sw * g.sh + 1;
  hipError_t e;
  if ((e = hipMemsetAsync(b.scount, 0, sizeof(uint32_t) * (nb + 1), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.sfill, 0, sizeof(uint32_t) * (nb + 1), st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_smp_count, dim3((B + 255) / 256), dim3(256), 0, st, S, B, g, b.scount);
  LAUNCH_CHECK2();
  hipLaunchKernelGGL(k_nng_scan, dim3(1), dim3(1024), 0, st, b.scount, nb, b.sstart);
  LAUNCH_CHECK2();
  hipLaunchKernelGGL(k_smp_scatter, dim3((B + 255) / 256), dim3(256), 0, st, S, B, g, b.sstart, b.sfill, b.order,
                     b.home);
  LAUNCH_CHECK2();
  return hipSuccess;
}

hipError_t launch_nn_grid_search(hipStream_t st, const clrrt_sample* S, int B, const NnGrid& g, const DevParams& p,
                                 int* cand, float* ckey, int* ncand, int* ctie, int cap, int* fb_list,
                                 int* fb_count, NnGridBufs& b, unsigned long long* stats) {
  hipError_t e = launch_sample_order(st, S, B, g, b);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_nn_tile, dim3((B + 255) / 256), dim3(256), 0, st, S, B, b.order, g, p, cand, ckey, ncand, ctie,
                     cap, fb_list, fb_count, stats);
  LAUNCH_CHECK2();
  return hipSuccess;
}

}  // namespace clrrt
