// clrrt_nnwalk.hip — nearest-node search (sortNodesExplore / sortNodesOptimize + feasibleNode,
// rrtplanner.cpp:227-289) by a bounded walk over a place-ordered tree, one wave per sample.
//
// The reference keys every node by its Dubins distance to the sample (explore) or costE + Dubins
// distance (optimize), sorts, and keeps the first sortLimit feasible nodes.  The result is the
// sortLimit smallest (key, node index) pairs among the feasible nodes (+ one more entry that
// reveals a key tie at the selection boundary), which the brute-force kernels find by scanning all
// N nodes for every sample.  On bench trees a sample's list depends on ~0.1% of the nodes, so:
//
// Index (rebuilt every round): nodes sorted by ang_par sector and a 16-bit-per-axis Morton code of
// their position (radix sort), copied into place order as float records relative to the round's frame origin,
// padded to a multiple of 1024.  Every 32 consecutive records form a tile, every 32 tiles a
// super-tile; each carries conservative bounds (WalkTile): a disc around the positions and one
// around the ref.back() points, the arc of headings and the arc of ang_par directions, the minimum
// costE and the minimum of costE - |position - disc centre|.
//
// Search (k_walk_search, one 64-lane wave per sample): lower bounds on the keys of every super-tile
// are kept in LDS; tiles are visited in passes of growing bound threshold (so the list fills with
// near nodes first and its 11th key prunes the rest): a super-tile's 32 tile bounds are computed by
// 32 lanes, the tiles under the threshold are visited two at a time (one node per lane) through the
// necessary conditions of the brute-force prefilter plus the turning bound below, and the
// super-tile's bound becomes that of its remaining tiles.  Survivors are queued in LDS and their
// exact keys computed 64 at a time, so lanes stay converged.
// The sample's list lives in lanes 0..10 (sorted), the 11th entry (kth, idk) is wave-uniform.
//
// Bounds (each lower-bounds the float key the reference computes; margins cover float rounding):
//   * key >= |q|                 (Dubins length >= Euclidean; |q| (1 - 1e-5) - 1e-4 in float);
//   * key >= rho * beta          beta = angle between the node heading and the direction to the
//                                sample: a left-turn-then-straight path ending at bearing beta
//                                turns by psi >= beta (psi <= pi: the end point lies between the
//                                arc chord bearing psi / 2 and psi), and the inside-circle case
//                                has key >= rho * pi (checked numerically by tests/test_nnwalk_bounds.py);
//   * optimize: key = costE + dubins >= costE - |p - c| + |s - c| for any point c;
//   * feasibleNode: the direction from ref.back() to the sample must lie within pi/4 of ang_par and
//     |sample - ref.back()| >= 2.1 ref_res.
// A skipped node, tile or super-tile can hold no pair that enters the list, so every list equals
// the brute-force one bit for bit (ties included: pairs are ordered by (key, node index) in both).
#include <hip/hip_runtime.h>
#include <climits>
#include <hip/hip_fp16.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_merge.hpp>
#include <algorithm>
#include <stdint.h>

#include "clrrt_dev.hpp"
#include "clrrt_internal.hpp"

namespace clrrt {

#define CAND_K 10
#define NN_K (CAND_K + 1)
#define WALK_TILE 32
#define WALK_SUPER 32  // tiles per super-tile
#define WALK_FMT_STATE 0  // k_walk_search LDS formats: float bound + visited mask per super-tile,
#define WALK_FMT_HALF 1   // fp16 bound (stateless),
#define WALK_FMT_CODED 2  // one log-coded byte (stateless; large trees)
#ifndef WALK_STAGE1_QUEUE
#define WALK_STAGE1_QUEUE 0  // measured neutral (round 4); off saves 768 B of LDS per wave
#endif
#ifndef WALK_HALF_SUPER
#define WALK_HALF_SUPER 1  // HALF format: keep each super-tile's phase-1 bound in LDS (2 more bytes per super-tile)
#endif
#define WALK_TQ 68      // tile stack entries (a super-tile pair adds <= 64 to <= 3 pending)
#ifndef WALK_SPLIT_SHARE
#define WALK_SPLIT_SHARE 1  // the overflow split waves of one record share their bounds (round 5)
#endif
#ifndef WALK_APBINS
#define WALK_APBINS 8  // ang_par sectors (top key bits)
#endif
#ifndef WALK_SECTOR_BITS
#define WALK_SECTOR_BITS 3  // 2^WALK_SECTOR_BITS >= WALK_APBINS
#endif

#define LAUNCH_CHECK3()                          \
  do {                                           \
    hipError_t e_ = hipGetLastError();           \
    if (e_ != hipSuccess) return e_;             \
  } while (0)

__device__ __forceinline__ uint32_t w_spread(uint32_t v) {
  v &= 0xffff;
  v = (v | (v << 8)) & 0x00ff00ff;
  v = (v | (v << 4)) & 0x0f0f0f0f;
  v = (v | (v << 2)) & 0x33333333;
  v = (v | (v << 1)) & 0x55555555;
  return v;
}

__device__ __forceinline__ uint64_t w_spread3(uint32_t v) {  // 16 bits -> every third bit of 48
  uint64_t x = v & 0xffff;
  x = (x | (x << 16)) & 0x0000ff0000ffull;
  x = (x | (x << 8)) & 0x00f00f00f00full;
  x = (x | (x << 4)) & 0x0c30c30c30c3ull;
  x = (x | (x << 2)) & 0x249249249249ull;
  return x;
}

// Sort key of each node (the index's place order; any order gives valid bounds, the order sets how tight they are).
// kind 0: ang_par sector (3 bits), Morton code of its position in the frame box (non-finite positions last
// within the sector), then the costE bits (top 29).  kind 1 / 2: 3D Morton code (16 bits per axis) of (x, y,
// rho * angle) in one metric scale -- angle = the node's heading (kind 1, from the Dubins rotation (c, s) = (cos,
// sin)(-heading)) or ang_par (kind 2), wrapped to [-pi, pi) -- then the top 16 costE bits.  kind 3 / 4: the
// ang_par sector, then kind 1's / kind 2's 3D code, then the top 13 costE bits.  kind 5 (round 6): kind 3 with a
// coarse 13-bit Morton code of ref.back() (7 / 6 bits of x / y) in place of the costE bits: records whose position,
// heading and cost are equal -- the root's zero-length children, one run of 10^4 per ang_par sector whose
// ref.back() points are their samples, anywhere -- then lie in ref.back() order, so their tiles' ref.back() discs are
// small and the feasibleNode cone bound can drop them.  Records with equal key inputs (e.g. the root's zero-length
// children) end up next to each other in every kind.
__global__ void k_walk_keys(const NnRec* __restrict__ nodes, int N, double x0, double y0, double scale,
                            uint64_t* __restrict__ keys, int* __restrict__ vals, int first = 0, int kind = 0,
                            double hrho = 4.77) {
  const int k0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (k0 >= N - first) return;
  const int i = first + k0;
  keys += -first;  // entries are written at [k0] (keys[i] below)
  vals += -first;
  const double x = nodes[i].x, y = nodes[i].y;
  // ang_par octant (kinds 0, 3, 4)
  const float apf = (float)nodes[i].ang_par;
  int bin = (int)floorf((apf + 3.14159265f) * (WALK_APBINS / 6.2831853f));
  bin = bin < 0 ? 0 : (bin >= WALK_APBINS ? WALK_APBINS - 1 : bin);
  if (kind >= 3) {  // octant, then the 3D Morton code of (x, y, rho * heading | ang_par) inside it
    const float ang = kind != 4 ? atan2f(-nodes[i].s, nodes[i].c) : apf;
    const double a = isfinite(ang) ? (double)ang - 6.283185307179586 * floor(((double)ang + M_PI) / 6.283185307179586)
                                   : 0.0;  // [-pi, pi)
    uint64_t m = 0xffffffffffffull;
    if (isfinite(x) && isfinite(y)) {
      const double fx = fmin(fmax((x - x0) * scale, 0.0), 65535.0);
      const double fy = fmin(fmax((y - y0) * scale, 0.0), 65535.0);
      const double fz = fmin(fmax((a + M_PI) * hrho * scale, 0.0), 65535.0);
      m = w_spread3((uint32_t)fx) | (w_spread3((uint32_t)fy) << 1) | (w_spread3((uint32_t)fz) << 2);
    }
    uint64_t low = __float_as_uint(nodes[i].costE) >> (16 + WALK_SECTOR_BITS);
    if (kind == 5) {  // coarse ref.back() cell instead of the cost (13 = 16 - WALK_SECTOR_BITS bits)
      const double bx = nodes[i].bx, by = nodes[i].by;
      uint32_t cx = 0, cy = 0;
      if (isfinite(bx) && isfinite(by)) {
        cx = (uint32_t)fmin(fmax((bx - x0) * scale, 0.0), 65535.0) >> 9;  // 7 bits
        cy = (uint32_t)fmin(fmax((by - y0) * scale, 0.0), 65535.0) >> 10;  // 6 bits
      }
      low = (w_spread(cx) | (w_spread(cy) << 1)) & 0x1fffu;
    }
    keys[i] = ((uint64_t)bin << (64 - WALK_SECTOR_BITS)) | (m << (16 - WALK_SECTOR_BITS)) | low;
    vals[i] = i;
    return;
  }
  if (kind != 0) {
    const float ang = kind == 1 ? atan2f(-nodes[i].s, nodes[i].c) : apf;
    const double a = isfinite(ang) ? (double)ang - 6.283185307179586 * floor(((double)ang + M_PI) / 6.283185307179586)
                                   : 0.0;  // [-pi, pi)
    uint64_t m = 0xffffffffffffull;
    if (isfinite(x) && isfinite(y)) {
      const double fx = fmin(fmax((x - x0) * scale, 0.0), 65535.0);
      const double fy = fmin(fmax((y - y0) * scale, 0.0), 65535.0);
      const double fz = fmin(fmax((a + M_PI) * hrho * scale, 0.0), 65535.0);
      m = w_spread3((uint32_t)fx) | (w_spread3((uint32_t)fy) << 1) | (w_spread3((uint32_t)fz) << 2);
    }
    keys[i] = (m << 16) | (__float_as_uint(nodes[i].costE) >> 16);
    vals[i] = i;
    return;
  }
  uint32_t k = 0xffffffffu;
  if (isfinite(x) && isfinite(y)) {
    const double fx = fmin(fmax((x - x0) * scale, 0.0), 65535.0);
    const double fy = fmin(fmax((y - y0) * scale, 0.0), 65535.0);
    k = w_spread((uint32_t)fx) | (w_spread((uint32_t)fy) << 1);
  }
  // ang_par octant first: tiles then hold similar reference directions, which sharpens the tiles'
  // feasibleNode bound (measured: 555 -> 332 tiles per explore sample, same work for optimize)
  keys[i] = ((uint64_t)bin << (64 - WALK_SECTOR_BITS)) | ((uint64_t)k << (32 - WALK_SECTOR_BITS)) |
            (__float_as_uint(nodes[i].costE) >> WALK_SECTOR_BITS);
  vals[i] = i;
}

// Morton key of each sample (same frame as the nodes).
// (zero: counters the search that follows takes from -- the overflow record count and the persistent grid's per-XCD
// sample counters -- reset here instead of by fills of their own)
__global__ void k_walk_skeys(const clrrt_sample* __restrict__ S, int B, double x0, double y0, double scale,
                             uint32_t* __restrict__ keys, int* __restrict__ vals, int* __restrict__ zero1,
                             int* __restrict__ zero8) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (zero1 && i == 0) *zero1 = 0;
  if (zero8 && i < 8) zero8[i] = 0;
  if (i >= B) return;
  const double x = S[i].x, y = S[i].y;
  uint32_t k = 0xffffffffu;
  if (isfinite(x) && isfinite(y)) {
    const double fx = fmin(fmax((x - x0) * scale, 0.0), 65535.0);
    const double fy = fmin(fmax((y - y0) * scale, 0.0), 65535.0);
    k = w_spread((uint32_t)fx) | (w_spread((uint32_t)fy) << 1);
  }
  keys[i] = k;
  vals[i] = i;
}

// Longest-first order inside each XCD's eighth of the place-ordered samples (option nn_walk_lpt): the persistent
// walk hands an eighth's samples out in order, so its optimize samples (several times an explore sample's exact
// keys, profiles/r06g_walk_audit.txt) go first and the cheap explore samples fill the end; each class keeps its
// place order (a stable partition, one 1024-thread block per eighth).  Scheduling only: every list is the same.
__global__ void __launch_bounds__(1024) k_walk_lpt(const clrrt_sample* __restrict__ S, int B,
                                                   const int* __restrict__ sorder, int* __restrict__ out) {
  __shared__ int part[1024];
  const int per = (B + 7) >> 3;
  const int base = (int)blockIdx.x * per;
  const int n = min(per, B - base);
  if (n <= 0) return;
  const int t = threadIdx.x;
  const int ipt = (n + 1023) >> 10;
  const int i0 = min(n, t * ipt), i1 = min(n, i0 + ipt);
  int c = 0;
  for (int i = i0; i < i1; i++) c += S[sorder[base + i]].explore == 0;
  part[t] = c;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan of the optimize counts
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int total = part[1023];
  int po = part[t] - c;  // optimize samples before this thread's items
  int pe = i0 - po;      // explore samples before them
  for (int i = i0; i < i1; i++) {
    const int v = sorder[base + i];
    if (S[v].explore == 0) out[base + po++] = v;
    else out[base + total + pe++] = v;
  }
}

// Per tile: (run head, smallest id) when all 32 records lie in one run of equal key inputs (HEAD is the
// run's first record: equal at the tile's ends), else (-1, -1).
__global__ void k_walk_trun(const int* __restrict__ HEAD, const int* __restrict__ ID, int ntiles,
                            int2* __restrict__ trun) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const int j0 = t * WALK_TILE;
  const int h = HEAD[j0];
  if (HEAD[j0 + WALK_TILE - 1] != h) {
    trun[t] = make_int2(-1, -1);
    return;
  }
  int m = 0x7fffffff;
  for (int q = 0; q < WALK_TILE; q++) m = min(m, ID[j0 + q]);
  trun[t] = m >= 0 ? make_int2(h, m) : make_int2(-1, -1);
}

// Place-ordered float records (relative to the frame origin); entries N .. Npad are padding (id -1).
__global__ void k_walk_gather(const NnRec* __restrict__ nodes, int N, int Npad, const int* __restrict__ order,
                              double ox, double oy, float4* __restrict__ P, float4* __restrict__ Q,
                              float* __restrict__ CE, int* __restrict__ ID, int* __restrict__ dup) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Npad) return;
  if (j < N) {
    const int i = order[j];
    const NnRec& r = nodes[i];
    P[j] = make_float4((float)(r.x - ox), (float)(r.y - oy), r.c, r.s);
    Q[j] = make_float4((float)(r.bx - ox), (float)(r.by - oy), r.ca, r.sa);
    CE[j] = r.costE;
    ID[j] = i;
    // a record whose Dubins-key inputs equal its predecessor's has the same key for every sample
    bool same = false;
    if (j > 0) {
      const NnRec& o = nodes[order[j - 1]];
      same = r.x == o.x && r.y == o.y && r.c == o.c && r.s == o.s && r.costE == o.costE;
    }
    dup[j] = same ? -1 : j;
  } else {
    dup[j] = j;
    P[j] = make_float4(0.f, 0.f, 1.f, 0.f);
    Q[j] = make_float4(0.f, 0.f, 1.f, 0.f);
    CE[j] = 0.f;
    ID[j] = -1;
  }
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wmin(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bounds of `size` consecutive records per tile, one wave per tile.  `slack` inflates the discs by
// the float frame's coordinate error so the bounds hold for the exact positions too.
__global__ void __launch_bounds__(256) k_walk_tiles(const float4* __restrict__ P, const float4* __restrict__ Q,
                                                    const float* __restrict__ CE, const int* __restrict__ ID,
                                                    int ntiles, int size, float slack,
                                                    const NnRec* __restrict__ nodes, double ox, double oy,
                                                    WalkTile* __restrict__ out) {
  // R = node 0's position in the frame (any fixed point gives a valid bound; the root gives a tight one)
  const float Rx = (float)(nodes[0].x - ox), Ry = (float)(nodes[0].y - oy);
  const int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // one wave per tile
  const int lane = threadIdx.x & 63;
  if (t >= ntiles) return;
  const int b = t * size;
  float spx = 0, spy = 0, srx = 0, sry = 0, sux = 0, suy = 0, sax = 0, say = 0, cnt = 0, bad = 0;
  for (int k = lane; k < size; k += 64) {
    const int j = b + k;
    if (ID[j] < 0) continue;
    const float4 p = P[j], q = Q[j];
    const float ce = CE[j];
    const bool fin = isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w) && isfinite(q.x) &&
                     isfinite(q.y) && isfinite(q.z) && isfinite(q.w) && isfinite(ce);
    if (!fin) { bad += 1; continue; }
    spx += p.x; spy += p.y; srx += q.x; sry += q.y;
    sux += p.z; suy -= p.w;  // heading direction (cos th, sin th) = (c, -s)
    sax += q.z; say += q.w;
    cnt += 1;
  }
  cnt = wsum(cnt);
  bad = wsum(bad);
  WalkTile w;
  w.nonfinite = bad > 0;
  w.eroot = 0.f;
  if (cnt == 0) {  // padding only (or only non-finite records)
    w.pcx = w.pcy = w.rcx = w.rcy = 0.f;
    w.pr = w.rr = -1.f;  // empty
    w.thx = 1.f; w.thy = 0.f; w.thh = 4.f;
    w.apx = 1.f; w.apy = 0.f; w.aph = 4.f;
    w.cemin = w.aopt = w.eroot = 0.f;
    if (lane == 0) out[t] = w;
    return;
  }
  const float pcx = wsum(spx) / cnt, pcy = wsum(spy) / cnt;
  const float rcx = wsum(srx) / cnt, rcy = wsum(sry) / cnt;
  float ux = wsum(sux), uy = wsum(suy), ax = wsum(sax), ay = wsum(say);
  const float un = sqrtf(ux * ux + uy * uy), an = sqrtf(ax * ax + ay * ay);
  const bool uok = un > 1e-3f * cnt, aok = an > 1e-3f * cnt;
  ux = uok ? ux / un : 1.f; uy = uok ? uy / un : 0.f;
  ax = aok ? ax / an : 1.f; ay = aok ? ay / an : 0.f;
  float pr = 0, rr = 0, ud = 1, ad = 1, cmin = __builtin_inff(), aopt = __builtin_inff(), eroot = __builtin_inff();
  for (int k = lane; k < size; k += 64) {
    const int j = b + k;
    if (ID[j] < 0) continue;
    const float4 p = P[j], q = Q[j];
    const float ce = CE[j];
    const bool fin = isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w) && isfinite(q.x) &&
                     isfinite(q.y) && isfinite(q.z) && isfinite(q.w) && isfinite(ce);
    if (!fin) continue;
    const float dp = sqrtf((p.x - pcx) * (p.x - pcx) + (p.y - pcy) * (p.y - pcy));
    const float dr = sqrtf((q.x - rcx) * (q.x - rcx) + (q.y - rcy) * (q.y - rcy));
    pr = fmaxf(pr, dp);
    rr = fmaxf(rr, dr);
    // unit-length up to float rounding: normalise before the dot product
    const float hn = sqrtf(p.z * p.z + p.w * p.w), qn = sqrtf(q.z * q.z + q.w * q.w);
    ud = fminf(ud, (p.z * ux - p.w * uy) / hn);
    ad = fminf(ad, (q.z * ax + q.w * ay) / qn);
    cmin = fminf(cmin, ce);
    aopt = fminf(aopt, ce - dp);
    eroot = fminf(eroot, ce - sqrtf((p.x - Rx) * (p.x - Rx) + (p.y - Ry) * (p.y - Ry)));
  }
  pr = wmax(pr); rr = wmax(rr); ud = wmin(ud); ad = wmin(ad); cmin = wmin(cmin); aopt = wmin(aopt);
  eroot = wmin(eroot);
  w.pcx = pcx; w.pcy = pcy; w.pr = pr * (1.f + 1e-5f) + 2.f * slack + 1e-5f;
  w.rcx = rcx; w.rcy = rcy; w.rr = rr * (1.f + 1e-5f) + 2.f * slack + 1e-5f;
  w.thx = ux; w.thy = uy; w.thh = uok ? acosf(fminf(fmaxf(ud, -1.f), 1.f)) + 2e-3f : 4.f;
  w.apx = ax; w.apy = ay; w.aph = aok ? acosf(fminf(fmaxf(ad, -1.f), 1.f)) + 2e-3f : 4.f;
  w.cemin = cmin;
  w.aopt = aopt - 2.f * slack - 1e-4f - 1e-5f * fabsf(aopt);
  // R is a float frame point (exact as given); the node positions err by the frame's slack
  w.eroot = eroot - 2.f * slack - 1e-4f - 1e-5f * fabsf(eroot);
  if (lane == 0) out[t] = w;
}

// Bounds need no correctly rounded division / square root (the build flag makes '/' and sqrtf
// correctly rounded for the exact keys): hardware reciprocal and square root, ~1 ulp, far inside the
// bounds' margins.
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// acos on [-1, 1] (Abramowitz & Stegun 4.4.45), |error| <= 7e-5 rad (float evaluation included).
__device__ __forceinline__ float acos_apx(float x) {
  const float ax = fminf(fabsf(x), 1.f);
  const float r = fsqrt(1.f - ax) * (1.5707288f + ax * (-0.2121144f + ax * (0.0742610f + ax * -0.0187293f)));
  return x < 0.f ? 3.14159265f - r : r;
}

// atan2 in float, |error| <= 1e-6 rad (Abramowitz & Stegun 4.4.49 on the reduced ratio, 2e-8, plus
// float evaluation; tests/test_nnwalk_bounds.py).  (x, y) != (0, 0).
__device__ __forceinline__ float atan2_apx(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float z = fminf(ax, ay) * frcp(fmaxf(ax, ay));
  const float z2 = z * z;
  float p = 0.0028662257f;
  p = p * z2 - 0.0161657367f;
  p = p * z2 + 0.0429096138f;
  p = p * z2 - 0.0752896400f;
  p = p * z2 + 0.1065626393f;
  p = p * z2 - 0.1420889944f;
  p = p * z2 + 0.1999355085f;
  p = p * z2 - 0.3333314528f;
  float a = z + z * z2 * p;
  if (ay > ax) a = 1.57079633f - a;
  if (x < 0.f) a = 3.14159265f - a;
  return y < 0.f ? -a : a;
}

// Lower bound on the float Dubins key (dubins_key) of a node whose rotated offset to the sample,
// (tx, ty >= 0) as dubins_key forms it, lies within pos_err of the given one.  Well outside the turning
// circle (tangent length t >= 0.1) the key is the length of the
// turn-then-straight path, t + rho (thc - acos(rho / dc)) with acos(rho / dc) = atan2(t, rho): a
// function of the offset with gradient norm 1 (continuous outside the circle: thc wraps only inside
// it), so moving the offset by pos_err moves the key by at most pos_err; the margin also covers the
// float evaluation here and in the reference (checked by tests/test_nnwalk_bounds.py).
// The same margin bounds the key from above: lo <= key <= hi (lo = -inf, hi = +inf when undecided).
template <bool BRK>
__device__ __forceinline__ void walk_key_range(float tx, float ty, float pos_err, float& lo, float& hi) {
  const float rho = 4.77f;
  const float t2 = tx * tx + ty * (ty - 2.f * rho);  // dc^2 - rho^2
  if (t2 <= -0.01f) {
    // surely inside the circle: dubins_key's inside branch, rho (alpha + asin(qx / df) - asin(rho sin(alpha)
    // / df)) with alpha = 2 pi - acos((5 rho^2 - df^2) / (4 rho^2)), is >= rho pi = 14.98 anywhere
    lo = 14.9f;
    hi = __builtin_inff();
    if constexpr (BRK) {
      // BRK (large trees, where the inside records' exact keys dominate): a bracket of that branch, restated
      // with atan2: asin(qx / df) = atan2(qx, qy + rho), sin(alpha) = -sqrt(1 - c^2).  Its gradient grows
      // like 1 / sqrt(1 - c^2) and df / sqrt(df^2 - (rho sin alpha)^2): the margin carries those factors,
      // and near their poles the plain rho pi bound stays (tests/test_nnwalk_bounds.py, jittered offsets).
      // On bench-size trees it costs the visits more than it saves (cfg3 0.94 -> 0.89 M nodes/s, round 2).
      const float df2 = tx * tx + (ty + rho) * (ty + rho);
      const float cA = fminf(fmaxf((5.f * rho * rho - df2) * (1.f / (4.f * rho * rho)), -1.f), 1.f);
      const float sA = fsqrt(fmaxf((1.f - cA) * (1.f + cA), 0.f));
      const float u = rho * sA;
      const float w = fsqrt(fmaxf(df2 - u * u, 0.f));
      const float cw = w * frcp(fsqrt(df2));
      if (sA >= 0.05f && cw >= 0.05f) {
        const float alpha = 6.28318531f - atan2_apx(sA, cA);
        const float L = rho * (alpha + atan2_apx(tx, ty + rho) + atan2_apx(u, w));
        const float m = 2e-3f + 1e-4f * L + pos_err * (8.f + 8.f * frcp(sA) + 8.f * frcp(cw));
        lo = fmaxf(L - m, 14.9f);
        hi = L + m;
      }
    }
    return;
  }
  if (!(t2 > -0.01f)) {  // NaN
    lo = -__builtin_inff();
    hi = __builtin_inff();
    return;
  }
  const float t = fsqrt(fmaxf(t2, 0.f));
  float th = atan2_apx(tx, rho - ty);
  if (th < 0.f) th += 6.28318531f;
  const float L = t + rho * (th - atan2_apx(t, rho));
  const float m = 2.f * pos_err + 2e-4f + 2e-5f * L;
  if (t2 >= 0.01f) {  // surely outside (the reference's float inside test errs by ~1e-5)
    lo = L - m;
    hi = L + m;
  } else {
    // near the circle: the outside key (near t = 0 it depends on t only through t^3 / (3 rho^2), so the
    // cancellation in t costs nothing) or, if the reference's point falls inside, the inside key
    lo = fminf(L - m - 1e-4f, 14.9f);
    hi = __builtin_inff();
  }
}

// Lower bound on the keys of a tile's nodes for the sample at (rsx, rsy) (frame coordinates);
// +inf: no node of the tile can enter the list (empty, or feasibleNode fails for all of them);
// -inf: no bound (non-finite records).  flen = feasibility length lower limit.  Angles come from
// acos_apx; each angle test carries 5e-4 rad per approximated term on top of its float margin.
__device__ __forceinline__ float walk_lb(const WalkTile& w, float rsx, float rsy, bool ex, float flen,
                                         float dsR = 0.f) {
  if (w.nonfinite) return -__builtin_inff();
  if (w.pr < 0.f) return __builtin_inff();
  const float rho = 4.77f;
  // feasibility: direction from the ref.back() disc to the sample vs the ang_par arc
  const float ex2 = rsx - w.rcx, ey2 = rsy - w.rcy;
  const float E2 = fsqrt(ex2 * ex2 + ey2 * ey2);
  if (E2 + w.rr < flen) return __builtin_inff();
  if (E2 > w.rr && w.aph < 3.f) {
    const float iE = frcp(E2);
    const float a2 = 1.57079633f - acos_apx(w.rr * iE);  // asin
    const float ang2 = acos_apx((ex2 * w.apx + ey2 * w.apy) * iE);
    if (ang2 - a2 - w.aph > 0.78539816f + 5e-3f) return __builtin_inff();
  }
  const float dx = rsx - w.pcx, dy = rsy - w.pcy;
  const float D = fsqrt(dx * dx + dy * dy);
  float lb = D - w.pr;
  if (D > w.pr && w.thh < 3.f) {
    const float iD = frcp(D);
    const float al = 1.57079633f - acos_apx(w.pr * iD);
    const float bmin = acos_apx((dx * w.thx + dy * w.thy) * iD) - al - w.thh - 3e-3f;
    lb = fmaxf(lb, rho * bmin);
  }
  lb = lb - 2e-3f - 1e-5f * fabsf(lb);
  // optimize: costE + key >= costE + |s - p| >= (costE - |p - c|) + |s - c| for c = the tile centre
  // and for c = R (the root: near-straight branches have costE - |p - R| ~ 0, so only tiles whose
  // branches bend less than the 11th key allows survive)
  if (!ex) lb = fmaxf(fmaxf(w.aopt + D * (1.f - 1e-5f) - 2e-3f, w.cemin + lb), w.eroot + dsR);
  return lb == lb ? lb : -__builtin_inff();
}

// The distance-only part of walk_lb (no feasibility cone, no turning bound): walk_lb >= walk_lb_dist.
#ifndef WALK_CHEAP_FIRST
#define WALK_CHEAP_FIRST 1
#endif
__device__ __forceinline__ float walk_lb_dist(const WalkTile& w, float rsx, float rsy, bool ex, float dsR = 0.f) {
  if (w.nonfinite) return -__builtin_inff();
  if (w.pr < 0.f) return __builtin_inff();
  const float dx = rsx - w.pcx, dy = rsy - w.pcy;
  const float D = fsqrt(dx * dx + dy * dy);
  float lb = D - w.pr;
  lb = lb - 2e-3f - 1e-5f * fabsf(lb);
  if (!ex) lb = fmaxf(fmaxf(w.aopt + D * (1.f - 1e-5f) - 2e-3f, w.cemin + lb), w.eroot + dsR);
  return lb == lb ? lb : -__builtin_inff();
}

// Wave-uniform values kept in scalar registers.
__device__ __forceinline__ float uni(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ bool w_less(float ka, int ia, float kb, int ib) {
  return (ka < kb) || (ka == kb && ia < ib);
}

// The sample's list: lane j < NN_K holds entry j (ascending); insert (k, i) when it precedes entry 10.
__device__ __forceinline__ void w_insert(float& lk, int& li, float k, int i, int lane) {
  const bool before = w_less(lk, li, k, i) && lane < NN_K;  // entries that stay ahead of the new one
  const int pos = __popcll(__ballot(before));
  const float uk = __shfl_up(lk, 1, 64);
  const int ui = __shfl_up(li, 1, 64);
  if (lane < NN_K) {
    if (lane == pos) { lk = k; li = i; }
    else if (lane > pos) { lk = uk; li = ui; }
  }
}

// Writes a sample's list (lanes 0..10, ascending) in k_nn_merge's format: the first min(sortLimit,
// valid entries) node ids, the keys, the count and whether a key tie crosses the selection boundary.
__device__ __forceinline__ void walk_emit(float lk, int li, int lane, int s, int sort_limit, int* __restrict__ cand,
                                          float* __restrict__ ckey, int* __restrict__ ncand, int* __restrict__ ctie) {
  const bool valid = lane < NN_K && li != 0x7fffffff;
  const int nvalid = __popcll(__ballot(valid));
  const int sel = min(sort_limit, nvalid);
  const float nk = __shfl_down(lk, 1, 64);
  const bool tie = lane < CAND_K && lane < sel && lane + 1 < nvalid && lk == nk;
  const bool anytie = __ballot(tie) != 0;
  if (lane < CAND_K) {
    cand[s * CAND_K + lane] = lane < sel ? li : -1;
    ckey[s * CAND_K + lane] = lk;
  }
  if (lane == 0) {
    ncand[s] = sel;
    ctie[s] = anytie;
  }
}

// Stateless bounds in LDS: one byte per super-tile, a lower bound on a log scale (16 codes per octave from
// 2^-4 to 2^12; code 0: no bound, 255: nothing left).  Decoding is monotone, so a bound is compared with a
// threshold in the code domain (lc_le: the largest code that decodes to <= the threshold).
__device__ __forceinline__ float lc_dec(int c) {
  return c == 0 ? -__builtin_inff() : (c == 255 ? __builtin_inff() : exp2f((float)(c - 64) * 0.0625f));
}
__device__ __forceinline__ int lc_enc(float b) {  // the largest code whose value is <= b
  if (b == __builtin_inff()) return 255;
  if (!(b >= lc_dec(1))) return 0;
  int c = (int)floorf(log2f(b) * 16.f) + 64;
  c = c < 1 ? 1 : (c > 254 ? 254 : c);
  while (c > 1 && lc_dec(c) > b) c--;
  while (c < 254 && lc_dec(c + 1) <= b) c++;
  return c;
}
__device__ __forceinline__ int lc_le(float v) {  // the largest code c with lc_dec(c) <= v
  return v == __builtin_inff() ? 255 : lc_enc(v);
}

// One wave per sample.  LDS per super-tile: s_lb = a lower bound (one log-coded byte, rounded down) of the keys in
// its tiles not yet visited.  Pass k visits the tiles whose bound lies in (T_{k-1}, min(T_k, kth)]
// (T_k grows geometrically from the smallest bound; a tile's bound is max(tile bound, super-tile
// bound), so the intervals of successive passes partition the tiles and no per-tile state is kept),
// two tiles of 32 nodes per step (lanes 0-31 / 32-63), so nodes are visited roughly in the order of
// their bounds and the list's 11th key prunes the rest.  The search ends after the first pass whose
// threshold reaches kth: every tile with a bound <= kth has then been visited.  LDS is 1 byte per
// super-tile (16 KB at 16 M nodes: LDS, not registers, sets the walk's occupancy on large trees).
// Tiles taken by the super-tile visits go to a small LDS stack and are visited four at a time (128
// records over the 64 lanes), so the visits' lanes stay busy however few tiles each super-tile gives.
// Waves per SIMD the walk kernels are compiled for: 5 since round 6 (96 VGPRs, 64-128 B/lane of scratch for the
// persistent variants), so two walk waves fit on a SIMD beside a 320-register rollout wave (4: 128 VGPRs, one); with
// a 2304-wave grid cfg3 1.289 -> 1.306-1.310 M nodes/s (profiles/r06r_*, r06s_*).
#ifndef CLRRT_WALK_WAVES
#define CLRRT_WALK_WAVES 5
#endif
// STATE = true (trees up to ~1.3 M nodes): per super-tile a float bound and a visited-tile mask
// (8 bytes) instead of the stateless coded interval scheme, which spends an extra bound per visit.
//
// Overflow.  A round's search lasts as long as its slowest samples, and a few samples need 10-100x
// the median work (optimize samples near the root, where the costE bound is weak: 1e5 exact keys).
// A sample whose walk passes the budget (bud_tiles tiles or bud_ex exact keys; 0 = no budget) claims
// an overflow record (sample, the list's 11th entry) and stops; SPLIT = true then runs nch waves per
// record, wave ch searching the super-tiles ch, ch + nch, ch + 2 nch, ... (interleaved, so the dense
// region near the sample spreads over all of them) with the 11th entry as the initial bound, and
// k_walk_merge takes the 11 smallest (key, node) pairs of the nch partial lists.  Every pair of the
// sample's true list precedes that 11th entry, each wave's list is exact over its super-tiles, so the
// merged list equals the walk's (and the brute force's).  Records beyond max_over: the walk goes on.
template <int FMT, bool SPLIT, bool BRK>
__device__ __forceinline__ void walk_one(const clrrt_sample* __restrict__ S, int B,
                                                    const NnRec* __restrict__ nodes, const float4* __restrict__ P,
                                                    const float4* __restrict__ Q, const float* __restrict__ CE,
                                                    const int* __restrict__ ID, const int* __restrict__ HEAD,
                                                    const int2* __restrict__ trun,
                                                    const WalkTile* __restrict__ tiles, int ntiles,
                                                    const WalkTile* __restrict__ sup, int nsup, DevParams p,
                                                    NnFrame fr, int* __restrict__ cand, float* __restrict__ ckey,
                                                    int* __restrict__ ncand, int* __restrict__ ctie,
                                                    const int* __restrict__ sorder,
                                                    unsigned long long* __restrict__ stats, int bud_tiles,
                                                    int bud_ex, int* __restrict__ ovf_n, int4* __restrict__ ovf,
                                                    int max_over, int nch, float* __restrict__ pk,
                                                    int* __restrict__ pi, int nloc_max, int s, int ch, int nloc, float kb, int ib, int o_sp) {
  // LDS is indexed by the wave's local super-tile index l (super-tile gst(l))
  constexpr bool STATE = FMT == WALK_FMT_STATE, CODED = FMT == WALK_FMT_CODED;
  extern __shared__ uint8_t s_lb[];  // [nloc] bounds of the super-tiles' remaining tiles (stateless) ...
  __half* s_lbh = (__half*)s_lb;             // ... fp16, rounded down, or (CODED) one log-coded byte
  __half* s_sh = s_lbh + nloc_max;           // HALF: the super-tiles' own bounds (phase 1), fp16 rounded down
  float* s_lbf = (float*)s_lb;               // STATE: [nloc] float bounds ...
  uint32_t* s_vis = (uint32_t*)(s_lbf + nloc_max);  // ... and [nloc] visited / discarded tile masks
  __shared__ int s_q2[64];  // records past stage 1 (stage 2: exact keys) ...
  __shared__ float s_b2[64];  // ... and their key lower bounds
#if WALK_STAGE1_QUEUE
  __shared__ int s_q1[192];        // records past the prefilter (stage 1 queue)
#endif
  __shared__ int s_tq[WALK_TQ];    // tile queue: tiles taken by the super-tile visits ...
  __shared__ float s_tb[WALK_TQ];  // ... and their bounds
  const int lane = threadIdx.x;
  // SPLIT: the pairs sought precede (kb, ib); ch / nloc: the wave's interleaved super-tile subset
  auto gst = [&](int l) -> int { return SPLIT ? ch + l * nch : l; };  // super-tile of local index l
  const double sx = S[s].x, sy = S[s].y;
  const bool ex = S[s].explore != 0;
  const float rsx = (float)(sx - fr.ox), rsy = (float)(sy - fr.oy);
  const float dl = fr.delta;
  const float flen = (float)p.feas_len - 2.f * dl;
  const float fl2 = flen > 0.f ? flen * flen : 0.f;
  const float c45 = 0.69276f;  // cos(pi/4 + 0.02), rounded down (see k_nn_partial)
  const float rho = 4.77f, rin = rho - 0.01f - 4.f * dl;
  const float rin2 = rin > 0.f ? rin * rin : -1.f;
  const float flen_t = (float)p.feas_len * (1.f - 1e-5f) - 4.f * dl;
  // |sample - R| for the root-anchored optimize bound (R = node 0, as in k_walk_tiles), rounded down
  const float Rx = (float)(nodes[0].x - fr.ox), Ry = (float)(nodes[0].y - fr.oy);
  const float dsR = sqrtf((rsx - Rx) * (rsx - Rx) + (rsy - Ry) * (rsy - Ry)) * (1.f - 1e-5f) - 2.f * dl - 1e-4f;
  float lk = __builtin_inff();
  int li = 0x7fffffff;
  // lanes 0..10: the 11 smallest key upper bounds (walk_key_range) of visited nodes that are surely
  // feasible; 11 nodes have keys <= uk[10], so no pair with a larger key enters the list
  float uk = __builtin_inff();
  float kth = __builtin_inff();
  int kth_c = 255;    // stateless: lc_le(kth - base)
  float base = 0.f;   // the smallest super-tile bound (pass thresholds and stateless codes are relative to it)
  int idk = 0x7fffffff;
  float lim = __builtin_inff();  // explore: (prune radius + delta)^2
  float cb0 = -2.f;             // explore: cos of the largest heading-to-sample angle a node may have
  int n2 = 0;
#ifdef CLRRT_WALK_PROFILE
  const bool prof = fr.debug == 2;  // diagnostics: per-phase shader clocks into stats[4..8]
#else
  constexpr bool prof = false;
#endif
  uint64_t cyc[4] = {0, 0, 0, 0};   // super bounds, visit_super (incl.), visit4 (incl.), drain
#ifdef CLRRT_WALK_PROFILE
  unsigned long long hist[6] = {0, 0, 0, 0, 0, 0};  // exact keys: gap to the 11th key <= 0, 1e-3, 1e-2, 0.1, more; kth inf
#endif
  int hc = -1;       // run head whose key is known ...
  float kc = 0.f;    // ... and that key
  unsigned long long n_sup = 0, n_tile = 0, n_q = 0, n_ex = 0, n_und = 0, n_sure = 0, n_drop = 0;

  auto refresh = [&]() __attribute__((always_inline)) {
    kth = uni(__shfl(lk, NN_K - 1, 64));
    idk = uni(__shfl(li, NN_K - 1, 64));
    if (SPLIT && w_less(kb, ib, kth, idk)) { kth = kb; idk = ib; }
    const float u10 = uni(__shfl(uk, NN_K - 1, 64));
    if (u10 < kth) { kth = u10; idk = 0x7fffffff; }
#if WALK_SPLIT_SHARE
    if constexpr (SPLIT) {
      // the record's nch waves share their bounds: each one's 11th entry (or u10, or the handed-over entry) bounds
      // the sample's true 11th key, so a pair above the smallest of them enters no list (a key-only bound, ties
      // kept); published with an ordered-int atomicMin (keys are >= 0) in the record's spare word
      int* sh = &ovf[o_sp].w;
      if (lane == 0 && kth < __builtin_inff() && !(kth < 0.f)) atomicMin(sh, kth > 0.f ? __float_as_int(kth) : 0);
      const float shv = __int_as_float(uni(__atomic_load_n(sh, __ATOMIC_RELAXED)));
      if (shv < kth) { kth = shv; idk = 0x7fffffff; }
    }
#endif
    if constexpr (CODED) kth_c = uni(lc_le(kth - base));
    if (kth < __builtin_inff()) {
      const float R = (kth + 2e-4f) * (1.0f / 0.9999f);
      lim = uni(R < 0.f ? -1.f : (R + dl) * (R + dl));
      const float b0 = (kth + 0.01f) * (1.f / rho) + 2e-3f;
      cb0 = uni(b0 < 3.1f ? __cosf(b0) - 1e-4f : -2.f);  // hardware cos (abs error << 1e-4 on [0, pi])
    }
  };
  // Exact keys of the queued records; feasibleNode decided in float where the float angle / length
  // is far (> 1e-4 rad, relative 1e-5) from the limit, else in double as the reference does.  The key
  // of the last record is remembered with its run head (records of one run share their key).
  // Stage 2: the records past stage 1 whose bound still does not exceed the 11th entry; their exact
  // keys are computed once fewer than `room` slots remain (room 64: always).
  auto drain_exact = [&](int room) __attribute__((always_inline)) {
    if (n2 == 0) return;
    {
      const int jj = lane < n2 ? s_q2[lane] : 0;
      const float bb = lane < n2 ? s_b2[lane] : 0.f;
      const bool k2 = lane < n2 && !(bb > kth);
      const uint64_t m2 = __ballot(k2);
      __builtin_amdgcn_wave_barrier();
      if (k2) {
        const int pos = __popcll(m2 & ((1ull << lane) - 1));
        s_q2[pos] = jj;
        s_b2[pos] = bb;
      }
      __builtin_amdgcn_wave_barrier();
      n_drop += n2 - __popcll(m2);
      n2 = __popcll(m2);
      if (n2 == 0 || n2 + room <= 64) return;
    }
    const int nq = n2;
    const uint64_t c0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    n_ex += nq;
    bool c = false;
    float key = 0.f;
    int id = 0, j = 0;
    if (lane < nq) {
      j = s_q2[lane];
      id = ID[j];
      const NnRec& r = nodes[id];
      key = dubins_key(sx, sy, r.x, r.y, r.c, r.s);
      if (!ex) key = r.costE + key;
      if (w_less(key, id, kth, idk)) {
        // feasibleNode in float, exactly as the reference within the float error of a limit
        c = feasible_search(sx, sy, r.bx, r.by, r.ca, r.sa, r.ang_par, p.feas_len);
      }
    }
    // remember the key of the queued record deepest inside a run of equal records (the longest runs,
    // e.g. the root's zero-length children, are the ones whose remaining records this saves)
    {
      const int hd = lane < nq ? HEAD[j] : 0;
      const int depth = lane < nq ? j - hd : -1;
      int best = depth;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
      best = uni(best);
      if (best > 0) {
        const int l = __ffsll((unsigned long long)__ballot(depth == best)) - 1;
        kc = uni(__shfl(key, l, 64));
        hc = uni(__shfl(hd, l, 64));
      }
    }
#ifdef CLRRT_WALK_PROFILE
    if (prof) {  // diagnostics: exact keys by their distance above the 11th key at the drain
      const float gap = key - kth;
      const bool v = lane < nq;
      hist[0] += __popcll(__ballot(v && !(gap > 0.f)));
      hist[1] += __popcll(__ballot(v && gap > 0.f && gap <= 1e-3f));
      hist[2] += __popcll(__ballot(v && gap > 1e-3f && gap <= 1e-2f));
      hist[3] += __popcll(__ballot(v && gap > 1e-2f && gap <= 0.1f));
      hist[4] += __popcll(__ballot(v && gap > 0.1f));
      hist[5] += __popcll(__ballot(v && kth == __builtin_inff()));
    }
#endif
    uint64_t m = __ballot(c);
    while (m) {
      const int l = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const float k = __shfl(key, l, 64);
      const int i = __shfl(id, l, 64);
      if (w_less(k, i, kth, idk)) {
        w_insert(lk, li, k, i, lane);
        refresh();
      }
    }
    n2 = 0;
    if (prof) cyc[3] += __builtin_amdgcn_s_memtime() - c0;
  };
  // Stage 1 (on the visited records that pass the prefilter): key bounds by walk_key_range.  The
  // upper bounds of surely feasible records tighten the 11th entry; the records whose lower bound does
  // not exceed it are queued for the exact keys (stage 2), which run on full waves of them.
  const float f2_sure = fmaxf((float)(p.feas_len * p.feas_len) * 1.002f + 1e-3f, (1e4f * dl) * (1e4f * dl));
  auto stage1 = [&](bool ok, float4 pp, float4 qq, float ce, float& lbt, float& ubt) __attribute__((always_inline)) {
    lbt = __builtin_inff();
    ubt = __builtin_inff();
    if (!ok) return;
    const float qx = rsx - pp.x, qy = rsy - pp.y;
    const float tx = pp.z * qx - pp.w * qy, ty = fabsf(pp.w * qx + pp.z * qy);
    float lo, hi;
    walk_key_range<BRK>(tx, ty, 4.f * dl + 1e-6f * (fabsf(tx) + ty), lo, hi);
    const float cst = ex ? 0.f : ce;  // explore keys carry no cost
    const float tlo = cst + lo, thi = cst + hi;
    lbt = tlo - 1e-6f * fabsf(tlo);
    // feasibleNode surely holds: the frame offset v errs by < 3 delta and |v| >= 1e4 delta, so its
    // direction errs by < 3e-4 rad (the cos^2 margin 0.502 is 2e-3 rad inside pi/4); |v| errs by
    // < 3 delta (the length margin is relative 1e-3 + 1e-3 absolute on |v|^2)
    const float vx = rsx - qq.x, vy = rsy - qq.y;
    const float dot = vx * qq.z + vy * qq.w, vv = vx * vx + vy * vy;
    const bool sure = dot > 0.f && dot * dot >= 0.502f * vv && vv >= f2_sure;
    ubt = sure ? thi + 1e-6f * fabsf(thi) : __builtin_inff();
  };
  // upper bounds below the 11th entry enter the bound list (lanes 0..10)
  auto ub_insert = [&](float ubt) __attribute__((always_inline)) {
    uint64_t mu = __ballot(ubt < kth);
    if (!mu) return false;
    while (mu) {
      const int l = __ffsll((unsigned long long)mu) - 1;
      mu &= mu - 1;
      const float v = __shfl(ubt, l, 64);
      const float u10 = uni(__shfl(uk, NN_K - 1, 64));
      if (v < u10) {
        const int pos = __popcll(__ballot(uk <= v && lane < NN_K));
        const float up = __shfl_up(uk, 1, 64);
        if (lane < NN_K) {
          if (lane == pos) uk = v;
          else if (lane > pos) uk = up;
        }
      }
    }
    return true;
  };
  auto enqueue = [&](bool ok, float lbt, int j) __attribute__((always_inline)) {
    const bool keep = ok && !(lbt > kth);
    const uint64_t m = __ballot(keep);
    const int cnt = __popcll(m);
    if (cnt == 0) return;
    if (n2 + cnt > 64) drain_exact(cnt);
    __builtin_amdgcn_wave_barrier();
    if (keep) {
      const int pos = n2 + __popcll(m & ((1ull << lane) - 1));
      s_q2[pos] = j;
      s_b2[pos] = lbt;
    }
    n2 += cnt;
    __builtin_amdgcn_wave_barrier();
  };
  auto drain = [&]() __attribute__((always_inline)) { drain_exact(64); };
  // Necessary conditions for record j to enter the list (the brute-force prefilter + turning bound).
  auto prefilter = [&](int id, int hd, float4 pp, float4 qq, float ce) __attribute__((always_inline)) -> bool {
    if (hd == hc && !w_less(kc, id, kth, idk)) return false;  // key known: kc
    const float qx = rsx - pp.x, qy = rsy - pp.y;
    const float d2 = qx * qx + qy * qy;
    float l2 = lim;
    if (!ex) {
      const float R = (kth - ce + 2e-4f) * (1.0f / 0.9999f);
      l2 = R < 0.f ? -1.f : (R + dl) * (R + dl);
    }
    if (!(id >= 0 && ((d2 <= l2) || (l2 != l2)))) return false;
    const float vx = rsx - qq.x, vy = rsy - qq.y;
    const float dot = vx * qq.z + vy * qq.w, vv = vx * vx + vy * vy;
    const bool ang_bad = (vv < fl2) || (dot < -1e-3f) || (dot * dot < c45 * c45 * vv && dot >= 0.f);
    const float tx = pp.z * qx - pp.w * qy, ty = fabsf(pp.w * qx + pp.z * qy);
    const bool deep = tx * tx + (ty - rho) * (ty - rho) <= rin2;
    const bool in_bad = deep && !(ex ? (14.9f <= kth) : (ce + 14.9f <= kth));
    bool turn_bad = false;
    if (ex) {
      if (cb0 > -1.5f) {
        const float qn = fsqrt(d2);
        turn_bad = tx + 4.f * dl + 1e-6f * qn < cb0 * qn;
      }
    } else if (kth < __builtin_inff()) {
      // optimize: costE + key <= kth needs rho * beta <= kth - costE (+ margin)
      const float b0 = (kth - ce + 0.01f) * (1.f / rho) + 2e-3f;
      if (b0 < 3.1f) {
        const float cb = __cosf(b0) - 1e-4f;
        const float qn = fsqrt(d2);
        turn_bad = tx + 4.f * dl + 1e-6f * qn < cb * qn;
      }
    }
    return !ang_bad && !in_bad && !turn_bad;
  };
#if WALK_STAGE1_QUEUE
  // Records past the prefilter wait in an LDS stack (their place-order index) and run stage 1 in full
  // waves of 64: most visited records fail the prefilter (84% of an explore sample's on a 16 M-node tree),
  // so stage 1 on the visits' own lanes would run its key brackets for a few lanes at a time.
  int n1 = 0;
  auto push1 = [&](bool ok, int j) __attribute__((always_inline)) {
    const uint64_t m = __ballot(ok);
    if (ok) s_q1[n1 + __popcll(m & ((1ull << lane) - 1))] = j;
    n1 += __popcll(m);
    __builtin_amdgcn_wave_barrier();
  };
  auto run_stage1 = [&](int cnt) __attribute__((always_inline)) {  // the top cnt (<= 64) entries
    const int b0 = n1 - cnt;
    const bool v = lane < cnt;
    const int j = v ? s_q1[b0 + lane] : -1;
    __builtin_amdgcn_wave_barrier();
    n1 = b0;
    float4 pp = make_float4(0.f, 0.f, 1.f, 0.f), qq = pp;
    float ce = 0.f;
    if (v) { pp = P[j]; qq = Q[j]; ce = CE[j]; }
    float lt, ut;
    stage1(v, pp, qq, ce, lt, ut);
    n_und += __popcll(__ballot(lt == -__builtin_inff()));
    n_sure += __popcll(__ballot(ut < __builtin_inff()));
    if (ub_insert(ut)) refresh();
    enqueue(v, lt, j);
  };
#endif
  // nodes of up to four tiles: t0 / t1 on lanes 0-31 / 32-63 (first set), t2 / t3 (second set);
  // -1 = none.  Both sets' records are loaded before either is tested.
  auto visit4 = [&](int t0, int t1, int t2, int t3) __attribute__((always_inline)) {
    const uint64_t c0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    n_tile += (t0 >= 0) + (t1 >= 0) + (t2 >= 0) + (t3 >= 0);
    const int ta = lane < 32 ? t0 : t1, tb = lane < 32 ? t2 : t3;
    const int ja = ta >= 0 ? ta * WALK_TILE + (lane & 31) : -1;
    const int jb = tb >= 0 ? tb * WALK_TILE + (lane & 31) : -1;
    int ida = -1, idb = -1, ha = -2, hb = -2;
    float4 pa = make_float4(0.f, 0.f, 1.f, 0.f), qa = pa, pb = pa, qb = pa;
    float ca = 0.f, cb = 0.f;
    if (ja >= 0) { ida = ID[ja]; ha = HEAD[ja]; pa = P[ja]; qa = Q[ja]; ca = CE[ja]; }
    if (jb >= 0) { idb = ID[jb]; hb = HEAD[jb]; pb = P[jb]; qb = Q[jb]; cb = CE[jb]; }
    const bool oka = prefilter(ida, ha, pa, qa, ca);
    const bool okb = prefilter(idb, hb, pb, qb, cb);
    n_q += __popcll(__ballot(oka)) + __popcll(__ballot(okb));
#if WALK_STAGE1_QUEUE
    push1(oka, ja);
    push1(okb, jb);
    while (n1 >= 64) run_stage1(64);
#else
    float la, ua, lb, ub;
    stage1(oka, pa, qa, ca, la, ua);
    stage1(okb, pb, qb, cb, lb, ub);
    n_und += __popcll(__ballot(la == -__builtin_inff())) + __popcll(__ballot(lb == -__builtin_inff()));
    n_sure += __popcll(__ballot(ua < __builtin_inff())) + __popcll(__ballot(ub < __builtin_inff()));
    const bool ia = ub_insert(ua);
    const bool ib2 = ub_insert(ub);
    if (ia || ib2) refresh();
    enqueue(oka, la, ja);
    enqueue(okb, lb, jb);
#endif
    if (prof) cyc[2] += __builtin_amdgcn_s_memtime() - c0;
  };
  // visit the tiles of super-tile st whose bounds lie in (Tp, min(T, kth)] (pass 0: <= min(T, kth));
  // s_lb[st] becomes the bound of the tiles beyond T
  // half-wave minimum (lanes 0-31 and 32-63 separately)
  auto hmin = [&](float v) -> float {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
  };
  // A tile whose 32 records all belong to the run whose key is known (kc, run head hc), none of them with
  // an id below the tile's smallest, holds no pair that precedes the 11th entry: (kc, min id) >= (kth,
  // idk) stays so as the list only improves.  (The root's zero-length children form runs of 10^4-10^5
  // identical records on large trees; optimize samples' lists fill with their smallest ids.)
  auto run_out = [&](int tl) -> bool {
    const int2 tr = trun[tl];
    return tr.x >= 0 && tr.x == hc && !w_less(kc, tr.y, kth, idk);
  };
  // Tile stack (LDS, WALK_TQ entries: tile, bound), wave-uniform depth.  Tiles the list has pruned since
  // they were pushed are skipped.
  int qn = 0;
  auto next_q = [&]() __attribute__((always_inline)) -> int {
    while (qn > 0) {
      qn--;
      const int t = uni(s_tq[qn]);
      if (!(uni(s_tb[qn]) > kth)) return t;
    }
    return -1;
  };
  auto visit_queue = [&]() __attribute__((always_inline)) {
    const int t0 = next_q();
    const int t1 = next_q();
    const int t2 = next_q();
    const int t3 = next_q();
    if (t0 >= 0) visit4(t0, t1, t2, t3);
    __builtin_amdgcn_wave_barrier();
  };
  auto flush_queue = [&]() __attribute__((always_inline)) {
    while (qn > 0) visit_queue();
#if WALK_STAGE1_QUEUE
    while (n1 > 0) run_stage1(n1 < 64 ? n1 : 64);
#endif
  };
  // visit the tiles of super-tiles sa (lanes 0-31) and sb (lanes 32-63, -1: none) whose bounds lie in
  // (Tp, min(T, kth)] (STATE: not visited yet and <= min(T, kth)); the super-tiles' LDS bounds become
  // those of their tiles beyond T
  auto visit_supers = [&](int la, int lb2, float Tp, float T, bool first) {
    const uint64_t c0 = prof ? __builtin_amdgcn_s_memtime() : 0;
#if WALK_SPLIT_SHARE
    if constexpr (SPLIT) refresh();  // the other waves' bounds
#endif
    n_sup += 1 + (lb2 >= 0);
    const int sa = gst(la), sb = lb2 >= 0 ? gst(lb2) : -1;
    const int lo = lane < 32 ? la : lb2;  // local index (LDS)
    const int st = lane < 32 ? sa : sb;
    const int tl = st * WALK_SUPER + (lane & 31);
    float lb = __builtin_inff();
    uint64_t tm;
    if constexpr (STATE) {
      const uint32_t vis = st >= 0 ? s_vis[lo] : 0xffffffffu;
      if (st >= 0 && tl < ntiles && !((vis >> (lane & 31)) & 1u)) {
#if WALK_CHEAP_FIRST
        // the distance-only part of the bound first: a tile it already places beyond min(T, kth) skips the
        // feasibility / turning terms (their arccosines); the weaker value is still a valid bound for
        // the super-tile's rest (a state tile is never taken twice: visited mask)
        const WalkTile tt = tiles[tl];
        lb = walk_lb_dist(tt, rsx, rsy, ex, dsR);
        if (!(lb > fminf(T, kth))) lb = walk_lb(tt, rsx, rsy, ex, flen_t, dsR);
#else
        lb = walk_lb(tiles[tl], rsx, rsy, ex, flen_t, dsR);
#endif
        if (run_out(tl)) lb = __builtin_inff();
      }
      const bool take = st >= 0 && lb <= T && !(lb > kth);
      const bool drop = st >= 0 && lb > kth;  // never needed again (kth only decreases)
      tm = __ballot(take);
      const uint64_t dm = __ballot(drop);
      const float rest = hmin(take || drop || st < 0 ? __builtin_inff() : lb);
      if ((lane & 31) == 0 && st >= 0) {
        const int sh = lane;  // 0 or 32
        s_vis[lo] = vis | (uint32_t)(tm >> sh) | (uint32_t)(dm >> sh);
        s_lbf[lo] = rest;
      }
    } else {
      float slb;
      if constexpr (FMT == WALK_FMT_HALF && WALK_HALF_SUPER) {
        // the super-tile's own bound, kept from phase 1 (rounded down: still <= every tile's effective bound)
        slb = st >= 0 ? __half2float(s_sh[lo]) : __builtin_inff();
      } else {
        float sl = __builtin_inff();
        if ((lane & 31) == 0 && st >= 0) sl = walk_lb(sup[st], rsx, rsy, ex, flen_t, dsR);
        slb = __shfl(sl, lane & 32, 64);
      }
#ifdef WALK_CHEAP_STATELESS
      // the distance-only bound first; the full one only for tiles it does not place beyond min(T, kth)
      // (the weaker value still bounds the super-tile's rest)
      if (st >= 0 && tl < ntiles) {
        const WalkTile tt = tiles[tl];
        lb = fmaxf(walk_lb_dist(tt, rsx, rsy, ex, dsR), slb);
        if (!(lb > fminf(T, kth))) lb = fmaxf(walk_lb(tt, rsx, rsy, ex, flen_t, dsR), slb);
      }
#else
      if (st >= 0 && tl < ntiles) lb = fmaxf(walk_lb(tiles[tl], rsx, rsy, ex, flen_t, dsR), slb);  // both bound
#endif
      if (st >= 0 && tl < ntiles && run_out(tl)) lb = __builtin_inff();
      const bool take = st >= 0 && (first || lb > Tp) && lb <= T && !(lb > kth);
      tm = __ballot(take);
      const float rest = hmin(st >= 0 && lb > T ? lb : __builtin_inff());
      if ((lane & 31) == 0 && st >= 0) {
        if constexpr (CODED) s_lb[lo] = (uint8_t)lc_enc(rest - base);
        else s_lbh[lo] = __float2half_rd(rest);
      }
    }
    // the taken tiles join the wave's tile queue; full sets of four are visited at once (the lanes of a
    // visit stay busy however few tiles each super-tile gives)
    const bool tk = (tm >> lane) & 1ull;
    if (tk) {
      const int pos = qn + __popcll(tm & ((1ull << lane) - 1));
      s_tq[pos] = st * WALK_SUPER + (lane & 31);
      s_tb[pos] = lb;
    }
    qn += __popcll(tm);
    __builtin_amdgcn_wave_barrier();
    while (qn >= 4) visit_queue();
    if (prof) cyc[1] += __builtin_amdgcn_s_memtime() - c0;
  };

  // 1. super-tile bounds
  const uint64_t ct0 = prof ? __builtin_amdgcn_s_memtime() : 0;
  auto flush_stats = [&]() {
    if (stats && lane == 0) {
      atomicAdd(&stats[0], n_sup);
      atomicAdd(&stats[1], n_tile);
      atomicAdd(&stats[2], n_q);
      atomicAdd(&stats[3], n_ex);
      atomicAdd(&stats[10], n_und);   // stage 1: undecided bounds (near the turning circle)
      atomicAdd(&stats[11], n_sure);  // stage 1: surely feasible (upper bounds)
      atomicAdd(&stats[12], n_drop);  // stage 2: dropped by the refilter
      if (prof) {
        atomicAdd(&stats[4], (unsigned long long)cyc[0]);
        atomicAdd(&stats[5], (unsigned long long)cyc[1]);
        atomicAdd(&stats[6], (unsigned long long)cyc[2]);
        atomicAdd(&stats[7], (unsigned long long)cyc[3]);
        atomicAdd(&stats[8], (unsigned long long)(__builtin_amdgcn_s_memtime() - ct0));
#ifdef CLRRT_WALK_PROFILE
        atomicAdd(&stats[13], hist[0]);  // work_ctr[31]
        for (int q = 1; q < 6; q++) atomicAdd(&stats[14 + q], hist[q]);  // work_ctr[33..37]
#endif
      }
    }
  };
  if (SPLIT) refresh();  // the initial bound
  float mlb = __builtin_inff();
  for (int t0 = 0; t0 < nloc; t0 += 64) {
    const int t = t0 + lane;
    if (t < nloc) {
      const float lb = walk_lb(sup[gst(t)], rsx, rsy, ex, flen_t, dsR);
      if constexpr (STATE) {
        s_lbf[t] = lb;
        s_vis[t] = 0u;
      } else if constexpr (!CODED) {
        s_lbh[t] = __float2half_rd(lb);
        if constexpr (WALK_HALF_SUPER) s_sh[t] = s_lbh[t];
      }
      mlb = fminf(mlb, lb);
    }
  }
  mlb = wmin(mlb);
  base = mlb > 0.f && mlb < __builtin_inff() ? mlb : 0.f;
  if constexpr (CODED) {
    // codes relative to the smallest bound: their resolution (1/16 octave of the distance above it) then
    // follows the pass thresholds' geometric spacing; the bounds are recomputed rather than kept
    for (int t0 = 0; t0 < nloc; t0 += 64) {
      const int t = t0 + lane;
      if (t < nloc) s_lb[t] = (uint8_t)lc_enc(walk_lb(sup[gst(t)], rsx, rsy, ex, flen_t, dsR) - base);
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (prof) cyc[0] += __builtin_amdgcn_s_memtime() - ct0;
  // 2. passes of growing threshold
#ifndef WALK_T0
#define WALK_T0 0.5f
#endif
#ifndef WALK_GROW
#define WALK_GROW 2.f
#endif
  float T = base + WALK_T0, Tp = -__builtin_inff();
  bool budget = !SPLIT && (bud_tiles > 0 || bud_ex > 0);
  for (int pass = 0;; pass++) {
    const float lim_t = fminf(T, kth);
    const int lim_c = CODED ? uni(lc_le(lim_t - base)) : 0;
    for (int t0 = 0; t0 < nloc; t0 += 64) {
      const int t = t0 + lane;
      bool want;
      if constexpr (CODED) {
        const int c = t < nloc ? s_lb[t] : 255;
        want = c != 255 && c <= lim_c;
      } else {
        const float lb = t < nloc ? (STATE ? s_lbf[t] : __half2float(s_lbh[t])) : __builtin_inff();
        want = lb < __builtin_inff() && lb <= lim_t;
      }
      uint64_t m = __ballot(want);
      while (m) {
        // two super-tiles per visit (one per half wave)
        int sa = -1, sb = -1;
        while (m && sb < 0) {
          const int st = t0 + __ffsll((unsigned long long)m) - 1;
          m &= m - 1;
          if (CODED ? (int)s_lb[st] > kth_c : (STATE ? s_lbf[st] : __half2float(s_lbh[st])) > kth) continue;
          if (sa < 0) sa = st; else sb = st;
        }
        if (sa >= 0) visit_supers(sa, sb, Tp, T, pass == 0);
        if (budget && ((bud_tiles > 0 && n_tile > (unsigned long long)bud_tiles) ||
                       (bud_ex > 0 && n_ex > (unsigned long long)bud_ex))) {
          int slot = 0;
          if (lane == 0) slot = atomicAdd(ovf_n, 1);
          slot = uni(__shfl(slot, 0, 64));
          if (slot < max_over) {  // hand over: the split waves and the merge write this sample's list
            if (lane == 0)
              ovf[slot] = make_int4(s, __float_as_int(kth), idk == 0x7fffffff ? idk : idk + 1,
                                    kth > 0.f ? __float_as_int(kth) : kth == 0.f ? 0 : 0x7f800000);  // .w: shared bound
            if (stats && lane == 0) atomicAdd(&stats[14], 1ull);  // overflow records (work_ctr[32])
            flush_stats();
            return;
          }
          budget = false;  // no record left: finish here
        }
      }
    }
    flush_queue();
    drain();
    if (T == __builtin_inff() || kth <= T) break;
    Tp = T;
    T = base + (T - base) * WALK_GROW;
    if (T > 1e7f) T = __builtin_inff();
  }
  // 3. output (k_nn_merge's format); SPLIT: the wave's partial list
  if constexpr (SPLIT) {
    const int o = o_sp;
    if (lane < NN_K) {
      pk[((size_t)o * nch + ch) * NN_K + lane] = lk;
      pi[((size_t)o * nch + ch) * NN_K + lane] = li;
    }
  } else {
    walk_emit(lk, li, lane, s, p.sort_limit, cand, ckey, ncand, ctie);
  }
  flush_stats();
}

// One wave per sample (or, with wctr, a persistent grid of waves taking samples from per-XCD counters: the
// walk then holds a fixed number of wave slots and leaves the rest to the kernels beside it); SPLIT: the
// overflow records' waves.
template <int FMT, bool SPLIT, bool BRK, bool PERS = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(CLRRT_WALK_WAVES))) k_walk_search(const clrrt_sample* __restrict__ S, int B,
                                                    const NnRec* __restrict__ nodes, const float4* __restrict__ P,
                                                    const float4* __restrict__ Q, const float* __restrict__ CE,
                                                    const int* __restrict__ ID, const int* __restrict__ HEAD,
                                                    const int2* __restrict__ trun,
                                                    const WalkTile* __restrict__ tiles, int ntiles,
                                                    const WalkTile* __restrict__ sup, int nsup, DevParams p,
                                                    NnFrame fr, int* __restrict__ cand, float* __restrict__ ckey,
                                                    int* __restrict__ ncand, int* __restrict__ ctie,
                                                    const int* __restrict__ sorder,
                                                    unsigned long long* __restrict__ stats, int bud_tiles,
                                                    int bud_ex, int* __restrict__ ovf_n, int4* __restrict__ ovf,
                                                    int max_over, int nch, float* __restrict__ pk,
                                                    int* __restrict__ pi, int nloc_max, int* __restrict__ wctr) {
  if constexpr (SPLIT) {
    const int o = (int)blockIdx.x / nch;
    const int ch = (int)blockIdx.x % nch;
    if (o >= min(*ovf_n, max_over)) return;
    const int4 rec = ovf[o];
    const int nloc = ch < nsup ? (nsup - ch + nch - 1) / nch : 0;
    walk_one<FMT, SPLIT, BRK>(S, B, nodes, P, Q, CE, ID, HEAD, trun, tiles, ntiles, sup, nsup, p, fr, cand, ckey, ncand, ctie, sorder, stats, bud_tiles, bud_ex, ovf_n, ovf, max_over, nch, pk, pi, nloc_max, rec.x, ch, nloc, __int_as_float(rec.y), rec.z, o);
  } else {
    // XCD-aware: consecutive blocks go to the 8 XCDs in turn; XCD x takes the x-th eighth of the
    // place-ordered samples, so its L2 holds the tree region those samples search (persistent waves then
    // help the other XCDs' eighths)
    const int per = (B + 7) >> 3;
    const int x0 = (int)(blockIdx.x & 7);
    if constexpr (!PERS) {
      const int t = x0 * per + (int)(blockIdx.x >> 3);
      if (t >= B) return;
      walk_one<FMT, SPLIT, BRK>(S, B, nodes, P, Q, CE, ID, HEAD, trun, tiles, ntiles, sup, nsup, p, fr, cand, ckey, ncand,
                                ctie, sorder, stats, bud_tiles, bud_ex, ovf_n, ovf, max_over, nch, pk, pi, nloc_max,
                                sorder[t], 0, nsup, __builtin_inff(), 0x7fffffff, 0);
      return;
    }
    int k = 0;
    for (;;) {
      int t = -1;
      while (k < 8) {
        const int x = (x0 + k) & 7;
        int i = 0;
        if (threadIdx.x == 0) i = atomicAdd(&wctr[x], 1);
        i = __shfl(i, 0, 64);
        if (i < per && x * per + i < B) { t = x * per + i; break; }
        k++;
      }
      if (t < 0) break;
      walk_one<FMT, SPLIT, BRK>(S, B, nodes, P, Q, CE, ID, HEAD, trun, tiles, ntiles, sup, nsup, p, fr, cand, ckey, ncand, ctie, sorder, stats, bud_tiles, bud_ex, ovf_n, ovf, max_over, nch, pk, pi, nloc_max, sorder[t], 0, nsup, __builtin_inff(), 0x7fffffff, 0);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// The 11 smallest (key, node) pairs of an overflow sample's nch partial lists (one wave per record);
// pairs of different waves differ in the node, padding entries (inf, INT_MAX) sort last.
__global__ void __launch_bounds__(64) k_walk_merge(const int* __restrict__ ovf_n, const int4* __restrict__ ovf,
                                                   int max_over, int nch, const float* __restrict__ pk,
                                                   const int* __restrict__ pi, int sort_limit, int* __restrict__ cand,
                                                   float* __restrict__ ckey, int* __restrict__ ncand,
                                                   int* __restrict__ ctie) {
  const int o = blockIdx.x;
  if (o >= min(*ovf_n, max_over)) return;
  const int lane = threadIdx.x;
  const int s = ovf[o].x;
  const int n = nch * NN_K;
  const float* k = pk + (size_t)o * n;
  const int* id = pi + (size_t)o * n;
  float lk = __builtin_inff(), pkey = -__builtin_inff();
  int li = 0x7fffffff, pid = INT_MIN;
  for (int r = 0; r < NN_K; r++) {
    // the smallest pair after (pkey, pid)
    float bk = __builtin_inff();
    int bi = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
      const float kj = k[j];
      const int ij = id[j];
      if (w_less(pkey, pid, kj, ij) && w_less(kj, ij, bk, bi)) { bk = kj; bi = ij; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ok = __shfl_xor(bk, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (w_less(ok, oi, bk, bi)) { bk = ok; bi = oi; }
    }
    if (lane == r) { lk = bk; li = bi; }
    pkey = bk;
    pid = bi;
  }
  walk_emit(lk, li, lane, s, sort_limit, cand, ckey, ncand, ctie);
}

// Diagnostics (clrrt_walk_audit; no product path uses it): for each sample, what any search over this index's tile
// bounds must touch.  The sample's true 11th key kth (brute force over every record, pairs ordered as the lists
// order them) decides which tiles can hold a list member: a tile whose bound (walk_lb, the walk's own bound, max'ed
// with its super-tile's) exceeds kth holds none, so every tile-bound search visits at least the tiles whose bound is
// <= kth ("admissible"), while the tiles that hold a list member -- a feasible record whose (key, id) pair does not
// follow the 11th entry's -- ("useful") are what a perfect tile bound would leave.  out[12 s + q]: q = 0 admissible
// tiles, 1 useful tiles, 2 feasible records with key <= kth (ties included), 3 records of admissible tiles whose
// stage-1 lower bound (walk_key_range) is <= kth -- the exact keys a search knowing kth from its start would
// compute, feasibility aside --, 4 admissible super-tiles, 5 explore flag, 6 kth (float bits), 7 records of
// admissible tiles, and why those records are not members: 8 infeasible, 9 feasible but farther than kth
// (Euclidean), 10 feasible, within kth but key > kth (heading); 11 admissible tiles holding a feasible record with
// key <= kth (ties included); of the admissible tiles: 12 those whose ref.back() disc holds the sample (no
// feasibility cone), 13 / 14 their position / ref.back() disc radii summed (mm), 15 those with an unbounded
// heading or ang_par arc, 16 those inside one run of equal key inputs (trun), 17 their records that are in such a
// run at all (HEAD[j] != j or the next record shares it).
template <bool BRK>
__global__ void __launch_bounds__(64) k_walk_audit(const clrrt_sample* __restrict__ S, int B,
                                                   const NnRec* __restrict__ nodes, const float4* __restrict__ P,
                                                   const float* __restrict__ CE, const int* __restrict__ ID,
                                                   const int* __restrict__ HEAD, const int2* __restrict__ trun,
                                                   const WalkTile* __restrict__ tiles, int ntiles,
                                                   const WalkTile* __restrict__ sup, DevParams p, NnFrame fr,
                                                   int* __restrict__ out) {
  const int s = blockIdx.x, lane = threadIdx.x;
  if (s >= B) return;
  const double sx = S[s].x, sy = S[s].y;
  const bool ex = S[s].explore != 0;
  // 1. the true list's 11th entry (kth, idk): every record's exact key and feasibleNode
  float lk = __builtin_inff(), kth = __builtin_inff();
  int li = 0x7fffffff, idk = 0x7fffffff;
  const int Npad = ntiles * WALK_TILE;
  for (int j0 = 0; j0 < Npad; j0 += 64) {
    const int j = j0 + lane;
    const int idj = ID[j];
    float key = __builtin_inff();
    bool c = false;
    if (idj >= 0) {
      const NnRec& r = nodes[idj];
      key = dubins_key(sx, sy, r.x, r.y, r.c, r.s);
      if (!ex) key = r.costE + key;
      c = w_less(key, idj, kth, idk) && feasible_search(sx, sy, r.bx, r.by, r.ca, r.sa, r.ang_par, p.feas_len);
    }
    uint64_t m = __ballot(c);
    while (m) {
      const int l = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const float k = __shfl(key, l, 64);
      const int i = __shfl(idj, l, 64);
      if (w_less(k, i, kth, idk)) {
        w_insert(lk, li, k, i, lane);
        kth = uni(__shfl(lk, NN_K - 1, 64));
        idk = uni(__shfl(li, NN_K - 1, 64));
      }
    }
  }
  // 2. tiles against kth (the walk's bound terms, as walk_one sets them up)
  const float rsx = (float)(sx - fr.ox), rsy = (float)(sy - fr.oy);
  const float dl = fr.delta;
  const float flen_t = (float)p.feas_len * (1.f - 1e-5f) - 4.f * dl;
  const float Rx = (float)(nodes[0].x - fr.ox), Ry = (float)(nodes[0].y - fr.oy);
  const float dsR = sqrtf((rsx - Rx) * (rsx - Rx) + (rsy - Ry) * (rsy - Ry)) * (1.f - 1e-5f) - 2.f * dl - 1e-4f;
  int n_adm = 0, n_use = 0, n_le = 0, n_s1 = 0, n_sup = 0, n_rec = 0, n_inf = 0, n_far = 0, n_head = 0, n_usele = 0;
  int n_in = 0, n_unb = 0, n_run1 = 0, n_inrun = 0;
  float s_pr = 0.f, s_rr = 0.f;
  for (int t0 = 0; t0 < ntiles / WALK_SUPER; t0 += 64) {
    const int t = t0 + lane;
    const bool a = t < ntiles / WALK_SUPER && !(walk_lb(sup[t], rsx, rsy, ex, flen_t, dsR) > kth);
    n_sup += __popcll(__ballot(a));
  }
  for (int t0 = 0; t0 < ntiles; t0 += 64) {
    const int t = t0 + lane;
    bool adm = false;
    if (t < ntiles) {
      const float lb = fmaxf(walk_lb(tiles[t], rsx, rsy, ex, flen_t, dsR),
                             walk_lb(sup[t / WALK_SUPER], rsx, rsy, ex, flen_t, dsR));
      adm = !(lb > kth);
    }
    uint64_t m = __ballot(adm);
    n_adm += __popcll(m);
    if (adm) {
      const WalkTile& tw = tiles[t];
      const float ex2 = rsx - tw.rcx, ey2 = rsy - tw.rcy;
      const bool in = sqrtf(ex2 * ex2 + ey2 * ey2) <= tw.rr;
      n_in += in;
      n_unb += tw.thh >= 3.f || tw.aph >= 3.f;
      n_run1 += trun[t].x >= 0;
      s_pr += fmaxf(tw.pr, 0.f);
      s_rr += fmaxf(tw.rr, 0.f);
    }
    while (m) {  // two admissible tiles per step (lanes 0-31 / 32-63)
      const int ta = t0 + __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      int tb = -1;
      if (m) {
        tb = t0 + __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
      }
      const int tt = lane < 32 ? ta : tb;
      const int j = tt >= 0 ? tt * WALK_TILE + (lane & 31) : -1;
      const int idj = j >= 0 ? ID[j] : -1;
      bool member = false, le = false, s1 = false, inf = false, far = false, head = false;
      if (idj >= 0) {
        const NnRec& r = nodes[idj];
        float key = dubins_key(sx, sy, r.x, r.y, r.c, r.s);
        if (!ex) key = r.costE + key;
        const bool feas = feasible_search(sx, sy, r.bx, r.by, r.ca, r.sa, r.ang_par, p.feas_len);
        le = !(key > kth) && feas;
        member = feas && (w_less(key, idj, kth, idk) || idj == idk);
        const float ex2 = (float)(sx - r.x), ey2 = (float)(sy - r.y);
        const float dq = sqrtf(ex2 * ex2 + ey2 * ey2) + (ex ? 0.f : r.costE);
        inf = !feas;
        far = feas && !le && dq > kth;
        head = feas && !le && !(dq > kth);
        const float4 pp = P[j];
        const float qx = rsx - pp.x, qy = rsy - pp.y;
        const float tx = pp.z * qx - pp.w * qy, ty = fabsf(pp.w * qx + pp.z * qy);
        float lo, hi;
        walk_key_range<BRK>(tx, ty, 4.f * dl + 1e-6f * (fabsf(tx) + ty), lo, hi);
        const float tlo = (ex ? 0.f : CE[j]) + lo;
        s1 = !(tlo - 1e-6f * fabsf(tlo) > kth);
      }
      const uint64_t mm = __ballot(member), ml = __ballot(le);
      n_use += ((mm & 0xffffffffull) != 0) + ((mm >> 32) != 0);
      n_usele += ((ml & 0xffffffffull) != 0) + ((ml >> 32) != 0);
      n_le += __popcll(ml);
      n_inf += __popcll(__ballot(inf));
      n_far += __popcll(__ballot(far));
      n_head += __popcll(__ballot(head));
      n_s1 += __popcll(__ballot(s1));
      n_rec += __popcll(__ballot(idj >= 0));
      const bool inrun = idj >= 0 && (HEAD[j] != j || (j + 1 < Npad && HEAD[j + 1] == j));
      n_inrun += __popcll(__ballot(inrun));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n_in += __shfl_xor(n_in, o, 64);
    n_unb += __shfl_xor(n_unb, o, 64);
    n_run1 += __shfl_xor(n_run1, o, 64);
    s_pr += __shfl_xor(s_pr, o, 64);
    s_rr += __shfl_xor(s_rr, o, 64);
  }
  if (lane == 0) {
    int* o = out + 20 * (size_t)s;
    o[12] = n_in; o[13] = (int)fminf(s_pr * 1000.f, 2e9f); o[14] = (int)fminf(s_rr * 1000.f, 2e9f); o[15] = n_unb;
    o[16] = n_run1; o[17] = n_inrun; o[18] = 0; o[19] = 0;
    o[0] = n_adm; o[1] = n_use; o[2] = n_le; o[3] = n_s1; o[4] = n_sup; o[5] = ex; o[6] = __float_as_int(kth);
    o[7] = n_rec; o[8] = n_inf; o[9] = n_far; o[10] = n_head; o[11] = n_usele;
  }
}

hipError_t launch_walk_audit(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N, const DevParams& p,
                             const NnFrame& fr, const WalkBufs& w, int* out) {
  if (N <= 0 || B <= 0) return hipSuccess;
  const int Npad = (N + WALK_TILE * WALK_SUPER - 1) / (WALK_TILE * WALK_SUPER) * (WALK_TILE * WALK_SUPER);
  const int ntiles = Npad / WALK_TILE, nsup = ntiles / WALK_SUPER;
  // the stage-1 bracket of the walk format this tree would use (launch_nn_walk_search)
  if (nsup > w.half_max)
    hipLaunchKernelGGL(k_walk_audit<true>, dim3(B), dim3(64), 0, st, S, B, nodes, w.P, w.CE, w.ID, w.HEAD, w.trun,
                       w.tiles, ntiles, w.supers, p, fr, out);
  else
    hipLaunchKernelGGL(k_walk_audit<false>, dim3(B), dim3(64), 0, st, S, B, nodes, w.P, w.CE, w.ID, w.HEAD, w.trun,
                       w.tiles, ntiles, w.supers, p, fr, out);
  LAUNCH_CHECK3();
  return hipSuccess;
}

int64_t walk_tile_count(int64_t n) {
  const int64_t sz = WALK_TILE * WALK_SUPER;
  return (n + sz - 1) / sz * WALK_SUPER;
}
int64_t walk_super_count(int64_t n) { return walk_tile_count(n) / WALK_SUPER; }

size_t walk_sort_bytes(int n) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const int*)nullptr, (int*)nullptr, n, 0, 64);
  size_t b2 = 0;
  hipcub::DeviceScan::InclusiveScan(nullptr, b2, (const int*)nullptr, (int*)nullptr, hipcub::Max(), n + 1024);
  size_t b3 = 0;
  rocprim::merge(nullptr, b3, (const uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                 (const int*)nullptr, (const int*)nullptr, (int*)nullptr, (size_t)n, (size_t)n);
  return std::max(bytes, std::max(b2, b3));
}

// Inclusive max-scan of the run markers in three plain passes (tile scans, one-block scan of the tile
// maxima, fix-up).  A single-pass look-back scan waits on its predecessor blocks, which starves when
// the scan runs beside the rollout kernel (the pipelined rounds) and only a few CUs free up at a time.
#define WSCAN_TILE 1024
__global__ void __launch_bounds__(256) k_wscan_tiles(const int* __restrict__ in, int n, int* __restrict__ out,
                                                     int* __restrict__ tmax) {
  __shared__ int s_w[4];
  const int base = blockIdx.x * WSCAN_TILE + threadIdx.x * 4;
  int v[4];
#pragma unroll
  for (int q = 0; q < 4; q++) v[q] = base + q < n ? in[base + q] : INT_MIN;
#pragma unroll
  for (int q = 1; q < 4; q++) v[q] = max(v[q], v[q - 1]);
  // inclusive scan of the threads' maxima within the wave, then across the 4 waves
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v[3];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x = max(x, y);
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int pre = INT_MIN;
  for (int q = 0; q < wv; q++) pre = max(pre, s_w[q]);
  int ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = INT_MIN;
  ex = max(ex, pre);
#pragma unroll
  for (int q = 0; q < 4; q++)
    if (base + q < n) out[base + q] = max(v[q], ex);
  if (threadIdx.x == 255) tmax[blockIdx.x] = max(x, pre);
}

__global__ void __launch_bounds__(1024) k_wscan_top(int* __restrict__ tmax, int nt) {
  // exclusive max-scan of the tile maxima, one block (sequential chunks per thread)
  __shared__ int s_t[1024];
  const int per = (nt + 1023) / 1024;
  const int b = threadIdx.x * per, e = min(nt, b + per);
  int m = INT_MIN;
  for (int i = b; i < e; i++) m = max(m, tmax[i]);
  s_t[threadIdx.x] = m;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int y = threadIdx.x >= o ? s_t[threadIdx.x - o] : INT_MIN;
    __syncthreads();
    s_t[threadIdx.x] = max(s_t[threadIdx.x], y);
    __syncthreads();
  }
  int run = threadIdx.x > 0 ? s_t[threadIdx.x - 1] : INT_MIN;
  for (int i = b; i < e; i++) {
    const int t = tmax[i];
    tmax[i] = run;
    run = max(run, t);
  }
}

__global__ void __launch_bounds__(256) k_wscan_fix(int* __restrict__ out, int n, const int* __restrict__ tpre) {
  const int t = blockIdx.x;
  if (t == 0) return;
  const int p = tpre[t];
  for (int i = threadIdx.x; i < WSCAN_TILE; i += 256) {
    const int j = t * WSCAN_TILE + i;
    if (j < n) out[j] = max(out[j], p);
  }
}

hipError_t launch_nn_walk(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N, const DevParams& p,
                          const NnFrame& fr, double x0, double y0, double x1, double y1, WalkBufs& w, int* cand,
                          float* ckey, int* ncand, int* ctie, unsigned long long* stats, bool stateless) {
  if (N <= 0 || B <= 0) return hipSuccess;
  hipError_t e = launch_nn_walk_build(st, nodes, N, fr, x0, y0, x1, y1, w);
  if (e != hipSuccess) return e;
  return launch_nn_walk_search(st, S, B, nodes, N, p, fr, x0, y0, x1, y1, w, cand, ckey, ncand, ctie, stats, stateless);
}

// The place-ordered index of nodes [0, N) (Morton sort, gathered records, run heads, tile bounds).
// prev: another buffer set whose sort result covers nodes [0, prev->sorted_n) in the same frame (the
// previous round's index): only the appended nodes are keyed and sorted, then merged with it (nodes
// never change once appended; ties take the older, lower-id entries first, so the order equals a full
// stable sort's).
hipError_t launch_nn_walk_build(hipStream_t st, const NnRec* nodes, int N, const NnFrame& fr, double x0, double y0,
                                double x1, double y1, WalkBufs& w, const WalkBufs* prev) {
  if (N <= 0) return hipSuccess;
  if (N > w.cap_nodes) return hipErrorInvalidValue;  // the buffers' shapes (alloc_walk)
  const int Npad = (N + WALK_TILE * WALK_SUPER - 1) / (WALK_TILE * WALK_SUPER) * (WALK_TILE * WALK_SUPER);
  const int ntiles = Npad / WALK_TILE, nsup = ntiles / WALK_SUPER;
  const int kind = w.index_kind;
  // 3D keys: one metric scale for x, y and rho * angle (2 pi rho = 30 m of the third axis)
  // the 3D codes' third axis: heading (or ang_par) x hrho metres per radian (rho = 4.77 by default, option
  // nn_walk_hscale: percent of rho)
  const double hrho = 4.77 * (w.hscale_pct > 0 ? w.hscale_pct : 100) * 0.01;
  const double span = kind ? fmax(fmax(x1 - x0, y1 - y0), 2.0 * M_PI * hrho) : fmax(x1 - x0, y1 - y0);
  // (kinds 3 / 4 keep the sector on top: the same scale)
  const double scale = span > 0 ? 65535.0 / span : 1.0;
  hipError_t e;
  const bool incremental = prev && prev != &w && prev->sorted_n > 0 && prev->sorted_n <= N &&
                           prev->sorted_x0 == x0 && prev->sorted_y0 == y0 && prev->sorted_scale == scale &&
                           prev->sorted_kind == kind;
  if (incremental) {
    const int n0 = (int)prev->sorted_n, nn = N - n0;
    if (nn > 0) {
      hipLaunchKernelGGL(k_walk_keys, dim3((nn + 63) / 64), dim3(64), 0, st, nodes, N, x0, y0, scale,
                         (uint64_t*)w.keys, w.vals, n0, kind, hrho);
      LAUNCH_CHECK3();
      size_t bytes = w.tmp_bytes;
      e = hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, (const uint64_t*)w.keys, (uint64_t*)w.keys2, w.vals,
                                             w.vals2, nn, 0, 64, st);
      if (e != hipSuccess) return e;
      bytes = w.tmp_bytes;
      e = rocprim::merge(w.tmp, bytes, (const uint64_t*)prev->skeys, (const uint64_t*)w.keys2, w.skeys,
                         (const int*)prev->sids, (const int*)w.vals2, w.sids, (size_t)n0, (size_t)nn,
                         rocprim::less<uint64_t>(), st);
      if (e != hipSuccess) return e;
    } else {
      if ((e = hipMemcpyAsync(w.skeys, prev->skeys, sizeof(uint64_t) * N, hipMemcpyDeviceToDevice, st)) != hipSuccess)
        return e;
      if ((e = hipMemcpyAsync(w.sids, prev->sids, sizeof(int) * N, hipMemcpyDeviceToDevice, st)) != hipSuccess)
        return e;
    }
  } else {
    hipLaunchKernelGGL(k_walk_keys, dim3((N + 63) / 64), dim3(64), 0, st, nodes, N, x0, y0, scale,
                       (uint64_t*)w.keys, w.vals, 0, kind, hrho);
    LAUNCH_CHECK3();
    size_t bytes = w.tmp_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, (const uint64_t*)w.keys, w.skeys, w.vals, w.sids, N, 0, 64,
                                           st);
    if (e != hipSuccess) return e;
  }
  w.sorted_n = N;
  w.sorted_x0 = x0;
  w.sorted_y0 = y0;
  w.sorted_scale = scale;
  w.sorted_kind = kind;
  // one-wave blocks (see launch_nn_delta)
  hipLaunchKernelGGL(k_walk_gather, dim3((Npad + 63) / 64), dim3(64), 0, st, nodes, N, Npad, w.sids, fr.ox, fr.oy,
                     w.P, w.Q, w.CE, w.ID, w.vals);
  LAUNCH_CHECK3();
  // HEAD[j] = first record of j's run of equal key inputs (inclusive max-scan of dup markers)
  {
    const int nt = (Npad + WSCAN_TILE - 1) / WSCAN_TILE;
    int* tmax = (int*)w.keys2;  // free between the two sorts
    hipLaunchKernelGGL(k_wscan_tiles, dim3(nt), dim3(256), 0, st, w.vals, Npad, w.HEAD, tmax);
    LAUNCH_CHECK3();
    hipLaunchKernelGGL(k_wscan_top, dim3(1), dim3(1024), 0, st, tmax, nt);
    LAUNCH_CHECK3();
    hipLaunchKernelGGL(k_wscan_fix, dim3(nt), dim3(256), 0, st, w.HEAD, Npad, tmax);
    LAUNCH_CHECK3();
  }
  hipLaunchKernelGGL(k_walk_trun, dim3((ntiles + 255) / 256), dim3(256), 0, st, w.HEAD, w.ID, ntiles, w.trun);
  LAUNCH_CHECK3();
  hipLaunchKernelGGL(k_walk_tiles, dim3(ntiles), dim3(64), 0, st, w.P, w.Q, w.CE, w.ID, ntiles, WALK_TILE,
                     fr.delta, nodes, fr.ox, fr.oy, w.tiles);
  LAUNCH_CHECK3();
  hipLaunchKernelGGL(k_walk_tiles, dim3(nsup), dim3(64), 0, st, w.P, w.Q, w.CE, w.ID, nsup,
                     WALK_TILE * WALK_SUPER, fr.delta, nodes, fr.ox, fr.oy, w.supers);
  LAUNCH_CHECK3();
  return hipSuccess;
}

// The walk search of samples S[0, B) over the index launch_nn_walk_build made of nodes [0, N).
// Key caps for the appended-node search taken right after the main walk grid (WalkBufs::seed_out: expand_lag2 starts
// that search before the overflow split and its merge have run).  A sample the main grid finished: its sort_limit-th
// key (+inf with fewer); an overflow record's sample, whose list the split's merge writes later: the 11th key it handed
// over, which bounds its final list's (the split only adds candidates).  Both caps bound the final list's from above,
// so no appended node that can enter it is cut (k_nn_partial keeps every key <= its cap).
__device__ __forceinline__ unsigned int w_ord32(float f) {
  const unsigned int b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);  // (clrrt_kernels.hip ord_enc32)
}
__global__ void k_walk_seed(int B, int limit, const float* __restrict__ ckey, const int* __restrict__ ncand,
                            float* __restrict__ seed) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B) return;
  const float k = (limit > 0 && ncand[s] >= limit) ? ckey[s * CAND_K + limit - 1] : __builtin_inff();
  ((unsigned int*)seed)[s] = w_ord32(k);
}
__global__ void k_walk_seed_ovf(const int* __restrict__ ovf_n, const int4* __restrict__ ovf, int max_over,
                                float* __restrict__ seed) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= min(*ovf_n, max_over)) return;
  const int4 rec = ovf[o];
  ((unsigned int*)seed)[rec.x] = w_ord32(__int_as_float(rec.y));
}

hipError_t launch_nn_walk_search(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                 const DevParams& p, const NnFrame& fr, double x0, double y0, double x1, double y1,
                                 WalkBufs& w, int* cand, float* ckey, int* ncand, int* ctie, unsigned long long* stats,
                                 bool stateless) {
  if (N <= 0 || B <= 0) return hipSuccess;
  if (N > w.cap_nodes || B > w.cap_batch) return hipErrorInvalidValue;
  const int Npad = (N + WALK_TILE * WALK_SUPER - 1) / (WALK_TILE * WALK_SUPER) * (WALK_TILE * WALK_SUPER);
  const int ntiles = Npad / WALK_TILE, nsup = ntiles / WALK_SUPER;
  const double span = fmax(x1 - x0, y1 - y0);
  const double scale = span > 0 ? 65535.0 / span : 1.0;
  hipError_t e = hipSuccess;
  size_t bytes = 0;
  // per-sample LDS: 8 B per super-tile with state (while it costs no occupancy), 2 B (fp16) while that costs
  // none, then one coded byte (+ the inside-circle key bracket: on such trees exact keys dominate)
  const int fmt = nsup <= 1280 && !stateless ? WALK_FMT_STATE : (nsup <= w.half_max ? WALK_FMT_HALF : WALK_FMT_CODED);
  const bool brk = fmt == WALK_FMT_CODED;
  // (a floor on it caps the walk's waves per CU, leaving room for the main stream's kernels beside it)
  const size_t lds = std::max<size_t>((size_t)w.lds_floor,
                                      (fmt == WALK_FMT_STATE ? 2 * sizeof(float)
                                       : fmt == WALK_FMT_HALF ? (WALK_HALF_SUPER ? 2 : 1) * sizeof(__half)
                                                              : 1) *
                                          (size_t)nsup);
  const bool pers_k = w.waves > 0 && w.wctr && B >= w.waves_min_batch;
  const void* kfn =
      fmt == WALK_FMT_STATE ? (pers_k ? (const void*)&k_walk_search<WALK_FMT_STATE, false, false, true>
                                      : (const void*)&k_walk_search<WALK_FMT_STATE, false, false, false>)
      : fmt == WALK_FMT_HALF ? (pers_k ? (const void*)&k_walk_search<WALK_FMT_HALF, false, false, true>
                                       : (const void*)&k_walk_search<WALK_FMT_HALF, false, false, false>)
                             : (pers_k ? (const void*)&k_walk_search<WALK_FMT_CODED, false, true, true>
                                       : (const void*)&k_walk_search<WALK_FMT_CODED, false, true, false>);
  if (lds > 64 * 1024) {
    e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const bool split = (w.bud_tiles > 0 || w.bud_ex > 0) && w.max_over > 0 && w.nch > 0 && w.ovf_n;
  const bool pers_z = w.waves > 0 && w.wctr && B >= w.waves_min_batch;
  // samples in place order (radix sort of their Morton keys; the node sort's buffers are free again); the
  // key kernel also resets the overflow count and the persistent grid's counters
  hipLaunchKernelGGL(k_walk_skeys, dim3((B + 255) / 256), dim3(256), 0, st, S, B, x0, y0, scale, w.keys, w.vals,
                     split ? w.ovf_n : nullptr, pers_z ? w.wctr : nullptr);
  LAUNCH_CHECK3();
  bytes = w.tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, w.keys, w.keys2, w.vals, w.sorder, B, 0, 32, st);
  if (e != hipSuccess) return e;
  const int* sorder = w.sorder;
  if (w.lpt && B >= 8) {  // (the sorted keys in keys2 are not read again: its 2 M words hold the new order)
    hipLaunchKernelGGL(k_walk_lpt, dim3(8), dim3(1024), 0, st, S, B, (const int*)w.sorder, (int*)w.keys2);
    LAUNCH_CHECK3();
    sorder = (const int*)w.keys2;
  }
  const int bt = split ? w.bud_tiles : 0, be = split ? w.bud_ex : 0;
  // persistent waves (option nn_walk_waves): a fixed grid taking samples from per-XCD counters
  const bool pers = pers_k;
  const int grid = pers ? std::min(((B + 7) >> 3) * 8, std::max(8, w.waves & ~7)) : ((B + 7) >> 3) * 8;
  int* wctr = pers ? w.wctr : nullptr;
#define WALK_LAUNCH1(F, BK, PS)                                                                                  \
  hipLaunchKernelGGL((k_walk_search<F, false, BK, PS>), dim3(grid), dim3(64), lds, st, S, B, nodes, w.P,          \
                     w.Q, w.CE, w.ID, w.HEAD, w.trun, w.tiles, ntiles, w.supers, nsup, p, fr, cand, ckey, ncand, ctie,  \
                     sorder, stats, bt, be, w.ovf_n, w.ovf, w.max_over, w.nch, w.pk, w.pi, nsup, wctr)
#define WALK_LAUNCH(F, BK)            \
  do {                                \
    if (pers) WALK_LAUNCH1(F, BK, true);  \
    else WALK_LAUNCH1(F, BK, false);  \
  } while (0)
  if (fmt == WALK_FMT_STATE) WALK_LAUNCH(WALK_FMT_STATE, false);
  else if (fmt == WALK_FMT_HALF) WALK_LAUNCH(WALK_FMT_HALF, false);
  else WALK_LAUNCH(WALK_FMT_CODED, true);
#undef WALK_LAUNCH
#undef WALK_LAUNCH1
  LAUNCH_CHECK3();
  if (w.seed_out) {  // the appended-node search's caps, before the split (its records are claimed by now)
    hipLaunchKernelGGL(k_walk_seed, dim3((B + 63) / 64), dim3(64), 0, st, B, p.sort_limit, (const float*)ckey,
                       (const int*)ncand, w.seed_out);
    LAUNCH_CHECK3();
    if (split) {
      hipLaunchKernelGGL(k_walk_seed_ovf, dim3((w.max_over + 63) / 64), dim3(64), 0, st, (const int*)w.ovf_n,
                         (const int4*)w.ovf, w.max_over, w.seed_out);
      LAUNCH_CHECK3();
    }
  }
  if (w.ev_main && (e = hipEventRecord(w.ev_main, st)) != hipSuccess) return e;
  if (split) {
    // the overflow records' split waves (state LDS over their interleaved super-tiles; blocks beyond the
    // claimed records exit at once) and the merge
    const int nl = (nsup + w.nch - 1) / w.nch;
    const void* sfn = brk ? (const void*)&k_walk_search<WALK_FMT_STATE, true, true>
                          : (const void*)&k_walk_search<WALK_FMT_STATE, true, false>;
    if (2 * sizeof(float) * (size_t)nl > 64 * 1024) {
      e = hipFuncSetAttribute(sfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(2 * sizeof(float) * (size_t)nl));
      if (e != hipSuccess) return e;
    }
#define WALK_SPLIT(BK)                                                                                           \
  hipLaunchKernelGGL((k_walk_search<WALK_FMT_STATE, true, BK>), dim3(w.max_over * w.nch), dim3(64),               \
                     2 * sizeof(float) * (size_t)nl, st, S, B, nodes, w.P, w.Q, w.CE, w.ID, w.HEAD, w.trun, w.tiles, \
                     ntiles, w.supers, nsup, p, fr, cand, ckey, ncand, ctie, sorder, stats, 0, 0, w.ovf_n, w.ovf,  \
                     w.max_over, w.nch, w.pk, w.pi, nl, nullptr)
    if (brk) WALK_SPLIT(true);
    else WALK_SPLIT(false);
#undef WALK_SPLIT
    LAUNCH_CHECK3();
    hipLaunchKernelGGL(k_walk_merge, dim3(w.max_over), dim3(64), 0, st, w.ovf_n, w.ovf, w.max_over, w.nch, w.pk, w.pi,
                       p.sort_limit, cand, ckey, ncand, ctie);
    LAUNCH_CHECK3();
  }
  return hipSuccess;
}

}  // namespace clrrt
