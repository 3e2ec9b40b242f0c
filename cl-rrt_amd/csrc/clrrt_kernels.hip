// clrrt_kernels.hip — gfx950 kernels of the expandTree hot path.
//
//   k_nn_partial / k_nn_merge : nearest-node search (sortNodesExplore/Optimize, rrtplanner.cpp:227-268)
//                               lanes = samples, loop over a node chunk with wave-uniform (scalar)
//                               node loads, per-lane top-K in registers, Euclidean prune (key >= |q|)
//   k_rollout                 : closed-loop rollouts (Simulation, simulation.cpp:36-143), one lane per
//                               rollout job; obstacle bounding circles staged in LDS
//   k_select / k_gb_select    : first successful candidate per sample (expandTree :150-160), goal-bias
//                               gate (feasibleGoalBias :292-315) and node construction (:156,170)
//   k_conflict                : EXACT mode — does a node appended earlier in the round reorder a
//                               later sample's candidate list?
//   k_compact                 : prefix scan over committed samples -> node records + arena offsets +
//                               replay jobs (wave ballot / block scan)
//   k_append                  : RRT.addNode for a batch of records (rrtplanner.h:111-113)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stddef.h>
#include <stdint.h>

#include "clrrt_dev.hpp"
#include "clrrt_internal.hpp"
#include "clrrt_stdsort.hpp"

namespace clrrt {

#define CAND_K 10
#define NN_K (CAND_K + 1)  // one extra entry reveals a key tie at the selection boundary
static_assert(CAND_K == 10, "sortLimit");

// --------------------------------------------------------------------------------------------
// nearest-node search
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ bool lex_less(float ka, int ia, float kb, int ib) {
  return (ka < kb) || (ka == kb && ia < ib);
}

// Insert (k, i) into the ascending register list (static indices only: stays in VGPRs).
__device__ __forceinline__ void topk_insert(float (&keys)[NN_K], int (&ids)[NN_K], float k, int i) {
#pragma unroll
  for (int j = 0; j < NN_K; j++) {
    bool sw = lex_less(k, i, keys[j], ids[j]);
    float tk = keys[j];
    int ti = ids[j];
    keys[j] = sw ? k : tk;
    ids[j] = sw ? i : ti;
    k = sw ? tk : k;
    i = sw ? ti : i;
  }
}

// Order-preserving float <-> uint32 (atomicMin over signed floats).
__device__ __forceinline__ unsigned int ord_enc32(float f) {
  unsigned int b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec32(unsigned int u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Prune radius for a lane: a node at Euclidean distance |q| > prune_r(kth - cost) cannot enter the
// list (key >= |q| (1 - 1e-5) - 1e-4 under float rounding, see dubins_key; this radius is looser).
// Negative: nothing can enter.  NaN slack gives NaN (never prunes).
__device__ __forceinline__ float prune_r(float slack) {
  const float r = (slack + 2e-4f) * (1.0f / 0.9999f);
  return r < 0.f ? -1.f : r;
}

// Brute-force candidate lists: block = 256 samples x one chunk of nodes; the chunk is staged through
// LDS 256 nodes at a time (coalesced loads, broadcast reads), each lane keeps its own top-11.
// Per tile, a branch-free float pass over every (lane, node) pair evaluates necessary conditions for
// the node to enter the lane's list on coordinates relative to the frame origin (each coordinate
// difference within fr.delta of the exact one), with margins that cover that error:
//   * Euclidean prune: |q| <= prune_r(kth - cost) + delta;
//   * feasibleNode: |sample - ref.back()| >= feas_len - 2 delta and the angle to ang_par
//     <= pi/4 + 0.02 rad (float error < 5e-3 rad for |v| >= 0.4 m and delta <= 2e-3 m);
//   * not deep inside a turning circle when (cost +) 14.9 > kth (inside -> Dubins key >= rho pi).
// Survivors are queued per lane; a second pass runs nn_prefilter, the exact Dubins key and
// feasibleNode on the queue, so lanes stay converged instead of diverging node by node.
#define NN_QCAP 32
// block sizes of the commit-path kernels that run beside the lag-2 walk (k_select; the appended-node search):
// one-wave blocks would fit the single wave slots the walk frees, but measured (round 4, tools/ab_bench.sh)
// k_select's block size does not matter and one-wave appended-node search blocks (4x the tile staging) cost
// 3% of cfg3's throughput
#ifndef CLRRT_SEL_BLK
#define CLRRT_SEL_BLK 256
#endif
#ifndef CLRRT_PATH_BLK
#define CLRRT_PATH_BLK 256
#endif
__global__ void __launch_bounds__(256) k_nn_partial(const clrrt_sample* __restrict__ S, int B,
                                                    const NnRec* __restrict__ nodes, int N, int chunk,
                                                    int nchunks, DevParams p, NnFrame fr, float* __restrict__ pk,
                                                    int* __restrict__ pi, const float* __restrict__ seed,
                                                    unsigned long long* tstat, const int* __restrict__ sord) {
  int n_queued = 0, n_exact = 0;
  __shared__ float4 s_r[256];   // node x, y and ref.back() x, y relative to the frame origin (float)
  __shared__ double2 s_p[256];  // node x, y
  __shared__ float4 s_f[256];   // c, s, ca, sa
  __shared__ float s_c[256];    // costE
  __shared__ int s_id[256];     // node id
  __shared__ uint8_t s_q[NN_QCAP][256];  // per-lane queue of tile positions (column = lane)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  const int n0 = c * chunk;
  const int n1 = min(N, n0 + chunk);
  const bool act = t < B;
  const int s = act && sord ? sord[t] : t;  // sord: the samples' order over the lanes (k_nn_order)
  double sx = 0, sy = 0;
  int ex = 1;
  if (act) { sx = S[s].x; sy = S[s].y; ex = S[s].explore; }
  const float rsx = (float)(sx - fr.ox), rsy = (float)(sy - fr.oy);
  float keys[NN_K];
  int ids[NN_K];
#pragma unroll
  for (int j = 0; j < NN_K; j++) { keys[j] = __builtin_inff(); ids[j] = 0x7fffffff; }
  const float feas2 = nn_feas2(p.feas_len);
  const float flen = (float)p.feas_len - 2.f * fr.delta;
  const float fl2 = flen > 0.f ? flen * flen : 0.f;
  const float c45 = 0.69276f;                    // cos(pi/4 + 0.02), rounded down
  const float rho = 4.77f, rin = rho - 0.01f - 4.f * fr.delta;  // "deep inside" radius
  const float rin2 = rin > 0.f ? rin * rin : -1.f;
  // kcap: an upper bound on the sample's final 11th key over the whole tree, so the chunk's pruning
  // starts tight: a node with key > kcap cannot be in the merged list.  It starts from the seed pass
  // and is shared between the sample's chunks through gcap[s] (order-preserving uint encoding,
  // atomicMin): every chunk's own 11th key bounds the tree's 11th key too.
  unsigned int* gcap = (unsigned int*)seed;
  float kcap = (seed && act) ? ord_dec32(__atomic_load_n(&gcap[s], __ATOMIC_RELAXED)) : __builtin_inff();
  float rr = __builtin_inff();  // explore: (prune radius + delta)^2 for the current 11th key
  if (kcap < __builtin_inff()) {
    const float R = prune_r(kcap);
    rr = R < 0.f ? -1.f : (R + fr.delta) * (R + fr.delta);
  }
  const int me = threadIdx.x;
  auto drain = [&](int b, int cnt) {
    if (fr.debug == 1) return;
    for (int i = 0; i < cnt; i++) {
      const int k = s_q[i][me];
      const int n = s_id[k];
      // cheap lower bound on the key first (clrrt_dubins_lb.hpp), from the LDS copy of the tile
      const double2 np = s_p[k];
      const float4 f = s_f[k];
      const float cost = s_c[k];
      const float qx = (float)(sx - np.x), qy = (float)(sy - np.y);
      const float tx = f.x * qx - f.y * qy, ty = fabsf(f.y * qx + f.x * qy);
      float lb = dubins_lb(tx, ty);
      if (!ex) lb = cost + lb;
      // kcap bounds the sample's 11th key over all chunks (and, for the appended-node search, the
      // `limit`-th key of the older nodes' list): a key above it cannot be in the merged list
      if (lb > keys[NN_K - 1] || lb > kcap) continue;
      n_exact++;
      float key = dubins_key(sx, sy, np.x, np.y, f.x, f.y);
      if (!ex) key = cost + key;
      if (!lex_less(key, n, keys[NN_K - 1], ids[NN_K - 1]) || key > kcap) continue;
      const NnRec& rec = nodes[b + k];
      if (feasible_search(sx, sy, rec.bx, rec.by, rec.ca, rec.sa, rec.ang_par, p.feas_len)) {
        topk_insert(keys, ids, key, n);
        if (seed && keys[NN_K - 1] < kcap) {
          kcap = keys[NN_K - 1];
          atomicMin(&gcap[s], ord_enc32(kcap));
        }
        const float R = prune_r(fminf(keys[NN_K - 1], kcap));
        rr = R < 0.f ? -1.f : (R + fr.delta) * (R + fr.delta);
      }
    }
  };
  const int tcount = (n1 - n0 + 255) >> 8;
  for (int it = 0; it < tcount; it++) {
    const int b = n0 + (it << 8);
    const int m = min(256, N - b);
    const bool need = act;
    if (seed && act) {  // pick up tighter bounds published by the sample's other chunks
      const float kc = ord_dec32(__atomic_load_n(&gcap[s], __ATOMIC_RELAXED));
      if (kc < kcap) {
        kcap = kc;
        const float R = prune_r(fminf(keys[NN_K - 1], kcap));
        rr = R < 0.f ? -1.f : (R + fr.delta) * (R + fr.delta);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
      const NnRec& rec = nodes[b + i];
      s_r[i] = make_float4((float)(rec.x - fr.ox), (float)(rec.y - fr.oy), (float)(rec.bx - fr.ox),
                           (float)(rec.by - fr.oy));
      s_f[i] = make_float4(rec.c, rec.s, rec.ca, rec.sa);
      s_c[i] = rec.costE;
      s_p[i] = make_double2(rec.x, rec.y);
      s_id[i] = b + i;
    }
    __syncthreads();
    if (!need) continue;
    int cnt = 0;
    const float kth = fminf(keys[NN_K - 1], kcap);
    const bool in_ok = (ex ? 14.9f : -__builtin_inff()) <= kth;  // explore: inside circles can enter
    for (int k0 = 0; k0 < m; k0 += 4) {
      // four nodes per pass: their LDS reads are issued together
      float4 q[4];
      float cst[4];
      bool nr[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int k = min(k0 + u, m - 1);
        q[u] = s_r[k];
        cst[u] = s_c[k];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const float dx = rsx - q[u].x, dy = rsy - q[u].y;
        const float d2 = dx * dx + dy * dy;
        float lim = rr;
        if (!ex) {
          const float R = prune_r(kth - cst[u]);
          lim = R < 0.f ? -1.f : (R + fr.delta) * (R + fr.delta);
        }
        nr[u] = (k0 + u < m) && ((d2 <= lim) || (lim != lim));  // a NaN limit never prunes
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (!nr[u]) continue;
        const int k = k0 + u;
        const float4 f = s_f[k];
        const float dx = rsx - q[u].x, dy = rsy - q[u].y;
        const float vx = rsx - q[u].z, vy = rsy - q[u].w;
        const float dot = vx * f.z + vy * f.w, vv = vx * vx + vy * vy;
        const bool ang_bad = (vv < fl2) || (dot < -1e-3f) || (dot * dot < c45 * c45 * vv && dot >= 0.f);
        const float tx = f.x * dx - f.y * dy, ty = fabsf(f.y * dx + f.x * dy);
        const bool deep = tx * tx + (ty - rho) * (ty - rho) <= rin2;
        const bool in_bad = deep && !(ex ? in_ok : (cst[u] + 14.9f <= kth));
        if (ang_bad || in_bad) continue;
        n_queued++;
        s_q[cnt][me] = (uint8_t)k;
        if (++cnt == NN_QCAP) {
          drain(b, cnt);
          cnt = 0;
        }
      }
    }
    drain(b, cnt);
  }
  if (act) {
    size_t base = ((size_t)s * nchunks + c) * NN_K;
#pragma unroll
    for (int j = 0; j < NN_K; j++) { pk[base + j] = keys[j]; pi[base + j] = ids[j]; }
  }
  if (tstat) {  // diagnostics: queued pairs, exact keys
    atomicAdd(&tstat[2], (unsigned long long)n_queued);
    atomicAdd(&tstat[3], (unsigned long long)n_exact);
  }
}

// Lanes of the appended-node search by heuristic (launch_nn_delta_partial with an order buffer): optimize samples
// (their cost-shifted caps admit many more pairs, each an exact key) first, explore samples after, each class in
// sample order, so a wave's lanes drain queues of similar length.  One block: a stable partition of the B samples.
__global__ void __launch_bounds__(1024) k_nn_order(const clrrt_sample* __restrict__ S, int B, int* __restrict__ out) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int ipt = (B + 1023) >> 10;
  const int i0 = min(B, t * ipt), i1 = min(B, i0 + ipt);
  int c = 0;
  for (int i = i0; i < i1; i++) c += S[i].explore == 0;
  part[t] = c;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int total = part[1023];
  int po = part[t] - c, pe = i0 - po;
  for (int i = i0; i < i1; i++) {
    if (S[i].explore == 0) out[po++] = i;
    else out[total + pe++] = i;
  }
}

__global__ void k_nn_merge(int B, int nchunks, int limit, const float* __restrict__ pk,
                           const int* __restrict__ pi, int* __restrict__ cand, float* __restrict__ ckey,
                           int* __restrict__ ncand, int* __restrict__ ctie) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B) return;
  const int s = t;
  float keys[NN_K];
  int ids[NN_K];
#pragma unroll
  for (int j = 0; j < NN_K; j++) { keys[j] = __builtin_inff(); ids[j] = 0x7fffffff; }
  for (int c = 0; c < nchunks; c++) {
    size_t base = ((size_t)t * nchunks + c) * NN_K;
    for (int j = 0; j < NN_K; j++) {
      int id = pi[base + j];
      if (id == 0x7fffffff) break;
      float k = pk[base + j];
      if (lex_less(k, id, keys[NN_K - 1], ids[NN_K - 1])) topk_insert(keys, ids, k, id);
      else break;  // chunk lists are sorted
    }
  }
  int n = 0, valid = 0;
#pragma unroll
  for (int j = 0; j < NN_K; j++) valid += ids[j] != 0x7fffffff;
  const int sel = min(limit, valid);
  int tie = 0;
#pragma unroll
  for (int j = 0; j < CAND_K; j++) {
    bool v = j < sel;
    cand[s * CAND_K + j] = v ? ids[j] : -1;
    ckey[s * CAND_K + j] = keys[j];
    n += v;
    // equal keys among the selected entries or across the selection boundary: the order std::sort
    // gives them is algorithm-defined (EXACT mode replays it in k_nn_exact)
    tie |= (j < sel && j + 1 < valid && keys[j] == keys[j + 1]);
  }
  ncand[s] = n;
  ctie[s] = tie;
}

// Pipelined BATCH rounds (clrrt_expand): the lists (cand, ckey, ncand) already hold the first `limit`
// feasible nodes of the older nodes [0, id0) in (key, id) order -- the walk search over the tree as it
// was when the previous round's rollouts started -- and the chunk lists pk/pi the top NN_K of the
// nodes that round appended, [id0, id0 + n) (ids relative to id0).  Every appended id is larger than
// every older one, so the first `limit` of the union in (key, id) order -- the list a search over the
// whole tree returns -- are the first `limit` of the two lists' merge.  ctie is not rebuilt exactly
// (the older list's entries past `limit` are not kept); only EXACT mode reads it, and EXACT rounds are
// never pipelined.
// Upper bound for the appended nodes' search: a node whose key exceeds the current list's `limit`-th
// key cannot enter the merged list (every listed node has a smaller id), so it seeds k_nn_partial's
// shared key cap.
__global__ void k_nn_delta_seed(int B, int limit, const float* __restrict__ ckey, const int* __restrict__ ncand,
                                float* __restrict__ seed) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B) return;
  const float k = (limit > 0 && ncand[s] >= limit) ? ckey[s * CAND_K + limit - 1] : __builtin_inff();
  ((unsigned int*)seed)[s] = ord_enc32(k);
}

__global__ void k_nn_merge_delta(int B, int nchunks, int limit, const float* __restrict__ pk,
                                 const int* __restrict__ pi, int id0, int* __restrict__ cand,
                                 float* __restrict__ ckey, int* __restrict__ ncand, int* __restrict__ ctie) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B) return;
  float keys[NN_K];
  int ids[NN_K];
  const int n0 = ncand[s];
#pragma unroll
  for (int j = 0; j < NN_K; j++) {
    const bool v = j < CAND_K && j < n0;
    keys[j] = v ? ckey[s * CAND_K + (j < CAND_K ? j : 0)] : __builtin_inff();
    ids[j] = v ? cand[s * CAND_K + (j < CAND_K ? j : 0)] : 0x7fffffff;
  }
  for (int c = 0; c < nchunks; c++) {
    const size_t base = ((size_t)s * nchunks + c) * NN_K;
    for (int j = 0; j < NN_K; j++) {
      const int id = pi[base + j];
      if (id == 0x7fffffff) break;
      const float k = pk[base + j];
      if (lex_less(k, id + id0, keys[NN_K - 1], ids[NN_K - 1])) topk_insert(keys, ids, k, id + id0);
      else break;  // chunk lists are sorted
    }
  }
  int n = 0, valid = 0;
#pragma unroll
  for (int j = 0; j < NN_K; j++) valid += ids[j] != 0x7fffffff;
  const int sel = min(limit, valid);
  int tie = 0;
#pragma unroll
  for (int j = 0; j < CAND_K; j++) {
    const bool v = j < sel;
    cand[s * CAND_K + j] = v ? ids[j] : -1;
    ckey[s * CAND_K + j] = keys[j];
    n += v;
    tie |= (j < sel && j + 1 < valid && keys[j] == keys[j + 1]);
  }
  ncand[s] = n;
  ctie[s] = tie;
}

// EXACT mode, samples whose candidate selection involves equal keys: rebuild the full (id, key)
// sequence in node order and replay libstdc++'s std::sort on it (one lane per sample), then walk it
// exactly as sortNodesExplore/Optimize do (rrtplanner.cpp:237-243).
__global__ void k_nn_exact(const clrrt_sample* __restrict__ S, int B, const NnRec* __restrict__ nodes, int N,
                           DevParams p, const int* __restrict__ ctie, KeyId* __restrict__ scratch,
                           int* __restrict__ cand, float* __restrict__ ckey, int* __restrict__ ncand) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B || !ctie[s]) return;
  const double sx = S[s].x, sy = S[s].y;
  const int ex = S[s].explore;
  KeyId* a = scratch + (size_t)s * N;
  for (int n = 0; n < N; n++) {
    const NnRec& rec = nodes[n];
    float k = dubins_key(sx, sy, rec.x, rec.y, rec.c, rec.s);
    if (!ex) k = rec.costE + k;
    a[n].id = n;
    a[n].key = k;
  }
  std_sort(a, N);
  int cnt = 0;
  for (int i = 0; i < N && cnt < p.sort_limit; i++) {
    const NnRec& rec = nodes[a[i].id];
    if (feasible_search(sx, sy, rec.bx, rec.by, rec.ca, rec.sa, rec.ang_par, p.feas_len)) {
      cand[s * CAND_K + cnt] = a[i].id;
      ckey[s * CAND_K + cnt] = a[i].key;
      cnt++;
    }
  }
  for (int j = cnt; j < CAND_K; j++) cand[s * CAND_K + j] = -1;
  ncand[s] = cnt;
}

// std_sort (clrrt_stdsort.hpp: libstdc++'s introsort) replayed by one 64-lane wave (a workgroup of 64)
// on an LDS array, the same permutation.  The introsort's control (median-of-three, the explicit range
// stack, the depth limit's heapsort, the final insertion sort) runs as in std_sort (the data moves of
// the pivot choice, the heapsort and the insertion sort on lane 0); the partition is parallel.
// __unguarded_partition's left scan stops at the positions L_0 < L_1 < ... with !(a < pivot) and its
// right scan at R_0 > R_1 > ... with !(pivot < a), both on the range as it was (a swap only changes
// positions the scans have passed); it swaps (L_k, R_k) while L_k < R_k and returns, at the first k
// with L_k >= R_k, L_k if L_k < R_{k-1} (else the left scan stops at the swapped R_{k-1}).  The wave
// finds the stops 64 positions at a time from both ends, pairs them, and swaps the pairs (disjoint) once
// the crossing is known.  pairs: LDS scratch of n / 2 + 64 int2.
// need: only positions [0, need) of the result are read.  libstdc++ recurses on the right part
// [cut, last) and loops on the left one; a right part that starts at or past `need` is left unsorted:
// its elements are >= every element before `cut`, and neither its recursion nor the final insertion
// sort (an element moves left only past strictly greater ones) changes a position before `cut`, so
// positions [0, need) come out as in the full sort.
__device__ __forceinline__ void wave_std_sort(KeyId* a, int n, int2* pairs, int need = INT_MAX) {
  const int lane = threadIdx.x & 63;
  if (n <= 1) return;
  int lim = n;  // positions [0, lim) are sorted as std::sort sorts them
  struct Rg { int lo, hi, depth; };
  Rg stack[64];
  int sp = 0;
  int lo = 0, hi = n;
  int depth = 2 * ilog2(n);
  __shared__ int s_l[64], s_r[64];  // pending stop positions of the two scans
  for (;;) {
    while (hi - lo > 16) {
      if (depth == 0) {
        if (lane == 0) heap_sort_(a + lo, hi - lo);
        __syncthreads();
        break;
      }
      --depth;
      if (lane == 0) {
        KeyId* first = a + lo;
        KeyId* last = a + hi;
        median_to_first_(first, first + 1, first + (last - first) / 2, last - 1);
      }
      __syncthreads();
      const float P = a[lo].key;
      const int f = lo + 1, l = hi;
      int lpos = f, rpos = l - 1;  // next positions the scans examine
      int nl = 0, hl = 0, nr = 0, hr = 0;  // pending stops (count, head) of each scan
      int np = 0;                  // pairs recorded
      int prevR = INT_MAX;         // R_{k-1}
      int cut = -1;
      while (cut < 0) {
        if (nl == 0) {  // the next 64 positions of the left scan
          const int i = lpos + lane;
          const bool st = i < l && !(a[i].key < P);
          const uint64_t m = __ballot(st);
          if (st) s_l[__popcll(m & ((1ull << lane) - 1))] = i;
          nl = __popcll(m);
          hl = 0;
          lpos += 64;
        }
        if (nr == 0) {  // the next 64 positions of the right scan, downwards
          const int i = rpos - lane;
          const bool st = i >= f && !(P < a[i].key);
          const uint64_t m = __ballot(st);
          if (st) s_r[__popcll(m & ((1ull << lane) - 1))] = i;
          nr = __popcll(m);
          hr = 0;
          rpos -= 64;
        }
        __syncthreads();
        const bool lend = nl == 0 && lpos >= l, rend = nr == 0 && rpos < f;  // a scan ran out of range
        const int m = min(nl, nr);
        int Lk = INT_MAX, Rk = INT_MIN;
        bool cross = false;
        if (lane < m) {
          Lk = s_l[hl + lane];
          Rk = s_r[hr + lane];
          cross = Lk >= Rk;
        }
        const uint64_t cm = __ballot(cross);
        const int kx = cm ? __ffsll((unsigned long long)cm) - 1 : m;  // pairs before the crossing
        if (lane < kx) pairs[np + lane] = make_int2(Lk, Rk);
        const int prev = kx > 0 ? __shfl(Rk, kx - 1, 64) : prevR;
        if (cm) {
          const int Lx = __shfl(Lk, kx, 64);
          cut = Lx < prev ? Lx : prev;
        } else if ((nl - m == 0 && lend) || (nr - m == 0 && rend)) {
          // a scan has no further stop in range: the sequential scans would meet the last swap
          // (a missing L_k: the left scan stops at R_{k-1}; a missing R_k: the right scan stops at L_{k-1}
          // and the left scan's next stop L_k, if any, is returned unless past R_{k-1})
          if (nl - m > 0) {
            const int Lx = s_l[hl + m];
            cut = Lx < prev ? Lx : prev;
          } else {
            cut = prev == INT_MAX ? l : prev;
          }
        }
        np += kx;
        prevR = prev;
        nl -= m; hl += m;
        nr -= m; hr += m;
        __syncthreads();
      }
      for (int k = lane; k < np; k += 64) {  // the swaps (disjoint positions)
        const int2 pr = pairs[k];
        const KeyId t = a[pr.x];
        a[pr.x] = a[pr.y];
        a[pr.y] = t;
      }
      __syncthreads();
      if (cut < need) stack[sp++] = Rg{cut, hi, depth};
      else lim = min(lim, cut);
      hi = cut;
    }
    if (sp == 0) break;
    --sp;
    lo = stack[sp].lo;
    hi = stack[sp].hi;
    depth = stack[sp].depth;
  }
  // __final_insertion_sort (elements only move within the final partitions: lane 0)
  if (lane == 0) {
    if (n > 16) {
      insertion_sort_(a, a + 16);
      for (KeyId* i = a + 16; i < a + lim; ++i) unguarded_linear_insert_(i);
    } else {
      insertion_sort_(a, a + n);
    }
  }
  __syncthreads();
}

// The same for trees whose (id, key) sequence fits in LDS: one workgroup (one wave) per sample; the 64
// lanes build the keys, replay std::sort on the LDS copy (wave_std_sort), and test feasibleNode on 64
// sorted entries at a time, the first `sort_limit` feasible ones in sorted order forming the list.
#define NN_EXACT_LDS_MAX 12000  /* entries: 8 B each + 4 B of partition pairs: 144 KB of dynamic LDS */
__global__ void __launch_bounds__(64) k_nn_exact_lds(const clrrt_sample* __restrict__ S, int B,
                                                     const NnRec* __restrict__ nodes, int N, DevParams p,
                                                     const int* __restrict__ ctie, int* __restrict__ cand,
                                                     float* __restrict__ ckey, int* __restrict__ ncand) {
  extern __shared__ KeyId s_kv[];
  int2* s_pairs = (int2*)(s_kv + N);  // [N / 2 + 64]
  const int s = blockIdx.x;
  if (s >= B || !ctie[s]) return;
  const int lane = threadIdx.x;
  const double sx = S[s].x, sy = S[s].y;
  const int ex = S[s].explore;
  for (int n = lane; n < N; n += 64) {
    const NnRec& rec = nodes[n];
    float k = dubins_key(sx, sy, rec.x, rec.y, rec.c, rec.s);
    if (!ex) k = rec.costE + k;
    s_kv[n].id = n;
    s_kv[n].key = k;
  }
  __syncthreads();
  wave_std_sort(s_kv, N, s_pairs);
  int cnt = 0;
  for (int i0 = 0; i0 < N && cnt < p.sort_limit; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    KeyId e{0, 0.f};
    if (i < N) {
      e = s_kv[i];
      const NnRec& rec = nodes[e.id];
      f = feasible_search(sx, sy, rec.bx, rec.by, rec.ca, rec.sa, rec.ang_par, p.feas_len);
    }
    const uint64_t m = __ballot(f);
    // the first (sort_limit - cnt) feasible entries of this chunk, in sorted order
    const int rank = cnt + __popcll(m & ((1ull << lane) - 1));
    if (f && rank < p.sort_limit) {
      cand[s * CAND_K + rank] = e.id;
      ckey[s * CAND_K + rank] = e.key;
    }
    cnt = min(p.sort_limit, cnt + __popcll(m));
  }
  for (int j = cnt + lane; j < CAND_K; j += 64) cand[s * CAND_K + j] = -1;
  if (lane == 0) ncand[s] = cnt;
}

// EXACT-mode lists of a tree that fits in LDS, one wave per sample, in one kernel: every node's key (and
// feasibleNode, kept in the id's top bit) into LDS; the first NN_K feasible entries in (key, id) order
// (per-lane top lists merged across the wave) give the list as the brute force gives it, with its tie
// flag; a tied sample replays std::sort on the LDS array (only the positions up to the last key <= the
// list's `sort_limit`-th key are needed) and walks the sorted order for the first `sort_limit` feasible
// entries (rrtplanner.cpp:227-268), exactly as k_nn_exact_lds does after the brute force.
// xrec / xcnt / slist (EXACT fix-ups, k_conflict_fix): block b searches sample slist[b] over the tree's N nodes
// followed by the first xcnt[b] records of xrec (the nodes the round appends before that sample, as they will
// stand in the tree: ids N, N + 1, ...) and writes its list at row b; Nlds = the LDS entries allotted per block.
__global__ void __launch_bounds__(64) k_nn_exact_fused(const clrrt_sample* __restrict__ S, int B,
                                                       const NnRec* __restrict__ nodes, int N0, DevParams p,
                                                       int* __restrict__ cand, float* __restrict__ ckey,
                                                       int* __restrict__ ncand, int* __restrict__ ctie,
                                                       const NnRec* __restrict__ xrec = nullptr,
                                                       const int* __restrict__ xcnt = nullptr,
                                                       const int* __restrict__ slist = nullptr, int Nlds = 0) {
  extern __shared__ KeyId s_kv[];
  int2* s_pairs = (int2*)(s_kv + (slist ? Nlds : N0));  // [N / 2 + 64]
  const int b = blockIdx.x;
  if (b >= B) return;
  const int s = slist ? slist[b] : b;  // the sample
  const int ob = slist ? b : s;        // its output row
  const int N = N0 + (xcnt ? xcnt[b] : 0);
  cand += (ob - s) * CAND_K;
  ckey += (ob - s) * CAND_K;
  ncand += ob - s;
  ctie += ob - s;
  const int lane = threadIdx.x;
  const double sx = S[s].x, sy = S[s].y;
  const int ex = S[s].explore;
  float tk[NN_K];
  int ti[NN_K];
#pragma unroll
  for (int j = 0; j < NN_K; j++) { tk[j] = __builtin_inff(); ti[j] = 0x7fffffff; }
  for (int n = lane; n < N; n += 64) {
    const NnRec& rec = n < N0 ? nodes[n] : xrec[n - N0];
    float k = dubins_key(sx, sy, rec.x, rec.y, rec.c, rec.s);
    if (!ex) k = rec.costE + k;
    const bool f = feasible_search(sx, sy, rec.bx, rec.by, rec.ca, rec.sa, rec.ang_par, p.feas_len);
    s_kv[n].id = f ? n : (int)((uint32_t)n | 0x80000000u);
    s_kv[n].key = k;
    if (f && lex_less(k, n, tk[NN_K - 1], ti[NN_K - 1])) topk_insert(tk, ti, k, n);
  }
  // wave merge of the lanes' sorted lists: NN_K times the (key, id)-smallest head
  float keys[NN_K];
  int ids[NN_K];
  int h = 0;
#pragma unroll
  for (int j = 0; j < NN_K; j++) {
    float hk = __builtin_inff();
    int hi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < NN_K; q++)
      if (q == h) { hk = tk[q]; hi = ti[q]; }
    float bk = hk;
    int bi = hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ok = __shfl_xor(bk, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (lex_less(ok, oi, bk, bi)) { bk = ok; bi = oi; }
    }
    keys[j] = bk;
    ids[j] = bi;
    if (bi != 0x7fffffff && hi == bi) h++;  // the owner's head moves on (ids are unique)
  }
  int valid = 0;
#pragma unroll
  for (int j = 0; j < NN_K; j++) valid += ids[j] != 0x7fffffff;
  const int sel = min(p.sort_limit, valid);
  int tie = 0;
#pragma unroll
  for (int j = 0; j < CAND_K; j++) tie |= (j < sel && j + 1 < valid && keys[j] == keys[j + 1]);
  if (!tie) {  // the (key, id) order is std::sort's on these entries
    if (lane < CAND_K) {
      float kk = 0.f;
      int ii = -1;
#pragma unroll
      for (int j = 0; j < CAND_K; j++)
        if (j == lane) { kk = keys[j]; ii = j < sel ? ids[j] : -1; }
      cand[s * CAND_K + lane] = ii;
      ckey[s * CAND_K + lane] = kk;
    }
    if (lane == 0) { ncand[s] = sel; ctie[s] = 0; }
    return;
  }
  // Only the order of equal keys is std::sort's: KT = the largest key of a tie in the list (list entry j and the
  // next feasible entry equal).  Every feasible entry with key <= KT takes its place from the replay, which
  // needs positions [0, need), need = the entries with key <= KT; the list's entries above KT have keys no other
  // feasible entry shares (a neighbour with an equal key would make theirs a tie <= KT), so they follow in key
  // order.  (Round 4 replayed up to the sort_limit-th key, and the whole array when fewer entries were feasible:
  // hundreds of microseconds per tied sample on one lane's final insertion sort.)
  float KT = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < CAND_K; j++)
    if (j < sel && j + 1 < valid && keys[j] == keys[j + 1]) KT = keys[j];  // (ascending: the last is the largest)
  int need, nan = 0;
  {
    int c = 0;
    for (int n = lane; n < N; n += 64) {
      const float k = s_kv[n].key;
      c += !(KT < k);
      nan |= k != k;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c += __shfl_xor(c, o, 64);
      nan |= __shfl_xor(nan, o, 64);
    }
    need = nan ? N : c;  // (a NaN key has no place in the order: the whole replay, and the walk below covers all)
  }
  __syncthreads();
  wave_std_sort(s_kv, N, s_pairs, need);
  int cnt = 0;
  for (int i0 = 0; i0 < need && cnt < p.sort_limit; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    KeyId e{0, 0.f};
    if (i < need) {
      e = s_kv[i];
      f = e.id >= 0;
    }
    const uint64_t m = __ballot(f);
    const int rank = cnt + __popcll(m & ((1ull << lane) - 1));
    if (f && rank < p.sort_limit) {
      cand[s * CAND_K + rank] = e.id;
      ckey[s * CAND_K + rank] = e.key;
    }
    cnt = min(p.sort_limit, cnt + __popcll(m));
  }
  if (!nan) {  // the list's entries above KT, in key order
#pragma unroll
    for (int j = 0; j < CAND_K; j++) {
      if (j < sel && KT < keys[j] && cnt < p.sort_limit) {
        if (lane == 0) {
          cand[s * CAND_K + cnt] = ids[j];
          ckey[s * CAND_K + cnt] = keys[j];
        }
        cnt++;
      }
    }
  }
  for (int j = cnt + lane; j < CAND_K; j += 64) cand[s * CAND_K + j] = -1;
  if (lane == 0) { ncand[s] = cnt; ctie[s] = 1; }
}

// EXACT-mode tie replay for the samples with ctie set: in LDS when the tree fits, else one lane per
// sample over the global scratch.
static hipError_t launch_nn_exact_any(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                      const DevParams& p, const int* ctie, KeyId* scratch, int* cand, float* ckey,
                                      int* ncand) {
  if (N <= NN_EXACT_LDS_MAX) {
    const size_t lds = sizeof(KeyId) * (size_t)N + sizeof(int2) * (size_t)(N / 2 + 64);
    if (lds > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute((const void*)&k_nn_exact_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_nn_exact_lds, dim3(B), dim3(64), lds, st, S, B, nodes, N, p, ctie, cand, ckey, ncand);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_nn_exact, dim3((B + 63) / 64), dim3(64), 0, st, S, B, nodes, N, p, ctie, scratch, cand, ckey,
                     ncand);
  return hipGetLastError();
}

// --------------------------------------------------------------------------------------------
// rollouts
// --------------------------------------------------------------------------------------------
struct ObsView {
  const BakedObs* __restrict__ g;  // global baked records
  const float4* cv;                // LDS: (cx, cy, vx, vy) float
  const float* rad;                // LDS: bounding radius + vehicle radius + margin
  const float4* ob;                // LDS: box axis (ux, uy) and half extents (+ rounding slack)
  const float4* sat;               // LDS: static obstacles' SAT vertices and normals (vx, vy, nx, ny)
  const uint32_t* gstart;          // LDS: grid cell -> first item (gw*gh + 1)
  const uint16_t* gitems;          // LDS: static obstacle ids per cell, ascending
  const uint16_t* gmov;            // LDS: moving obstacle ids, ascending
  int n;                           // obstacles (0: collision checking off)
  int gw, gh, nmov;                // grid shape (gw == 0: no grid), moving obstacles
  float gx0, gy0, ginv;            // grid origin and 1 / cell size
};

#define VEH_RAD 2.6220219f  /* sqrt(2.424^2 + 1^2), vehicle half-diagonal */
#define CULL_MARGIN 0.05f

// One obstacle against the vehicle box: bounding-circle cull (no overlap possible when the
// circles are apart), then the SAT gap.
// Vehicle bounding circle (VEH_RAD + margin around the box centre) against the obstacle box (with
// slack): apart -> the two boxes cannot overlap.  (The grid lists already come from this test at the
// cell level, so the bounding-circle pre-test of the brute-force path is not repeated.)
__device__ __forceinline__ bool obs_culled(const ObsView& ov, int j, float ft, float fvx, float fvy) {
  float4 q = ov.cv[j];
  float dx = q.x + q.z * ft - fvx, dy = q.y + q.w * ft - fvy;
  const float4 b = ov.ob[j];
  const float e1 = fmaxf(fabsf(dx * b.x + dy * b.y) - b.z, 0.f);
  const float e2 = fmaxf(fabsf(dy * b.x - dx * b.y) - b.w, 0.f);
  const float vr = VEH_RAD + CULL_MARGIN;
  return e1 * e1 + e2 * e2 > vr * vr;
}

// A static obstacle's SAT from the LDS copy of its vertices / normals (no global load inside the
// step loop: with the step's row stores in flight, a global load would wait for all of them).
__device__ __forceinline__ float obs_sat_static(const Box4& veh, const ObsView& ov, int j) {
  const float4 a = ov.sat[4 * j], b = ov.sat[4 * j + 1], c = ov.sat[4 * j + 2], d = ov.sat[4 * j + 3];
  const float vx[4] = {a.x, a.y, a.z, a.w}, vy[4] = {b.x, b.y, b.z, b.w};
  const float nx[4] = {c.x, c.y, c.z, c.w}, ny[4] = {d.x, d.y, d.z, d.w};
  return sat_gap(veh, vx, vy, nx, ny);
}

__device__ __forceinline__ float obs_sat(const Box4& veh, const ObsView& ov, int j, double t) {
  return obs_sat_baked(veh, ov.g[j], t);
}

__device__ __forceinline__ float obs_gap(const Box4& veh, const ObsView& ov, int j, double t, float ft,
                                         float fvx, float fvy, bool cull, bool& culled) {
  culled = false;
  if (cull) {
    float4 q = ov.cv[j];
    float dx = q.x + q.z * ft - fvx, dy = q.y + q.w * ft - fvy;
    float rr = ov.rad[j];
    if (dx * dx + dy * dy > rr * rr) { culled = true; return 1.0f; }
    // vehicle bounding circle against the obstacle box: apart -> no overlap possible
    const float4 b = ov.ob[j];
    const float e1 = fmaxf(fabsf(dx * b.x + dy * b.y) - b.z, 0.f);
    const float e2 = fmaxf(fabsf(dy * b.x - dx * b.y) - b.w, 0.f);
    const float vr = VEH_RAD + CULL_MARGIN;
    if (e1 * e1 + e2 * e2 > vr * vr) { culled = true; return 1.0f; }
  }
  return obs_sat_baked(veh, ov.g[j], t);
}

// checkObsDistance (stub collisioncheck.cpp:6-8 | OBB old_collisioncheck.cpp:24-51).
// Without the gap value (NEED_GAP false) only obstacles whose inflated bounding circle can reach
// the vehicle are tested: static ones come from the uniform grid cell of the vehicle centre (its
// list is a superset of every obstacle whose circle test can pass anywhere in the cell), moving
// ones from their own list; both lists ascend, and they are merged so the first overlap found is
// the reference's first overlap in obstacle order.  `tests` counts the reference's box tests.
template <bool NEED_GAP>
__device__ __forceinline__ double obs_distance(const Roll& r, const DevParams& p, const ObsView& ov,
                                               uint32_t& tests) {
  if (p.coll_mode == CLRRT_COLLISION_STUB) return 100.0;
  const double t = p.obs_use_pred ? r.x6 : 0.0;
  const double vpx = r.x0 + 1.424 * r.c2, vpy = r.x1 + 1.424 * r.s2;
  const float fvx = (float)vpx, fvy = (float)vpy, ft = (float)t;
  Box4 veh;
  if (!NEED_GAP && ov.gw > 0 && isfinite(fvx) && isfinite(fvy) && isfinite(ft)) {
    bool have_veh = false;  // the vehicle box (setVertices) is built only when an obstacle survives the cull
    int a = 0, ae = 0;
    const int gx = (int)floorf((fvx - ov.gx0) * ov.ginv), gy = (int)floorf((fvy - ov.gy0) * ov.ginv);
    if (gx >= 0 && gx < ov.gw && gy >= 0 && gy < ov.gh) {
      const int cell = gy * ov.gw + gx;
      a = ov.gstart[cell];
      ae = ov.gstart[cell + 1];
    }
    if (ov.nmov == 0) {  // static obstacles only: walk of the cell list, two entries at a time (their
                         // LDS loads and cull tests overlap; SATs still run in list order)
      for (; a < ae; a += 2) {
        const bool two = a + 1 < ae;
        const int j0 = ov.gitems[a];
        const int j1 = two ? (int)ov.gitems[a + 1] : j0;
        const bool c0 = obs_culled(ov, j0, ft, fvx, fvy);
        const bool c1 = !two || obs_culled(ov, j1, ft, fvx, fvy);
        if (c0 && c1) continue;
        if (!have_veh) {
          veh_box(vpx, vpy, r.x2, veh);
          have_veh = true;
        }
        if (!c0 && obs_sat_static(veh, ov, j0) == 0) { tests += j0 + 1; return 0.0; }
        if (!c1 && obs_sat_static(veh, ov, j1) == 0) { tests += j1 + 1; return 0.0; }
      }
      tests += ov.n;
      return 10000;
    }
    int b = 0;
    while (a < ae || b < ov.nmov) {
      const int ja = a < ae ? (int)ov.gitems[a] : 0x7fffffff;
      const int jb = b < ov.nmov ? (int)ov.gmov[b] : 0x7fffffff;
      int j;
      bool mv;
      if (ja < jb) { j = ja; a++; mv = false; } else { j = jb; b++; mv = true; }
      if (obs_culled(ov, j, ft, fvx, fvy)) continue;
      if (!have_veh) {
        veh_box(vpx, vpy, r.x2, veh);
        have_veh = true;
      }
      if ((mv ? obs_sat(veh, ov, j, t) : obs_sat_static(veh, ov, j)) == 0) { tests += j + 1; return 0.0; }
    }
    tests += ov.n;  // the reference tests every obstacle until the first overlap
    return 10000;
  }
  veh_box(vpx, vpy, r.x2, veh);
  double best = 10000;
  for (int j = 0; j < ov.n; j++) {
    bool culled;
    float D = obs_gap(veh, ov, j, t, ft, fvx, fvy, !NEED_GAP, culled);
    if (culled) continue;
    if (D == 0) { tests += j + 1; return 0.0; }
    if (NEED_GAP && (double)D < best) best = D;
  }
  tests += ov.n;
  return best;
}

// Diagnostics (built with -DCLRRT_ROLL_PROFILE only): time per phase of the rollout kernels, from the
// shader clock, accumulated into work counters 40..47.  k_rollout (one lane per job) keeps it per lane.
// k_roll_run keeps it per WAVE (wq: the wave's LDS slot, [0] the last mark, [1 + k] phase k): a mark closes
// the interval since the previous mark of ANY of the wave's lanes, so a phase that runs on some lanes while
// the others idle is charged to that phase (round 3's per-lane clocks, read from lane 0, charged everything
// lane 0 sat out -- 45-80% of the wave time -- to "loop top").
struct PhaseClk {
  uint64_t last;
  uint64_t t[8];
  uint64_t* wq = nullptr;
  __device__ __forceinline__ void mark(int k) {
#ifdef CLRRT_ROLL_PROFILE
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (wq) {
      const uint64_t m = __ballot(1);
      if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)m) - 1) {
        wq[1 + k] += now - wq[0];
        wq[0] = now;
      }
      __builtin_amdgcn_wave_barrier();
      return;
    }
    t[k] += now - last;
    last = now;
#endif
  }
};

// One Euler step of Simulation::propagate (simulation.cpp:58-137), in two parts around the collision
// check: roll_step_pre (controls, ODE, the heading's trigonometry; fills the logged row columns 7..9,
// returns the heading rate for the lateral-acceleration test) and roll_step_post (costs, limits, end
// and goal tests with the checkObsDistance value Dobs; returns CLRRT_ROLL_* or -1 to continue).
__device__ __forceinline__ double roll_step_pre(Roll& r, const DevParams& p, double& col7, double& col8,
                                                double& col9, WorkCtr& w, PhaseClk* pc) {
  double Px, Py;
  // Controller::getControls (controller.cpp:30-34): waypoint, steer, accel
  w.scan += (uint32_t)(r.R.N - r.wp);
  double dla = update_waypoint(r, p, Px, Py, false);
  if (pc) pc->mark(1);
  double ym = lateral_error(r, Px, Py);
  const double dc = steer_cmd(r, p, dla, ym);
  const double vref = prof_v(r.P, r.wp + 2);  // ref.v[IDwp + 2]: the PI error and the logged column 8
  const double ac = accel_cmd(r, p, vref);
  // VehicleODE + IntegrateEuler (simulation.cpp:11-34)
  const double d2 = ode_euler(r, p, dc, ac);
  if (pc) pc->mark(2);
  // (round 5: the branched functions for waves with at most 2 lanes in flight measured 5% slower per lone step
  // than this block, whose independent chains interleave -- profiles/r05l_sparse_trig_tie_replay_ab.txt)
  if (!glibc::step_trig(r.x2, r.x3, r.s2, r.c2, r.swp, r.cwp, r.t3)) {  // one branch-free block (in domain)
    glibc::sincos_sel(r.x2, r.s2, r.c2);
    r.t3 = glibc::tan(r.x3);
    glibc::sin_cos_fma_sel(r.x2, r.swp, r.cwp);
  }
  if (pc) pc->mark(3);
  col7 = (double)r.wp;
  col8 = vref;
  col9 = dc;
  return d2;
}

__device__ __forceinline__ int roll_step_post(Roll& r, const DevParams& p, double Dobs, double d2) {
  if (Dobs == 0) return CLRRT_ROLL_COLLISION;  // simulation.cpp:83-86
  // costs (simulation.cpp:89-95)
  r.costE += r.x4 * p.dt;
  double kappa = r.t3 / p.L;
  double term = p.W0 * r.x4 * p.dt + p.W1 * fabs(kappa);
  if (p.use_exp) term = term + p.W2 * glibc::exp(-p.W3 * Dobs);  // glibc's exp, restated
  r.costS += term;
  if (p.bend) r.costS += p.W4 * dist_to_lane(r.x0, r.x1, p.lane_shift0, p.Cxy1, p.Cxy2);
  // lateral acceleration limit (simulation.cpp:98-104)
  double ay = fabs(r.x4 * d2);
  if (ay + p.ay_road_max > 3) return CLRRT_ROLL_ACCLIMIT;
  // end / goal (simulation.cpp:110-133)
  double ex = r.x0 - p.g0, ey = r.x1 - p.g1;
  double Ve = (r.x4 - r.vback);
  if (r.endr && (Ve < 0.1)) return CLRRT_ROLL_END;
  // dg = sqrt(ex^2 + ey^2) <= 1 needs ex^2 + ey^2 <= 1 + 2^-52 (sqrt is correctly rounded and monotonic),
  // so the square root is taken only near the goal; the heading error (an fmod) only matters within
  // 1 m of the goal; all of these are side-effect free
  const double dg2 = ex * ex + ey * ey;
  if (dg2 <= 1.0000000000000004 && sqrt(dg2) <= 1 && (fabs(angle_diff(r.x2, p.g2)) < 0.05)) return CLRRT_ROLL_GOAL;
  return -1;
}

template <bool NEED_GAP>
__device__ __forceinline__ int roll_step(Roll& r, const DevParams& p, const ObsView& ov, double& col7,
                                         double& col8, double& col9, WorkCtr& w, PhaseClk* pc = nullptr) {
  const double d2 = roll_step_pre(r, p, col7, col8, col9, w, pc);
  // collision (simulation.cpp:83-86)
  const double Dobs = obs_distance<NEED_GAP>(r, p, ov, w.box);
  if (pc) pc->mark(4);
  return roll_step_post(r, p, Dobs, d2);
}

// Wave-cooperative checkObsDistance without the gap value (k_roll_run; OBB collision with the static
// grid): the same value and box-test count as obs_distance<false> for every lane with act set, with the
// work of all lanes spread over the wave.  The candidate pairs (lane, obstacle) of the active lanes -- each
// lane's grid-cell list of static obstacles, then the moving ones -- are numbered by a wave prefix sum and
// taken 64 at a time, one pair per lane: the lane culls its pair against the owner's vehicle circle and,
// if it survives, SAT-tests it against the owner's vehicle box (built only by owners with a survivor);
// an overlap lowers the owner's first-overlap index.  A lone rollout's ~10-30 candidates are thus culled
// and tested in one pass instead of one after another.  The result only depends on whether some candidate
// overlaps (Dobs = 0; checkObsDistance returns at its first overlap, old_collisioncheck.cpp:24-51) and,
// for the work counter, on the smallest overlapping index (the lists ascend, so that is the reference's
// first overlap).  A lane outside the grid's float frame takes obs_distance itself.  Called by every lane
// of the wave (wave-uniform control flow).
struct CoopLds {
  Box4* veh;      // [64] vehicle boxes
  double* t;      // [64] prediction time of each lane's step
  int* hit;       // [64] smallest overlapping obstacle index (INT_MAX: none)
  uint32_t* q;    // [cap] scratch: owner records (below)
  int cap;
};
#define COOP_QCAP 512
constexpr size_t kCoopLdsPerWave = 64 * sizeof(Box4) + 64 * sizeof(double) + 64 * sizeof(int) + COOP_QCAP * sizeof(uint32_t);

__device__ double obs_distance_coop(bool act, const Roll& r, const DevParams& p, const ObsView& ov, uint32_t& tests,
                                    const CoopLds& cl, unsigned long long* cs = nullptr) {
  const int lane = threadIdx.x & 63;
  // owner records in the scratch: (fvx, fvy, ft, first item) | pair-range start | static count | window
  // start owners | survivor flags
  float4* s_pos = (float4*)cl.q;            // [64]
  int* s_pre = (int*)(cl.q + 256);          // [64]
  int* s_nst = (int*)(cl.q + 320);          // [64]
  int* s_own = (int*)(cl.q + 384);          // [64]
  int* s_need = (int*)(cl.q + 448);         // [64]
  double t = 0.0, vpx = 0.0, vpy = 0.0;
  float fvx = 0.f, fvy = 0.f, ft = 0.f;
  bool use = false;  // this lane's check goes through the pairs
  int a = 0, ae = 0;
  if (act) {
    t = p.obs_use_pred ? r.x6 : 0.0;
    vpx = r.x0 + 1.424 * r.c2;
    vpy = r.x1 + 1.424 * r.s2;
    fvx = (float)vpx; fvy = (float)vpy; ft = (float)t;
    use = isfinite(fvx) && isfinite(fvy) && isfinite(ft);
    if (use) {
      const int gx = (int)floorf((fvx - ov.gx0) * ov.ginv), gy = (int)floorf((fvy - ov.gy0) * ov.ginv);
      if (gx >= 0 && gx < ov.gw && gy >= 0 && gy < ov.gh) {
        const int cell = gy * ov.gw + gx;
        a = ov.gstart[cell];
        ae = ov.gstart[cell + 1];
      }
    }
  }
  const int nst = ae - a;
  const int len = use ? nst + ov.nmov : 0;
  // exclusive prefix sum of the pair counts over the wave
  int inc = len;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  const int pre = inc - len;
  const int total = __shfl(inc, 63, 64);
  cl.hit[lane] = 0x7fffffff;
  cl.t[lane] = t;
  s_pos[lane] = make_float4(fvx, fvy, ft, __int_as_float(a));
  s_pre[lane] = pre;
  s_nst[lane] = nst;
  s_need[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  int carry = -1;  // owner of the window's first pair when its range began in an earlier window
#ifdef CLRRT_COLL_STATS
  // diagnostics: wave-steps, lanes checked, pairs, windows, windows with a survivor, survivors, vehicle boxes built
  unsigned long long st_w = 0, st_s = 0, st_v = 0;
#endif
  for (int t0 = 0; t0 < total; t0 += 64) {
    // the owners whose range starts inside this window, at their first position
    const bool starts = len > 0 && pre >= t0 && pre < t0 + 64;
    if (starts) s_own[pre - t0] = lane;
    unsigned long long sm = starts ? (1ull << (pre - t0)) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sm |= (unsigned long long)__shfl_xor((long long)sm, o, 64);
    __builtin_amdgcn_wave_barrier();
    const int pidx = t0 + lane;
    const bool valid = pidx < total;
    const unsigned long long below = sm & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
    const int owner = below ? s_own[63 - __clzll(below)] : carry;
    int jj = 0;
    bool mv = false, surv = false;
    float4 op = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) {
      op = s_pos[owner];
      const int idx = pidx - s_pre[owner];
      const int no = s_nst[owner];
      mv = idx >= no;
      jj = mv ? (int)ov.gmov[idx - no] : (int)ov.gitems[__float_as_int(op.w) + idx];
      surv = !obs_culled(ov, jj, op.z, op.x, op.y);
    }
    // the window's last pair's owner continues into the next window
    carry = __shfl(owner, 63, 64);
#ifdef CLRRT_COLL_STATS
    st_w++;
    st_s += __popcll(__ballot(surv));
#endif
    if (__ballot(surv)) {
#ifdef CLRRT_COLL_STATS
      st_v++;
#endif
      if (surv && s_need[owner] != 2) s_need[owner] = 1;
      __builtin_amdgcn_wave_barrier();
      if (s_need[lane] == 1) {  // setVertices of the lanes with a survivor (once per step)
        Box4 vb;
        veh_box(vpx, vpy, r.x2, vb);
        cl.veh[lane] = vb;
        s_need[lane] = 2;
      }
      __builtin_amdgcn_wave_barrier();
      if (surv) {
        const Box4 vb = cl.veh[owner];
        const float gap = mv ? obs_sat(vb, ov, jj, cl.t[owner]) : obs_sat_static(vb, ov, jj);
        if (gap == 0) atomicMin(&cl.hit[owner], jj);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
#ifdef CLRRT_COLL_STATS
  const unsigned long long st_u = __popcll(__ballot(use));
  if (cs && lane == 0) {
    atomicAdd(&cs[0], 1ull);
    atomicAdd(&cs[1], st_u);
    atomicAdd(&cs[2], (unsigned long long)total);
    atomicAdd(&cs[3], st_w);
    atomicAdd(&cs[4], st_v);
    atomicAdd(&cs[5], st_s);
  }
#endif
  double D = 10000;
  if (use) {
    const int h = cl.hit[lane];
    if (h != 0x7fffffff) {
      tests += h + 1;
      D = 0.0;
    } else {
      tests += ov.n;
    }
  } else if (act) {
    D = obs_distance<false>(r, p, ov, tests);  // outside the float frame: the lane's own scan
  }
  return D;
}

// One stateArray row; es = element stride (1 for row-major rows, the job count for the slot
// layout in which consecutive lanes' values are adjacent, so a wave's stores coalesce).
__device__ __forceinline__ void store_row(double* __restrict__ row, int64_t es, const Roll& r, double c7,
                                          double c8, double c9) {
  row[0] = r.x0; row[es] = r.x1; row[2 * es] = r.x2; row[3 * es] = r.x3; row[4 * es] = r.x4;
  row[5 * es] = r.x5; row[6 * es] = r.x6; row[7 * es] = c7; row[8 * es] = c8; row[9 * es] = c9;
}

// What Simulation exposes after propagate (stateArray.back(), costs, reference ends).
__device__ __forceinline__ void finish_rollout(const Roll& r, double c7, double c8, double c9, int outcome,
                                               int steps, RollRes& out) {
  out.st[0] = r.x0; out.st[1] = r.x1; out.st[2] = r.x2; out.st[3] = r.x3; out.st[4] = r.x4;
  out.st[5] = r.x5; out.st[6] = r.x6; out.st[7] = c7; out.st[8] = c8; out.st[9] = c9;
  out.costE = r.costE;
  out.costS = r.costS;
  out.bx = r.R.bx; out.by = r.R.by;
  out.fx = r.R.a1x; out.fy = r.R.a1y;
  out.vback = r.vback;
  out.outcome = outcome;
  out.nrows = steps + 1;
  out.refN = r.R.N;
}

// One whole rollout from parent state `ps` along reference R (ref.v generated from pvb = Vstart).  rows
// (nullable) receives stateArray: element k of row i at rows[(i * 10 + k) * es].  init (nullable)
// receives the Simulation state after its constructor (reference end and velocity profile).
template <bool NEED_GAP>
__device__ __forceinline__ void run_rollout_ref(const St10& ps, const RefD& R, double pvb, int gb, const DevParams& p,
                                                const ObsView& ov, double* __restrict__ rows, int64_t es,
                                                RollRes& out, WorkCtr& w, Roll* init = nullptr,
                                                PhaseClk* pc = nullptr) {
  Roll r;
  roll_init(r, ps.v, R, pvb, gb != 0, p);
  if (init) *init = r;
  double c7 = (double)r.wp, c8 = ps.v[8], c9 = ps.v[9];
  if (rows) {
#pragma unroll
    for (int k = 0; k < 10; k++) rows[k * es] = ps.v[k];
    rows[7 * es] = c7;
  }
  int outcome = CLRRT_ROLL_ITERLIMIT;
  int steps = 0;
  for (int i = 0; i < p.n_steps_max; i++) {
    steps++;
    if (pc) pc->mark(0);
    int o = roll_step<NEED_GAP>(r, p, ov, c7, c8, c9, w, pc);
    if (rows) store_row(rows + (int64_t)steps * 10 * es, es, r, c7, c8, c9);
    if (pc) pc->mark(5);
    if (o >= 0) { outcome = o; break; }
  }
  finish_rollout(r, c7, c8, c9, outcome, steps, out);
  w.steps += (uint32_t)steps;
}

// One whole rollout of expandTree: toward (sx, sy) (getReference) or the goal (getGoalReference) from a
// parent whose ref.back() is (pbx, pby) and ref.v.back() is pvb.
template <bool NEED_GAP>
__device__ __forceinline__ void run_rollout(const St10& ps, double pbx, double pby, double pvb, int gb, double sx,
                            double sy, const DevParams& p, const ObsView& ov, double* __restrict__ rows,
                            int64_t es, RollRes& out, WorkCtr& w) {
  const RefD R = gb ? make_goal_ref(pbx, pby, p) : make_ref(pbx, pby, sx, sy, p);
  run_rollout_ref<NEED_GAP>(ps, R, pvb, gb, p, ov, rows, es, out, w);
}


// feasibleGoalBias rrtplanner.cpp:292-
__device__ __forceinline__ bool feasible_goal_bias(const DevParams& p, const double* st, double bx,
                                                   double by) {
  bool outL = sqrt((st[0] - p.gbLx) * (st[0] - p.gbLx) + (st[1] - p.gbLy) * (st[1] - p.gbLy)) > p.gbR2;
  bool outR = sqrt((st[0] - p.gbRx) * (st[0] - p.gbRx) + (st[1] - p.gbRy) * (st[1] - p.gbRy)) > p.gbR2;
  double aRef = glibc::atan2(p.g1 - by, p.g0 - bx);
  double h1 = fabs(wrap_pi(p.g2 - aRef));
  double h2 = fabs(wrap_pi(p.g2 + M_PI - aRef));
  double m = mn(h1, h2);
  double cv = glibc::cos(p.g2 + M_PI_2 - aRef);
  double sg = (double)((0.0 < cv) - (cv < 0.0));
  double ang = sg * m;
  bool within = fabs(ang) < (M_PI_4 / 2);
  return outL && outR && within;
}

// Rollout jobs (Simulation::propagate, rrt/src/simulation.cpp:26-...).
//   SRC_SPEC: job j = (sample j / K, candidate j % K), parent = tree node cand[j]; after a successful
//             regular rollout whose end passes the goal-bias gate the same lane runs the goal-biased
//             rollout from the node it would append (expandTree rrtplanner.cpp:163-173), so goal
//             bias overlaps other samples' candidates instead of forming a serial tail.  Rows go to
//             job slots, interleaved across jobs: element k of row i of job j, pass p (0 regular,
//             1 goal-biased) at slots[((p * slot_jobs + j) * slot_rows + i) * 10 + k] (a job's rows are
//             contiguous, so a lane's consecutive row stores fill whole cache lines).
//   SRC_LIST: explicit jobs (parity entry): parent = tree node, rows to arena[row_off] when >= 0.
// Stage the obstacle cull table (and static-obstacle grid) of the query in LDS.
template <bool NEED_GAP>
__device__ __forceinline__ ObsView stage_obstacles(const RollArgs& a, float4* lds) {
  float4* cv = lds;
  float4* ob = lds + a.p.n_obs;
  float4* sat = ob + a.p.n_obs;
  float* rad = (float*)(sat + 4 * a.p.n_obs);
  uint32_t* gstart = (uint32_t*)(rad + a.p.n_obs);
  const int ncell = a.grid.gw * a.grid.gh;
  uint16_t* gitems = (uint16_t*)(gstart + (a.grid.gw > 0 ? ncell + 1 : 0));
  uint16_t* gmov = gitems + a.grid.nitems;
  if (a.p.coll_mode == CLRRT_COLLISION_OBB && !NEED_GAP) {
    for (int j = threadIdx.x; j < a.p.n_obs; j += blockDim.x) {
      const BakedObs& o = a.obs[j];
      cv[j] = make_float4((float)o.cx, (float)o.cy, (float)o.vlx, (float)o.vly);
      rad[j] = o.brad + VEH_RAD + CULL_MARGIN;
      // box axes from the baked products: P = cos*hh, R = sin*hh, Q = sin*ww, S = cos*ww
      const float hh = sqrtf(o.P * o.P + o.R * o.R), ww = sqrtf(o.Q * o.Q + o.S * o.S);
      const float ux = hh > 0.f ? o.P / hh : 1.f, uy = hh > 0.f ? o.R / hh : 0.f;
      ob[j] = make_float4(ux, uy, hh * 1.00001f + 1e-4f, ww * 1.00001f + 1e-4f);
      sat[4 * j] = make_float4(o.vx[0], o.vx[1], o.vx[2], o.vx[3]);
      sat[4 * j + 1] = make_float4(o.vy[0], o.vy[1], o.vy[2], o.vy[3]);
      sat[4 * j + 2] = make_float4(o.nx[0], o.nx[1], o.nx[2], o.nx[3]);
      sat[4 * j + 3] = make_float4(o.ny[0], o.ny[1], o.ny[2], o.ny[3]);
    }
    if (a.grid.gw > 0) {
      for (int j = threadIdx.x; j <= ncell; j += blockDim.x) gstart[j] = a.grid.start[j];
      for (int j = threadIdx.x; j < a.grid.nitems; j += blockDim.x) gitems[j] = a.grid.items[j];
      for (int j = threadIdx.x; j < a.grid.nmov; j += blockDim.x) gmov[j] = a.grid.mov[j];
    }
    __syncthreads();
  }
  return ObsView{a.obs, cv, rad, ob, sat, gstart, gitems, gmov, a.p.coll_mode == CLRRT_COLLISION_OBB ? a.p.n_obs : 0,
                 a.grid.gw, a.grid.gh, a.grid.nmov, a.grid.x0, a.grid.y0, a.grid.inv};
}

// The query's parameters in the rollout kernels: in LDS (CLRRT_PARAMS_LDS 1: the step reads each one when it needs it,
// instead of holding ~100 SGPRs of them all kernel long -- spilled to VGPR lanes and read back lane by lane) or the
// kernel argument (0).
#ifndef CLRRT_PARAMS_LDS
#define CLRRT_PARAMS_LDS 1
#endif
#if CLRRT_PARAMS_LDS
#define CLRRT_PARAMS_DECL(P)                    \
  __shared__ DevParams s_params_;               \
  if (threadIdx.x == 0) s_params_ = a.p;        \
  __syncthreads();                              \
  const DevParams& P = s_params_
#else
#define CLRRT_PARAMS_DECL(P) const DevParams& P = a.p
#endif

#ifndef CLRRT_ROLLOUT_WAVES
#define CLRRT_ROLLOUT_WAVES 1
#endif
template <int SRC, bool NEED_GAP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CLRRT_ROLLOUT_WAVES))) k_rollout(RollArgs a) {
  extern __shared__ float4 lds[];
  glibc::stage_tables();
  const ObsView ov = stage_obstacles<NEED_GAP>(a, lds);
  CLRRT_PARAMS_DECL(P);
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int js = a.job_stride > 1 ? a.job_stride : 1;
  const int j = gt / js;
  WorkCtr w{0, 0, 0};
  bool act = j < a.njobs && gt % js == 0;
  St10 ps;
  double pbx = 0, pby = 0, pvb = 0, sx = 0, sy = 0;
  int gb = 0;
  double* rows = nullptr;
  int64_t es = 1;
  const int64_t slot = (int64_t)a.slot_rows * 10;
  const int64_t pass_stride = slot * a.slot_jobs;
  if (act) {
    const clrrt_node* n = nullptr;
    if (SRC == SRC_EXPL) {
      const SimJob& sj = a.sims[j];
      RefD R;
      if (sj.gb) {
        R = make_goal_ref(sj.ax, sj.ay, P);
      } else {
        R.a1x = sj.ax; R.a1y = sj.ay; R.h1x = sj.hx; R.h1y = sj.hy;
        R.a2x = R.a2y = R.h2x = R.h2y = 0.0;
        R.n1 = sj.n; R.N = sj.n;
        R.bx = sj.ax; R.by = sj.ay;
      }
#pragma unroll
      for (int k = 0; k < 10; k++) ps.v[k] = sj.st[k];
      RollRes out;
      Roll ini;
      run_rollout_ref<NEED_GAP>(ps, R, sj.vstart, sj.gb, P, ov, sj.row_off >= 0 ? a.arena + sj.row_off * 10 : nullptr,
                                1, out, w, &ini);
      a.res[j] = out;
      if (sj.ref_off >= 0) {  // the reference the Simulation used, with the profile it generated
        double* o = a.refv + sj.ref_off;
        double x = ini.R.a1x, y = ini.R.a1y;
        for (int i = 0; i < ini.R.N && i < a.ref_cap; i++) {
          o[i] = x;
          o[a.ref_cap + i] = y;
          o[2 * a.ref_cap + i] = prof_v(ini.P, i);
          ref_next(ini.R, i, x, y);
        }
      }
      act = false;
    } else if (SRC == SRC_SPEC) {
      const int id = a.cand[j];
      if (id < 0) {
        a.res[j].outcome = -1;
        a.res_gb[j].outcome = -1;
        act = false;
      } else {
        n = &a.tree[id];
        sx = a.samples[j / CAND_K].x;
        sy = a.samples[j / CAND_K].y;
        if (a.slots) rows = a.slots + j * slot;
      }
    } else {
      const Job& jb = a.jobs[j];
      n = jb.from_reg == 1 ? &a.xreg[jb.parent] : jb.from_reg == 2 ? &a.xgb[jb.parent] : &a.tree[jb.parent];
      gb = jb.gb; sx = jb.sx; sy = jb.sy;
      if (jb.row_off >= 0) rows = a.arena + (size_t)jb.row_off * 10;
    }
    if (n) {
#pragma unroll
      for (int k = 0; k < 10; k++) ps.v[k] = n->state[k];
      pbx = n->ref_back[0]; pby = n->ref_back[1]; pvb = n->ref_vback;
    }
  }
#ifdef CLRRT_ROLL_PROFILE
  PhaseClk pclk{};
  pclk.last = __builtin_amdgcn_s_memtime();
  PhaseClk* pc = &pclk;
#else
  PhaseClk* pc = nullptr;
#endif
  if (act) {
    for (int pass = 0; pass < 2; pass++) {
      RollRes out;
      const RefD R = gb ? make_goal_ref(pbx, pby, P) : make_ref(pbx, pby, sx, sy, P);
      run_rollout_ref<NEED_GAP>(ps, R, pvb, gb, P, ov, rows, es, out, w, nullptr, pc);
      if (pass == 1) {
        a.res_gb[j] = out;
        break;
      }
      a.res[j] = out;
      if (SRC != SRC_SPEC) break;
      const bool ok = (out.outcome == CLRRT_ROLL_END || out.outcome == CLRRT_ROLL_GOAL) &&
                      feasible_goal_bias(P, out.st, out.bx, out.by);
      if (!ok) {
        a.res_gb[j].outcome = -1;
        break;
      }
#pragma unroll
      for (int k = 0; k < 10; k++) ps.v[k] = out.st[k];
      pbx = out.bx; pby = out.by; pvb = out.vback;
      gb = 1;
      if (a.slots) rows = a.slots + pass_stride + j * slot;
    }
  }
  if (a.ctr) {  // algorithmic work counters (roofline): block reduction, one atomic per block
    __shared__ __attribute__((aligned(16))) unsigned long long s_ctr[4];
    if (threadIdx.x < 3) s_ctr[threadIdx.x] = 0;
    __syncthreads();
    if (w.steps) {
      atomicAdd(&s_ctr[0], (unsigned long long)w.steps);
      atomicAdd(&s_ctr[1], (unsigned long long)w.scan);
      atomicAdd(&s_ctr[2], (unsigned long long)w.box);
    }
    __syncthreads();
    if (threadIdx.x < 3 && s_ctr[threadIdx.x]) atomicAdd(&a.ctr[threadIdx.x], s_ctr[threadIdx.x]);
  }
#ifdef CLRRT_ROLL_PROFILE
  if (a.ctr && j < a.njobs && gt % js == 0)
    for (int q = 0; q < 8; q++) atomicAdd(&a.ctr[40 + q], (unsigned long long)pclk.t[q]);
#endif
}

// --------------------------------------------------------------------------------------------
// persistent speculative rollouts
// --------------------------------------------------------------------------------------------
// The candidate rollouts of a round differ wildly in length (a collision can end one after a few
// steps, an end-of-reference one runs hundreds), so one lane per job leaves most lanes of a wave idle
// behind its longest rollout.  Instead:
//   k_roll_run  : persistent waves; idle lanes take the next jobs (j = (sample s, candidate k)) from a
//                 queue whose first positions replay the previous commit's accepted rollouts, then the
//                 round's jobs in candidate-major
//                 order (all first candidates, then all second ones, ...), so when candidate k of
//                 sample s is taken the earlier ones have usually finished: a job whose sample
//                 already has a successful earlier candidate is skipped (or abandoned while
//                 running) -- expandTree never looks past the first success (:150-160), so the
//                 round's result is unchanged.  A successful regular rollout that passes the
//                 goal-bias gate continues in the same lane with the goal-biased rollout.  Every start
//                 (getReference / getGoalReference + the Simulation ctor) is built in the kernel at one
//                 code site (until round 3 a k_roll_prep kernel materialised it per job).

// What a rollout starts from (getReference / getGoalReference + the Simulation ctor): the parent state,
// the parent's ref.back() and ref.v.back(), the sample (regular rollouts) and the goal-bias flag.
struct RollSrc {
  double st[10];
  double bx, by, vb;   // parent ref.back(), ref.v.back()
  double sx, sy;       // sample (regular)
  int32_t gb, pad;
};

// Deferred trajectory rows.  k_roll_run stores no rows for the speculative rollouts (most of them fail or
// are abandoned, and their rows would never be read); a commit records the accepted ones (k_replay_gather)
// and the next k_roll_run launch replays them from the same start, writing their rows straight into the
// arena (rollouts are deterministic: same start, same steps, same rows).  A regular rollout starts from its
// parent node and sample, a goal-biased one from the end of the regular rollout it followed.  Replays
// take the queue's first positions.
struct Replay {
  RollSrc src;
  int64_t row_off;     // arena row of stateArray[0]
  int32_t nrows;       // rows the committed node holds
  int32_t pad;
};

// Deferred samples (BATCH option "defer_steps" T).  A round's launch used to last as long as its longest
// chain (a regular rollout + its goal-biased follow-up, up to ~1000 steps), three quarters of it a few
// straggling lanes (profiles/r03x_roll_phases.txt).  With a cap T, every chain runs at most T more steps per
// launch; a chain that reaches its cap is suspended here (its whole lane state) and resumed at the front of
// the next launch's queue, and its sample is committed by the first commit after which every rollout its
// result depends on has ended -- deterministically launch ceil(C / T) - 1 after its own, C = the longest of
// those chains in steps (the oracle's orc_expand_batch_defer restates the rule).  Replays (deferred rows)
// are capped the same way; they only write rows.
struct Carry {
  Roll r;
  double c7, c8, c9;
  int64_t row_off;   // replays: arena row of stateArray[0]; -1: no rows
  int32_t j;         // ring index of the job (res / res_gb); 0 for replays
  int32_t bs;        // ring index of the sample (best)
  int32_t k, pass, steps, chain, rp, nrows_rp;
};

size_t carry_bytes() { return sizeof(Carry); }

// Scheduling only: a rollout toward a sample 8-20 m away (1.7-4.2 turning radii) at 30-90 degrees off
// the heading is the kind that ends in the iteration limit after the full horizon (the vehicle
// circles without reaching the reference: tools/orbit_predict.py, cfg3 round 40: this class is 3% of
// the jobs and holds 472 of the 501 jobs of >= 300 steps).  Served first, these chains no longer
// start late and set the kernel's makespan.
__device__ __forceinline__ int roll_likely_long(const double* st, double sx, double sy) {
  const float dx = (float)(sx - st[0]), dy = (float)(sy - st[1]);
  const float d2 = dx * dx + dy * dy;
  if (!(d2 >= 64.f && d2 < 400.f)) return 0;
  const float c = cosf((float)st[2]), s = sinf((float)st[2]);
  const float along = dx * c + dy * s, across = fabsf(dy * c - dx * s);
  // 30 <= angle < 90 degrees: along > 0 and across >= tan(30 deg) along
  return (along > 0.f && across >= 0.57735f * along) ? 1 : 0;
}

// Queue order: flagged positions first (in q order), then the rest (in q order).
__global__ void __launch_bounds__(256) k_roll_order(const int* __restrict__ pflag, const int* __restrict__ ppos,
                                                    int n, int* __restrict__ perm) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int nf = ppos[n - 1] + pflag[n - 1];
  const int pos = pflag[q] ? ppos[q] : nf + (q - ppos[q]);
  perm[pos] = q;
}

// Queue order flags (roll_priority): pflag[q] for queue position q = k B + s, 1 for the jobs likely to run
// the whole horizon (roll_likely_long); k_roll_order then serves them first.
__global__ void __launch_bounds__(256) k_roll_flag(RollArgs a) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.njobs) return;
  const int id = a.cand[j];
  a.pflag[(j % CAND_K) * a.B + j / CAND_K] =
      id < 0 ? 0 : roll_likely_long(a.tree[id].state, a.samples[j / CAND_K].x, a.samples[j / CAND_K].y);
}

#ifndef REFILL_MIN
#define REFILL_MIN 16
#endif

#ifndef CLRRT_ABANDON_EVERY  // steps between checks for an earlier candidate's success (power of 2)
#define CLRRT_ABANDON_EVERY 16
#endif

#ifndef CLRRT_ROLL_WAVES
#define CLRRT_ROLL_WAVES 1
#endif
constexpr int kFinSuspend = 1000;  // k_roll_run: `fin` of a lane whose chain reached its cap (defer_steps)
// COOP: the collision check is obs_distance_coop (OBB collision without the gap value, static grid built,
// the per-wave LDS scratch after the obstacle tables at a.coop_off)
// CARRY: the launch resumes / suspends chains (deferred samples, option defer_steps); the instantiation without
// it has none of that code (the step loop's register allocation is that of the plain kernel)
template <bool NEED_GAP, bool COOP, bool CARRY>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CLRRT_ROLL_WAVES))) k_roll_run(RollArgs a,
                                                  int* __restrict__ qnext, int* __restrict__ best, int B) {
  extern __shared__ float4 lds[];
  glibc::stage_tables();
  const ObsView ov = stage_obstacles<NEED_GAP>(a, lds);
  CLRRT_PARAMS_DECL(P);
  const int lane = threadIdx.x & 63;
  CoopLds cl{};
  if constexpr (COOP) {
    char* base = (char*)lds + a.coop_off + (size_t)(threadIdx.x >> 6) * kCoopLdsPerWave;
    cl.veh = (Box4*)base;
    cl.t = (double*)(base + 64 * sizeof(Box4));
    cl.hit = (int*)(base + 64 * sizeof(Box4) + 64 * sizeof(double));
    cl.q = (uint32_t*)(base + 64 * sizeof(Box4) + 64 * sizeof(double) + 64 * sizeof(int));
    cl.cap = COOP_QCAP;
  }
  const int64_t slot = (int64_t)a.slot_rows * 10;
  const int64_t pass_stride = slot * a.slot_jobs;
  WorkCtr w{0, 0, 0};
  Roll r;
  double c7 = 0, c8 = 0, c9 = 0;
  // j: ring index of the lane's job (res / res_gb; -1 idle, 0 for replays), bs: ring index of its sample
  // (best), k: its candidate; chain: steps of the chain so far (regular + goal-biased), cap_at: the chain
  // step count at which it is suspended (defer_steps)
  int j = -1, k = 0, bs = 0, pass = 0, steps = 0, chain = 0, cap_at = 0x7fffffff;
  bool exhausted = false;
  // rows: where this lane's rollout writes stateArray (a replay's arena rows; nullptr for the speculative
  // rollouts when rows are deferred, else their job slots); rp: the lane replays a committed rollout of
  // nrows_rp rows
  const Replay* __restrict__ reps = (const Replay*)a.rep;
  const Carry* __restrict__ cin = (const Carry*)a.carry_in;
  Carry* __restrict__ cout = (Carry*)a.carry_out;
  // queue: the suspended chains of the previous launch, the replays, then the round's jobs
  const int ncarry = CARRY ? a.ncarry : 0;
  const int nq = ncarry + a.nrep + a.njobs;
  double* rows = nullptr;
  bool rp = false;
  int nrows_rp = 0;
  unsigned long long n_rep = 0, n_rep_bad = 0;
  // a pending rollout start (a fetched job or replay, a successful rollout's goal-biased follow-up): the
  // Simulation is constructed for all of them at one code site (init_pending) after the fetch
  bool iq = false;
  RollSrc src;
  PhaseClk pclk{};
#ifdef CLRRT_ROLL_PROFILE
  __shared__ uint64_t s_phase[4][9];  // per wave of the block: last mark, phases 0..7
  PhaseClk* pc = &pclk;
  pclk.wq = s_phase[threadIdx.x >> 6];
  if ((threadIdx.x & 63) == 0) {
    pclk.wq[0] = __builtin_amdgcn_s_memtime();
    for (int q = 1; q < 9; q++) pclk.wq[q] = 0;
  }
  __builtin_amdgcn_wave_barrier();
#else
  PhaseClk* pc = nullptr;
#endif
  int fin = -1;  // >= 0: the lane's rollout ended with this outcome; finished in the next batch
#ifdef CLRRT_ROLL_PROFILE
  // longest chain (a regular rollout + its goal-biased follow-up) of the lane, the steps of its current
  // one, its steps after the wave found the queue empty, when that was
  unsigned long long chain_steps = 0, job_steps = 0, tail_steps = 0;
  uint64_t t_qdone = 0;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
  bool qdone = false;  // wave-uniform: a fetch of this wave found the job queue empty
#ifdef CLRRT_LANE_STATS
  // diagnostics (work counters 33..38, instead of CLRRT_COLL_STATS'): wave-steps and lanes stepping in them while the
  // queue still has jobs / after this wave found it empty, and the wave-steps with at most 8 lanes stepping
  unsigned long long ls_w[2] = {0, 0}, ls_l[2] = {0, 0}, ls_sparse[2] = {0, 0};
#endif
  // lanes that take jobs (a.lanes_per_wave: a short queue is spread over the grid's waves, so a rollout
  // shares its wave with few others -- each step of a wave runs the union of its lanes' paths -- and the
  // idle lanes still serve the cooperative collision checks)
  const bool lane_on = lane < a.lanes_per_wave;
  const int refill_min = min(REFILL_MIN, max(1, a.lanes_per_wave / 4));  // parked/idle lanes that trigger a batch

  // Rollouts that ended wait (parked) until enough lanes are parked or idle; then the wave finishes
  // them together (result store, best[], goal-bias gate + goal-biased rollout init) and refills the
  // idle lanes, so the long divergent end-of-rollout code runs once per batch instead of almost
  // every step for one or two lanes.
  auto finish_parked = [&]() {
    if (CARRY && fin == kFinSuspend) {  // a chain at its cap: suspended into carry_out, resumed by the next launch
      const int slot_c = atomicAdd(a.ncarry_out, 1);
      if (slot_c < a.carry_cap) {
        Carry& co = cout[slot_c];
        co.r = r;
        co.c7 = c7; co.c8 = c8; co.c9 = c9;
        co.row_off = rows ? (int64_t)((rows - a.arena) / 10) : -1;
        co.j = j; co.bs = bs; co.k = k; co.pass = pass; co.steps = steps; co.chain = chain;
        co.rp = rp ? 1 : 0;
        co.nrows_rp = nrows_rp;
        if (!rp) {  // the sample's result waits for this rollout (k_select: pending)
          if (pass == 0) a.res[j].outcome = CLRRT_ROLL_PENDING;
          else a.res_gb[j].outcome = CLRRT_ROLL_PENDING;
        }
      } else if (a.ctr) {  // no carry slot left: reported by the host (the round is void)
        atomicAdd(&a.ctr[62], 1ull);
      }
      rp = false;
      rows = nullptr;
      j = -1;
      fin = -1;
    }
    if (fin >= 0) {
      if (rp) {  // a replay: its rows are written; check it ran as long as the committed rollout
        n_rep++;
        n_rep_bad += (steps + 1 != nrows_rp);
        rp = false;
        rows = nullptr;
        j = -1;
      } else {
        RollRes out;
        finish_rollout(r, c7, c8, c9, fin, steps, out);
        if (pass == 1) {
          a.res_gb[j] = out;
          j = -1;
        } else {
          a.res[j] = out;
          const bool ok = fin == CLRRT_ROLL_END || fin == CLRRT_ROLL_GOAL;
          if (ok) atomicMin(&best[bs], k);
          if (ok && feasible_goal_bias(P, out.st, out.bx, out.by)) {
            // goal-biased rollout from the node this rollout would append (expandTree :163-173)
#pragma unroll
            for (int q = 0; q < 10; q++) src.st[q] = out.st[q];
            src.bx = out.bx; src.by = out.by; src.vb = out.vback;
            src.gb = 1;
            iq = true;
            pass = 1;
            rows = a.slots ? a.slots + pass_stride + j * slot : nullptr;
          } else {
            a.res_gb[j].outcome = -1;
            j = -1;
          }
        }
      }
      fin = -1;
    }
  };
  // getReference / getGoalReference + Simulation ctor of the pending starts (rrtplanner.cpp:146-149,
  // :165-168; simulation.cpp:36-47), and stateArray[0] when the lane writes rows
  auto init_pending = [&]() {
    if (iq) {
      const RefD R = src.gb ? make_goal_ref(src.bx, src.by, P) : make_ref(src.bx, src.by, src.sx, src.sy, P);
      roll_init(r, src.st, R, src.vb, src.gb != 0, P);
      c7 = (double)r.wp; c8 = src.st[8]; c9 = src.st[9];
      steps = 0;
      if (rows) {
#pragma unroll
        for (int q = 0; q < 10; q++) rows[q] = src.st[q];
        rows[7] = c7;
      }
      iq = false;
    }
  };
  // watchdog: every wave reaches an exit even if something goes wrong (a step always advances, so no
  // correct launch comes near the bound); a trip is counted and reported by the host
  uint32_t guard = 0;
  const uint64_t t_guard = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  for (;;) {
    if ((++guard & 255) == 0 && __builtin_amdgcn_s_memrealtime() - t_guard > 300000000ull) {  // 3 s
      if (a.ctr && lane == 0) {
        atomicAdd(&a.ctr[56], 1ull);
        atomicMax(&a.ctr[57], (unsigned long long)(((uint64_t)(uint32_t)j << 32) | (uint32_t)fin));
        atomicMax(&a.ctr[58], (unsigned long long)(((uint64_t)(uint32_t)steps << 32) | (uint32_t)chain));
        atomicMax(&a.ctr[59], (unsigned long long)(((uint64_t)qdone << 32) | (uint32_t)__popcll(__ballot(j >= 0))));
      }
      break;
    }
    if (pc) pc->mark(0);
    const uint64_t parked = __ballot(fin >= 0);
    const uint64_t busy0 = __ballot(j >= 0 && fin < 0);
    if (a.dbg && (guard & 63) == 0) {  // diagnostics heartbeat: the wave's state every 64 iterations
      const int fl = __ffsll((unsigned long long)busy0) - 1;
      const int wv = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
      unsigned long long* d = a.dbg + (size_t)wv * 8;
      const int fj = __shfl(j, fl < 0 ? 0 : fl, 64), fs = __shfl(steps, fl < 0 ? 0 : fl, 64);
      const int fc = __shfl(chain, fl < 0 ? 0 : fl, 64), fw = __shfl(r.wp, fl < 0 ? 0 : fl, 64);
      const int fn = __shfl(r.R.N, fl < 0 ? 0 : fl, 64), fp = __shfl(pass, fl < 0 ? 0 : fl, 64);
      if (lane == 0) {
        __atomic_store_n(&d[0], (unsigned long long)guard, __ATOMIC_RELAXED);
        __atomic_store_n(&d[1], (unsigned long long)busy0, __ATOMIC_RELAXED);
        __atomic_store_n(&d[2], (unsigned long long)parked, __ATOMIC_RELAXED);
        __atomic_store_n(&d[3], ((unsigned long long)qdone << 32) | (uint32_t)fl, __ATOMIC_RELAXED);
        __atomic_store_n(&d[4], ((unsigned long long)(uint32_t)fj << 32) | (uint32_t)fp, __ATOMIC_RELAXED);
        __atomic_store_n(&d[5], ((unsigned long long)(uint32_t)fs << 32) | (uint32_t)fc, __ATOMIC_RELAXED);
        __atomic_store_n(&d[6], ((unsigned long long)(uint32_t)fw << 32) | (uint32_t)fn, __ATOMIC_RELAXED);
        __atomic_store_n(&d[7], (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED);
      }
    }
    const uint64_t m0 = __ballot(j < 0 && !qdone && lane_on);
    // once the queue is empty, finish parked rollouts at once: a goal-biased follow-up (up to the whole
    // horizon) must not wait for other lanes to end
    if ((parked | m0) && (__popcll(parked | m0) >= refill_min || busy0 == 0 || (qdone && parked))) {
      finish_parked();
      if (pc) pc->mark(7);
      const bool idle = j < 0 && !qdone && lane_on;
      const uint64_t m = __ballot(idle);
      if (m) {
        // wave-aggregated fetch: the idle lanes take consecutive queue positions
        const int leader = __ffsll((unsigned long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(qnext, __popcll(m));
        base = __shfl(base, leader, 64);
        if (idle) {
          const int q0 = base + __popcll(m & ((1ull << lane) - 1));
          if (q0 >= nq) {
            exhausted = true;
          } else if (CARRY && q0 < ncarry) {  // a chain suspended by the previous launch: resumed where it stopped
            const Carry& cr = cin[q0];
            r = cr.r;
            c7 = cr.c7; c8 = cr.c8; c9 = cr.c9;
            j = cr.j; bs = cr.bs; k = cr.k; pass = cr.pass; steps = cr.steps; chain = cr.chain;
            rp = cr.rp != 0;
            nrows_rp = cr.nrows_rp;
            rows = cr.row_off >= 0 ? a.arena + cr.row_off * 10 : nullptr;
            cap_at = a.cap > 0 ? chain + a.cap : 0x7fffffff;
            if (!rp && __atomic_load_n(&best[bs], __ATOMIC_RELAXED) < k) {  // an earlier candidate succeeded
              if (pass == 0) a.res[j].outcome = -1;
              a.res_gb[j].outcome = -1;
              j = -1;
            }
          } else if (q0 - ncarry < a.nrep) {  // replay of a committed rollout: rows into the arena
            const Replay& rq = reps[q0 - ncarry];
            rp = true;
            nrows_rp = rq.nrows;
            rows = a.arena + rq.row_off * 10;
            j = 0;  // busy (replays touch no per-job result)
            k = 0; bs = 0; pass = 0; steps = 0; chain = 0;
            cap_at = a.cap > 0 ? a.cap : 0x7fffffff;
            src = rq.src;
            iq = true;
          } else {
            const int qj = q0 - ncarry - a.nrep;
            const int q = a.perm ? a.perm[qj] : qj;
            k = q / B;
            const int s = q - k * B;
            const int jl = s * CAND_K + k;
            j = a.jbase + jl;
            bs = a.sbase + s;
            const int id = a.cand[jl];
            if (id < 0 || __atomic_load_n(&best[bs], __ATOMIC_RELAXED) < k) {
              a.res[j].outcome = -1;
              a.res_gb[j].outcome = -1;
              j = -1;
            } else {
              const clrrt_node& n = a.tree[id];
#pragma unroll
              for (int q = 0; q < 10; q++) src.st[q] = n.state[q];
              src.bx = n.ref_back[0]; src.by = n.ref_back[1]; src.vb = n.ref_vback;
              src.sx = a.samples[s].x; src.sy = a.samples[s].y;
              src.gb = 0;
              iq = true;
              pass = 0;
              steps = 0;
              chain = 0;
              cap_at = a.cap > 0 ? a.cap : 0x7fffffff;
              rows = a.slots ? a.slots + jl * slot : nullptr;
#ifdef CLRRT_ROLL_PROFILE
              job_steps = 0;
#endif
            }
          }
        }
        qdone = qdone || __ballot(exhausted) != 0;
      }
      init_pending();
      if (pc) pc->mark(6);
      continue;
    }
    if (busy0 == 0) {
      if (parked == 0 && qdone) break;
      continue;
    }
    // a chain at its cap (defer_steps) takes no further step: it parks with fin = kFinSuspend and the next
    // batch (finish_parked) moves its lane state to carry_out
    if (CARRY && j >= 0 && fin < 0 && chain >= cap_at) fin = kFinSuspend;
    // the lanes with a rollout in flight take a step; with the cooperative collision check (COOP) the
    // whole wave takes part in its SAT tests, so the check sits outside the lanes' divergent region
    const bool act = j >= 0 && fin < 0;
#ifdef CLRRT_LANE_STATS
    {
      const int na = __popcll(__ballot(act));
      if (na > 0) {
        ls_w[qdone]++;
        ls_l[qdone] += na;
        ls_sparse[qdone] += na <= 8;
      }
    }
#endif
    if (!COOP && !act) continue;
    int best_s = 0x7fffffff;
    double d2 = 0.0;
    if (act) {
      steps++;
      chain++;
      // The abandon check's load of best[s] is issued BEFORE this step's row stores: vmcnt counts loads
      // and stores in issue order, so a load issued after the stores would wait for all ten of them to
      // complete (measured: ~60% of the kernel's wave time); issued here it only waits for the previous
      // step's stores, long retired.
      const bool check = !rp && (steps & (CLRRT_ABANDON_EVERY - 1)) == 0;
      best_s = check ? __atomic_load_n(&best[bs], __ATOMIC_RELAXED) : 0x7fffffff;
      if (pc) pc->mark(6);
      d2 = roll_step_pre(r, P, c7, c8, c9, w, pc);
    }
    double Dobs;
    if constexpr (COOP) {
      Dobs = obs_distance_coop(act, r, P, ov, w.box, cl, a.ctr ? a.ctr + 33 : nullptr);
      if (!act) continue;
    } else {
      Dobs = obs_distance<NEED_GAP>(r, P, ov, w.box);
    }
    if (pc) pc->mark(4);
    int o = roll_step_post(r, P, Dobs, d2);
#ifdef CLRRT_ROLL_PROFILE
    job_steps++;
    chain_steps = max(chain_steps, job_steps);
    if (qdone) {
      tail_steps++;
      if (!t_qdone) t_qdone = __builtin_amdgcn_s_memtime();
    }
#endif
    w.steps++;
    // a replay writes no row past its committed node's (a longer one is counted in n_rep_bad below)
    if (rows && (!rp || steps < nrows_rp)) store_row(rows + (int64_t)steps * 10, 1, r, c7, c8, c9);
    if (pc) pc->mark(5);
    if (o < 0 && steps >= P.n_steps_max) o = CLRRT_ROLL_ITERLIMIT;
    if (o >= 0) {
      fin = o;
    } else if (best_s < k) {
      // an earlier candidate of this sample succeeded: this result will not be looked at
      if (pass == 0) a.res[j].outcome = -1;
      a.res_gb[j].outcome = -1;
      j = -1;
    }
  }
  if (a.ctr) {  // per-wave sums (no block barrier)
    unsigned long long v0 = w.steps, v1 = w.scan, v2 = w.box;
#pragma unroll
    for (int q = 32; q > 0; q >>= 1) {
      v0 += (unsigned long long)__shfl_xor((long long)v0, q, 64);
      v1 += (unsigned long long)__shfl_xor((long long)v1, q, 64);
      v2 += (unsigned long long)__shfl_xor((long long)v2, q, 64);
    }
    if (lane == 0 && v0) {
      atomicAdd(&a.ctr[0], v0);
      atomicAdd(&a.ctr[1], v1);
      atomicAdd(&a.ctr[2], v2);
    }
    if (n_rep) {  // replays run, replays whose row count differs from the committed node's (must stay 0)
      atomicAdd(&a.ctr[60], n_rep);
      if (n_rep_bad) atomicAdd(&a.ctr[61], n_rep_bad);
    }
  }
#ifdef CLRRT_LANE_STATS
  if (a.ctr && lane == 0)
    for (int q = 0; q < 2; q++) {
      atomicAdd(&a.ctr[33 + 3 * q], ls_w[q]);
      atomicAdd(&a.ctr[34 + 3 * q], ls_l[q]);
      atomicAdd(&a.ctr[35 + 3 * q], ls_sparse[q]);
    }
#endif
#ifdef CLRRT_ROLL_PROFILE
  if (a.ctr && lane == 0)
    for (int q = 0; q < 8; q++) atomicAdd(&a.ctr[40 + q], (unsigned long long)pclk.wq[1 + q]);
  if (a.ctr) {
    // load balance: wave lifetimes (sum, max), the longest chain (max), waves; the queue drain (first
    // step after a fetch found it empty) of the wave, the busiest lane's steps after it
    unsigned long long cmax = chain_steps, tail = tail_steps;
#pragma unroll
    for (int q = 32; q > 0; q >>= 1) {
      cmax = max(cmax, (unsigned long long)__shfl_xor((long long)cmax, q, 64));
      tail = max(tail, (unsigned long long)__shfl_xor((long long)tail, q, 64));
    }
    if (lane == 0) {
      const unsigned long long life = __builtin_amdgcn_s_memtime() - t_start;
      atomicAdd(&a.ctr[48], life);
      atomicMax(&a.ctr[49], life);
      atomicMax(&a.ctr[50], cmax);
      atomicAdd(&a.ctr[51], 1ull);
      if (t_qdone) {
        atomicAdd(&a.ctr[52], t_qdone - t_start);
        atomicMax(&a.ctr[53], t_qdone - t_start);
      }
      atomicMax(&a.ctr[54], tail);
      atomicAdd(&a.ctr[55], tail);
    }
  }
#endif
}

// --------------------------------------------------------------------------------------------
// selection, goal bias, conflicts
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void fill_node(clrrt_node& n, const RollRes& r, int parent, float pcE,
                                          float pcS) {
  for (int k = 0; k < 10; k++) n.state[k] = r.st[k];
  n.ref_front[0] = r.fx; n.ref_front[1] = r.fy;
  n.ref_back[0] = r.bx; n.ref_back[1] = r.by;
  n.ref_vback = r.vback;
  n.ang_par = node_ang_par(r.bx, r.by, r.fx, r.fy);
  n.parent = parent;
  n.costE = (float)(r.costE + (double)pcE);
  n.costS = (float)(r.costS + (double)pcS);
  n.goal = r.outcome == CLRRT_ROLL_GOAL;
  n.nrows = r.nrows;
  n.owner = 0;
  n.row_offset = -1;
}


// The first candidate whose rollout succeeded (expandTree :150-160) and its goal-biased follow-up, for
// view v of the commit (SelArgs: a deferred sample of an earlier round, or a sample of this round).  A
// sample whose result still depends on a suspended rollout (deferred samples) is marked pending and
// commits nothing now.
__global__ void k_select(SelArgs a) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= a.B) return;
  const int g = v < a.nd ? a.view[v] : a.sbase + (v - a.nd);
  const int64_t g0 = (int64_t)g * CAND_K;
  const int nc = a.ncand[g];
  SampleOut o = {};
  o.k = -1;
  o.g = g;
  // (outcome, nrows) of every candidate loaded up front: independent loads, one memory latency instead
  // of one per candidate tried
  static_assert(offsetof(RollRes, nrows) == offsetof(RollRes, outcome) + 4 && offsetof(RollRes, outcome) % 8 == 0,
                "outcome and nrows load as one int2");
  int2 on[CAND_K];
#pragma unroll
  for (int k = 0; k < CAND_K; k++)
    on[k] = k < nc ? *(const int2*)&a.res[g0 + k].outcome : make_int2(-1, 1);
  bool pend = false;
#pragma unroll
  for (int k = 0; k < CAND_K; k++) {
    if (k >= nc || o.k >= 0 || pend) break;
    if (on[k].x == CLRRT_ROLL_PENDING) { pend = true; break; }
    o.rollouts++;
    o.steps += on[k].y - 1;
    o.f_col += on[k].x == CLRRT_ROLL_COLLISION;
    o.f_acc += on[k].x == CLRRT_ROLL_ACCLIMIT;
    o.f_it += on[k].x == CLRRT_ROLL_ITERLIMIT;
    if (on[k].x == CLRRT_ROLL_END || on[k].x == CLRRT_ROLL_GOAL) o.k = k;
  }
  if (!pend && o.k >= 0 && a.res_gb[g0 + o.k].outcome == CLRRT_ROLL_PENDING) pend = true;
  if (pend) {  // resolved by a later commit
    SampleOut z = {};
    z.k = -1;
    z.g = g;
    z.pend = 1;
    a.so[v] = z;
    if (a.gv) a.gv[v] = g;
    if (a.pend) a.pend[v] = 1;
    if (a.new_pend && v >= a.nd) atomicAdd(a.new_pend, 1);  // a sample of this round deferred (statistics)
    return;
  }
  if (a.gv) a.gv[v] = g;
  if (a.pend) a.pend[v] = 0;
  // EXACT-mode conflict threshold: the key a new node must beat (<=) to be tried before the result.
  // (keys are kept for the round's own samples only: null for views into the rings, BATCH needs no threshold)
  o.thr = !a.ckey ? __builtin_inff()
          : o.k >= 0 ? a.ckey[g0 + o.k] : (nc == a.p.sort_limit ? a.ckey[g0 + nc - 1] : __builtin_inff());
  o.gb_ok = 0;
  if (o.k >= 0) {
    const int pid = a.cand[g0 + o.k];
    const clrrt_node& par = a.tree[pid];
    clrrt_node n;
    fill_node(n, a.res[g0 + o.k], pid, par.costE, par.costS);
    a.regnodes[v] = n;
    o.nrows_reg = n.nrows;
    const RollRes& gr = a.res_gb[g0 + o.k];
    if (gr.outcome >= 0) {  // the gate passed and the goal-biased rollout ran (:163-173)
      o.rollouts++;
      o.steps += gr.nrows - 1;
      o.f_col += gr.outcome == CLRRT_ROLL_COLLISION;
      o.f_acc += gr.outcome == CLRRT_ROLL_ACCLIMIT;
      o.f_it += gr.outcome == CLRRT_ROLL_ITERLIMIT;
      if (gr.outcome == CLRRT_ROLL_END || gr.outcome == CLRRT_ROLL_GOAL) {
        clrrt_node gn;
        fill_node(gn, gr, CLRRT_PARENT_PREV, n.costE, n.costS);
        a.gbnodes[v] = gn;
        o.gb_ok = 1;
        o.nrows_gb = gn.nrows;
      }
    }
  }
  a.so[v] = o;
}

// EXACT mode: sample j conflicts when a node produced by an earlier sample of the round would sort
// at or before j's accepted candidate (or into j's candidate window when nothing was accepted).
// A sample whose selection involves equal keys conflicts with ANY node appended before it in the
// round: std::sort orders equal keys by its partitioning of the whole (grown) array.
__global__ void k_conflict(DevParams p, int B, const clrrt_sample* __restrict__ S,
                           const clrrt_node* __restrict__ regnodes, const clrrt_node* __restrict__ gbnodes,
                           const SampleOut* __restrict__ so, const int* __restrict__ ctie, int* first_conflict) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  const double sx = S[j].x, sy = S[j].y;
  const int ex = S[j].explore;
  const float thr = so[j].thr;
  const bool tie = ctie[j] != 0;
  bool conflict = false;
  for (int k = 0; k < j && !conflict; k++) {
    if (so[k].k < 0) continue;
    if (tie) { conflict = true; break; }
    for (int w = 0; w < 2; w++) {
      if (w == 1 && !so[k].gb_ok) break;
      const clrrt_node& n = w == 0 ? regnodes[k] : gbnodes[k];
      float c, s;
      glibc::sincosf((float)(-n.state[2] - 0.0), s, c);  // dubinsDistance: cos/sin of one float -> sincosf
      float key = dubins_key(sx, sy, n.state[0], n.state[1], c, s);
      if (!ex) key = n.costE + key;
      if (!(key > thr) && feasible_node(n.ref_back[0], n.ref_back[1], n.ang_par, sx, sy, p.feas_len)) {
        conflict = true;
        break;
      }
    }
  }
  if (conflict) atomicMin(first_conflict, j);
}

// EXACT mode, fix-ups: a conflict of sample j with nodes appended earlier in the round does not always change
// j's result.  The reference tries j's candidates in key order until the first success (rrtplanner.cpp:150-160):
// a new node n that sorts before j's accepted candidate k is tried before it, and if n's rollout fails the result
// is still k's (k stays inside the sortLimit window as long as k + m <= sortLimit - 1 for the m such nodes) with
// n's rollout added to j's counters.  So the conflicting nodes are rolled out for j (the fix-up launch) and j
// stands when all of them fail.  Not resolvable this way (fix_n = -1, j conflicts as before): a tie among j's
// keys (std::sort's order of equal keys depends on the whole array), a new node whose key equals j's threshold
// (its order against k is the sort's), more than FIX_MAX new nodes, and k pushed out of the window.  (A sample
// without a result is resolved by ranking the new nodes among its old candidates: the grown window's first
// sortLimit entries are rolled out and the old ones it no longer reaches have their counters subtracted.)
__global__ void k_conflict_fix(DevParams p, int B, const clrrt_sample* __restrict__ S,
                               const clrrt_node* __restrict__ regnodes, const clrrt_node* __restrict__ gbnodes,
                               const SampleOut* __restrict__ so, const int* __restrict__ ctie,
                               const int* __restrict__ ncand, const float* __restrict__ ckey,
                               const RollRes* __restrict__ res, int* __restrict__ fix_n, int* __restrict__ fix_ids,
                               int* __restrict__ fix_adj) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  const double sx = S[j].x, sy = S[j].y;
  const int ex = S[j].explore;
  const float thr = so[j].thr;
  const int kk = so[j].k, nc = ncand[j], lim = p.sort_limit;
  const int g0 = so[j].g * CAND_K;
  // Equal keys in j's list leave their order to std::sort, which the new nodes can change.  With a result k whose
  // key is unique in the list (and k not the window's last entry, whose successor is not kept), every
  // reordering keeps the set of candidates tried before k (all keys below k's: all failed) and k itself, so the
  // result stands; otherwise a tie ends the prefix at any appended node, as before.
  const bool tie = ctie[j] != 0 &&
                   !(kk >= 0 && kk < lim - 1 && (kk == 0 || ckey[g0 + kk - 1] != ckey[g0 + kk]) &&
                     (kk + 1 >= nc || ckey[g0 + kk + 1] != ckey[g0 + kk]));
  int m = 0;
  int ids[FIX_MAX];
  float nk[FIX_MAX];
  int bad = 0;  // why not resolvable: 1 tie, 2 a key equal to the threshold, 3 > FIX_MAX, 4 k pushed out
  for (int k = 0; k < j && !bad; k++) {
    if (so[k].k < 0) continue;
    if (tie) { bad = 1; break; }
    for (int w = 0; w < 2; w++) {
      if (w == 1 && !so[k].gb_ok) break;
      const clrrt_node& n = w == 0 ? regnodes[k] : gbnodes[k];
      float c, s;
      glibc::sincosf((float)(-n.state[2] - 0.0), s, c);  // dubinsDistance: cos/sin of one float -> sincosf
      float key = dubins_key(sx, sy, n.state[0], n.state[1], c, s);
      if (!ex) key = n.costE + key;
      if (!(key > thr) && feasible_node(n.ref_back[0], n.ref_back[1], n.ang_par, sx, sy, p.feas_len)) {
        if (key == thr || m == FIX_MAX) { bad = key == thr ? 2 : 3; break; }
        ids[m] = 2 * k + w;
        nk[m] = key;
        m++;
      }
    }
  }
  int adj[5] = {0, 0, 0, 0, 0};  // counters of old candidates the grown window no longer reaches (subtracted)
  int mw = m;                     // new nodes inside the window
  if (!bad && m > 0) {
    if (kk >= 0) {
      // every new node precedes the accepted candidate (key < thr): all are tried, k moves to k + m
      if (kk + m > lim - 1) bad = 4;
    } else {
      // no result: the reference tries the first sortLimit of (old candidates + new nodes) by key.  Equal keys
      // would leave that order to std::sort: not resolvable.
      for (int a = 0; a < m && !bad; a++) {
        for (int b = a + 1; b < m; b++)
          if (nk[a] == nk[b]) bad = 1;
        for (int o = 0; o < nc; o++)
          if (nk[a] == ckey[g0 + o]) bad = 1;
      }
      if (!bad) {
        mw = 0;
        for (int a = 0; a < m; a++) {  // rank among old and new
          int r = 0;
          for (int o = 0; o < nc; o++) r += ckey[g0 + o] < nk[a];
          for (int b = 0; b < m; b++) r += nk[b] < nk[a];
          if (r < lim) ids[mw++] = ids[a];
        }
        for (int o = 0; o < nc; o++) {
          int r = o;
          for (int b = 0; b < m; b++) r += nk[b] < ckey[g0 + o];
          if (r >= lim) {  // pushed out: its rollout (a failure, run speculatively) is not the reference's
            const RollRes& q = res[g0 + o];
            if (q.outcome < 0) continue;
            adj[0] -= 1;
            adj[1] -= q.nrows - 1;
            adj[2] -= q.outcome == CLRRT_ROLL_COLLISION;
            adj[3] -= q.outcome == CLRRT_ROLL_ACCLIMIT;
            adj[4] -= q.outcome == CLRRT_ROLL_ITERLIMIT;
          }
        }
      }
    }
  }
  for (int a = 0; a < (bad ? 0 : mw); a++) fix_ids[j * FIX_MAX + a] = ids[a];
#pragma unroll
  for (int q = 0; q < 5; q++) fix_adj[j * 5 + q] = adj[q];
  fix_n[j] = bad ? -bad : mw;
}

// --------------------------------------------------------------------------------------------
// compaction of committed samples (one block, sequential chunks + block scan)
// --------------------------------------------------------------------------------------------
// Compaction of committed samples in three passes: per-sample counts (nodes in the low 24 bits, rows
// above them; a round has < 2^24 nodes and < 2^40 rows), a device-wide exclusive scan (hipcub), and a
// scatter of the node records and row-copy jobs.  The round's work counters are block-reduced.
__global__ void __launch_bounds__(256) k_compact_count(int L, const SampleOut* __restrict__ so,
                                                       const clrrt_node* __restrict__ regnodes,
                                                       const clrrt_node* __restrict__ gbnodes,
                                                       uint64_t* __restrict__ packed, int64_t* __restrict__ totals) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long cnt[6] = {0, 0, 0, 0, 0, 0};
  if (s < L) {
    const SampleOut& o = so[s];
    uint64_t nn = 0, nr = 0;
    if (o.k >= 0) { nn++; nr += (uint64_t)o.nrows_reg; cnt[5] += regnodes[s].goal; }
    if (o.gb_ok) { nn++; nr += (uint64_t)o.nrows_gb; cnt[5] += gbnodes[s].goal; }
    cnt[0] = o.steps; cnt[1] = o.f_col; cnt[2] = o.f_acc; cnt[3] = o.f_it; cnt[4] = o.rollouts;
    packed[s] = (nr << 24) | nn;
  }
  __shared__ unsigned long long s_cnt[6];
  if (threadIdx.x < 6) s_cnt[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 6; c++) {
    unsigned long long v = cnt[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&s_cnt[c], v);
  }
  __syncthreads();
  if (threadIdx.x < 6 && s_cnt[threadIdx.x]) atomicAdd((unsigned long long*)&totals[2 + threadIdx.x], s_cnt[threadIdx.x]);
}

__global__ void __launch_bounds__(256) k_compact_scatter(int L, const SampleOut* __restrict__ so,
                                                         const clrrt_node* __restrict__ regnodes,
                                                         const clrrt_node* __restrict__ gbnodes,
                                                         const uint64_t* __restrict__ packed,
                                                         const uint64_t* __restrict__ scanned, int64_t row_base,
                                                         int rank, clrrt_node* __restrict__ out, Job* __restrict__ jobs,
                                                         int64_t* __restrict__ totals, int tag_slot, int tag_R,
                                                         int tag_B) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= L) return;
  const uint64_t off = scanned[s];
  int64_t node_off = (int64_t)(off & 0xffffffu), row_off = (int64_t)(off >> 24);
  if (s == L - 1) {
    const uint64_t tot = off + packed[s];
    totals[0] = (int64_t)(tot & 0xffffffu);
    totals[1] = (int64_t)(tot >> 24);
  }
  const SampleOut& o = so[s];
  // sharded rounds with deferred samples: the record's age in rounds (0: this round's sample) rides in
  // bits 8..15 of `goal` through the exchange, which orders the union oldest round first (k_xorder_keys)
  const int tag = tag_R > 0 ? ((tag_slot - o.g / tag_B + tag_R) % tag_R) << 8 : 0;
  if (o.k >= 0) {
    clrrt_node n = regnodes[s];
    n.goal |= tag;
    n.owner = rank;
    n.row_offset = row_base + row_off;
    out[node_off] = n;
    Job jb;  // row copy / replay: ring job (g, k*) pass 0 -> arena
    jb.parent = o.g * CAND_K + o.k; jb.from_reg = 0; jb.gb = 0; jb.pad = 0;
    jb.sx = 0; jb.sy = 0;
    jb.row_off = row_base + row_off;
    jobs[node_off] = jb;
    node_off++;
    row_off += o.nrows_reg;
  }
  if (o.gb_ok) {
    clrrt_node n = gbnodes[s];
    n.goal |= tag;
    n.owner = rank;
    n.row_offset = row_base + row_off;
    out[node_off] = n;
    Job jb;  // row copy / replay: ring job (g, k*) pass 1 (goal-biased rollout) -> arena
    jb.parent = o.g * CAND_K + o.k; jb.from_reg = 0; jb.gb = 1; jb.pad = 0;
    jb.sx = 0; jb.sy = 0;
    jb.row_off = row_base + row_off;
    jobs[node_off] = jb;
  }
}

// Move committed trajectories (Node::tra) from their job slots into the arena: one block per node.
__global__ void __launch_bounds__(256) k_copy_rows(const Job* __restrict__ jobs, const clrrt_node* __restrict__ recs,
                                                   const double* __restrict__ slots, int slot_rows, int slot_jobs,
                                                   double* __restrict__ arena) {
  const int i = blockIdx.x;
  const Job jb = jobs[i];
  const int n = recs[i].nrows * 10;
  const double* src = slots + ((int64_t)jb.gb * slot_jobs + jb.parent) * slot_rows * 10;
  double* dst = arena + jb.row_off * 10;
  for (int t = threadIdx.x; t < n; t += blockDim.x) dst[t] = src[t];
}

// Commit with deferred rows: the accepted rollouts' start states for the next k_roll_run's replays (one
// lane per committed node; jobs[] from k_compact_scatter: parent = the job, gb = pass).
__global__ void __launch_bounds__(256) k_replay_gather(const Job* __restrict__ jobs, const clrrt_node* __restrict__ recs,
                                                       int n, const clrrt_node* __restrict__ tree,
                                                       const int* __restrict__ cand, const clrrt_sample* __restrict__ S,
                                                       const RollRes* __restrict__ res, Replay* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Job jb = jobs[i];
  Replay o;
  o.row_off = jb.row_off;
  o.nrows = recs[i].nrows;
  o.pad = 0;
  o.src.gb = jb.gb;
  o.src.pad = 0;
  if (jb.gb) {  // from the end of the regular rollout of the same job
    const RollRes& g = res[jb.parent];
#pragma unroll
    for (int q = 0; q < 10; q++) o.src.st[q] = g.st[q];
    o.src.bx = g.bx; o.src.by = g.by; o.src.vb = g.vback;
    o.src.sx = o.src.sy = 0.0;
  } else {  // from the job's parent node toward its sample
    const clrrt_node& p = tree[cand[jb.parent]];
#pragma unroll
    for (int q = 0; q < 10; q++) o.src.st[q] = p.state[q];
    o.src.bx = p.ref_back[0]; o.src.by = p.ref_back[1]; o.src.vb = p.ref_vback;
    o.src.sx = S[jb.parent / CAND_K].x; o.src.sy = S[jb.parent / CAND_K].y;
  }
  out[i] = o;
}

size_t replay_bytes() { return sizeof(Replay); }

hipError_t launch_replay_gather(hipStream_t st, const Job* jobs, const clrrt_node* recs, int n, const clrrt_node* tree,
                                const int* cand, const clrrt_sample* S, const RollRes* res, void* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_replay_gather, dim3((n + 255) / 256), dim3(256), 0, st, jobs, recs, n, tree, cand, S, res,
                     (Replay*)out);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_bbox(const clrrt_node* __restrict__ recs, const int64_t* n_dev, int n_host,
                                              double* __restrict__ out4) {
  __shared__ double s[4][256];
  const int n = n_dev ? (int)*n_dev : n_host;
  double v[4] = {HUGE_VAL, HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = recs[i].state[0], y = recs[i].state[1];
    if (isfinite(x) && isfinite(y)) {
      v[0] = fmin(v[0], x); v[1] = fmin(v[1], y); v[2] = fmax(v[2], x); v[3] = fmax(v[3], y);
    }
  }
  for (int k = 0; k < 4; k++) s[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
      s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + off]);
      s[1][threadIdx.x] = fmin(s[1][threadIdx.x], s[1][threadIdx.x + off]);
      s[2][threadIdx.x] = fmax(s[2][threadIdx.x], s[2][threadIdx.x + off]);
      s[3][threadIdx.x] = fmax(s[3][threadIdx.x], s[3][threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) out4[threadIdx.x] = s[threadIdx.x][0];
}

// RRT.addNode for n records: resolve GB parents (CLRRT_PARENT_PREV -> the record before) and build
// the nearest-node mirror.
__global__ void k_append(const clrrt_node* __restrict__ in, int n, int64_t base, clrrt_node* __restrict__ tree,
                         NnRec* __restrict__ nn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  clrrt_node d = in[i];
  if (d.parent == CLRRT_PARENT_PREV) d.parent = (int32_t)(base + i - 1);
  tree[base + i] = d;
  NnRec r;
  r.x = d.state[0]; r.y = d.state[1];
  r.bx = d.ref_back[0]; r.by = d.ref_back[1];
  r.ang_par = d.ang_par;
  float ang = (float)(-d.state[2] - 0.0);
  glibc::sincosf(ang, r.s, r.c);  // dubinsDistance rrtplanner.cpp:376-378: glibc sincosf
  r.costE = d.costE;
  r.id = (int32_t)(base + i);
  r.ca = cosf((float)d.ang_par); r.sa = sinf((float)d.ang_par);
  nn[base + i] = r;
}

// Nearest-node mirror record of tree node `id`.
__device__ __forceinline__ NnRec nn_record(const clrrt_node& d, int64_t id) {
  NnRec r;
  r.x = d.state[0]; r.y = d.state[1];
  r.bx = d.ref_back[0]; r.by = d.ref_back[1];
  r.ang_par = d.ang_par;
  float ang = (float)(-d.state[2] - 0.0);
  glibc::sincosf(ang, r.s, r.c);  // dubinsDistance rrtplanner.cpp:376-378: glibc sincosf
  r.costE = d.costE;
  r.id = (int32_t)id;
  r.ca = cosf((float)d.ang_par); r.sa = sinf((float)d.ang_par);
  return r;
}

// addInitialNode rrtplanner.cpp:21-37: reference = linspace(0, 1, floor(1/0.1)) at v = state[4].
__device__ void init_root(const double* st, clrrt_node* tree, NnRec* nn, double* arena, int owner) {
  const int N = (int)floor(sqrt(1.0 * 1.0 + 0.0 * 0.0) / 0.1);
  double h = (1.0 - 0.0) / (double)(uint64_t)(N - 1);
  double x = 0.0;
  for (int i = 1; i < N; i++) x += h;
  clrrt_node n;
  for (int k = 0; k < 10; k++) { n.state[k] = st[k]; arena[k] = st[k]; }
  n.ref_front[0] = 0.0; n.ref_front[1] = 0.0;
  n.ref_back[0] = x; n.ref_back[1] = 0.0;
  n.ref_vback = st[4];
  n.ang_par = node_ang_par(x, 0.0, 0.0, 0.0);
  n.parent = -1;
  n.costE = 0.f; n.costS = 0.f;
  n.goal = 0;
  n.nrows = 1;
  n.owner = owner;
  n.row_offset = 0;
  tree[0] = n;
  nn[0] = nn_record(n, 0);
}

__global__ void k_init_root(const double* __restrict__ st, clrrt_node* tree, NnRec* nn, double* arena) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  init_root(st, tree, nn, arena, 0);
}

// Goal nodes of the tree (extractBestPath's pair_vector, rrtplanner.cpp:330-335) -- wave-aggregated
// append; the host restores tree order by id before replaying the reference's sort.
__global__ void __launch_bounds__(256) k_goal_gather(const clrrt_node* __restrict__ tree, int64_t n,
                                                     GoalRec* __restrict__ out, int* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - threadIdx.x < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool g = i < n && tree[i].goal != 0;
    const unsigned long long m = __ballot(g);
    if (m == 0) continue;
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(cnt, __popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (g) {
      const int off = __popcll(m & ((1ull << lane) - 1ull));
      out[base + off] = GoalRec{(int32_t)i, tree[i].costS};
    }
  }
}

// Backtracking from the chosen goal node to the root (rrtplanner.cpp:339-346): parents precede
// their children, so the chain ends at the root (parent -1) within n steps.
__global__ void k_backtrack(const clrrt_node* __restrict__ tree, int64_t n, int start, int cap,
                            int* __restrict__ path, int* __restrict__ len) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int k = 0;
  int64_t p = start;
  while (p >= 0 && p < n && k <= n) {
    if (k < cap) path[k] = (int)p;
    k++;
    p = tree[p].parent;
  }
  *len = (p == -1) ? k : -1;  // -1: a broken chain (parent outside the tree)
}

// ----------------------------------------------------------------- committed path / re-init
__global__ void k_gather_nodes(const clrrt_node* __restrict__ tree, const int* __restrict__ ids, int n,
                               clrrt_node* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = tree[ids[i]];
}

// transformPointWorldToCar / CarToWorld (transformations.cpp:6-17); sin and cos of one argument
// in one function: the generic sincos, as the oracle's restatement.
__device__ __forceinline__ void point_world_to_car(double& Xw, double& Yw, double P0, double P1, double s,
                                                   double c) {
  double Xc = Xw * c - P0 * c - P1 * s + Yw * s;
  double Yc = Yw * c - P1 * c + P0 * s - Xw * s;
  Xw = Xc; Yw = Yc;
}
__device__ __forceinline__ void point_car_to_world(double& Xc, double& Yc, double P0, double P1, double s,
                                                   double c) {
  double Xw = c * Xc - s * Yc + P0;
  double Yw = s * Xc + c * Yc + P1;
  Xc = Xw; Yc = Yw;
}

// transformNodesWorldToCar / CarToworld (transformations.cpp:289-315): node state (x, y, heading),
// the reference end points (the only reference points the engine keeps; the reference transforms
// each point independently, so front/back come out the same), and (x, y) of every row.
__global__ void __launch_bounds__(256) k_path_transform(clrrt_node* __restrict__ nodes, int n,
                                                        double* __restrict__ rows, int64_t nrows, int to_world,
                                                        double P0, double P1, double P2) {
  glibc::stage_tables();
  double s, c;
  glibc::sincos(P2, s, c);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    clrrt_node& d = nodes[i];
    if (to_world) {
      point_car_to_world(d.state[0], d.state[1], P0, P1, s, c);
      d.state[2] += P2;
      point_car_to_world(d.ref_front[0], d.ref_front[1], P0, P1, s, c);
      point_car_to_world(d.ref_back[0], d.ref_back[1], P0, P1, s, c);
    } else {
      point_world_to_car(d.state[0], d.state[1], P0, P1, s, c);
      d.state[2] -= P2;
      point_world_to_car(d.ref_front[0], d.ref_front[1], P0, P1, s, c);
      point_world_to_car(d.ref_back[0], d.ref_back[1], P0, P1, s, c);
    }
    d.ang_par = node_ang_par(d.ref_back[0], d.ref_back[1], d.ref_front[0], d.ref_front[1]);
  } else if (i - n < nrows) {
    double* r = rows + (i - n) * 10;
    if (to_world) point_car_to_world(r[0], r[1], P0, P1, s, c);
    else point_world_to_car(r[0], r[1], P0, P1, s, c);
  }
}

// initializeTree rrtplanner.cpp:39-95 + getNodeCost :104-119, one workgroup (a committed path is
// a few nodes / a few thousand rows: latency, not throughput).  Row checks run across the block;
// the cost recurrence (costS float, read back as the next node's double parent cost) on lane 0.
__global__ void __launch_bounds__(256) k_tree_reinit(ReinitArgs a) {
  glibc::stage_tables();
  __shared__ int s_kept, s_coll;
  __shared__ long long s_rows;
  const int tid = threadIdx.x;
  const DevParams& p = a.p;
  const ObsView ov{a.obs, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                   p.coll_mode == CLRRT_COLLISION_OBB ? p.n_obs : 0, 0, 0, 0, 0.f, 0.f, 0.f};
  int* goal = a.kidx + a.n;
  // :51-57 erase(it--) over the path = keep the nodes whose last row has x >= 0 (or NaN)
  if (tid == 0) {
    int k = 0;
    long long r = 0;
    for (int i = 0; i < a.n; i++) {
      const clrrt_node& h = a.pn[i];
      const double xb = a.prow[(h.row_offset + h.nrows - 1) * 10];
      if (!(xb < 0)) {
        a.kidx[k] = i;
        a.koff[k] = r;
        goal[k] = 0;
        r += h.nrows;
        k++;
      }
    }
    s_kept = k;
    s_rows = r;
    s_coll = 0;
  }
  __syncthreads();
  const int kept = s_kept;
  const int64_t rows = s_rows;
  if (a.n == 0 || kept == 0) {
    if (tid == 0) {
      init_root(a.car, a.tree, a.nn, a.arena, a.rank);
      a.out[0] = a.n == 0 ? CLRRT_REINIT_EMPTY : CLRRT_REINIT_ALL_ERASED;
      a.out[1] = 1; a.out[2] = 1;
    }
    return;
  }
  // :60-69 goal flags, :72-81 collisions, getNodeCost's per-row terms
  for (int k = 0; k < kept; k++) {
    const clrrt_node& h = a.pn[a.kidx[k]];
    for (int i = tid; i < h.nrows; i += blockDim.x) {
      const double* x = a.prow + (h.row_offset + i) * 10;
      const double ex = x[0] - p.g0;
      const double Dgoal = sqrt(ex * ex + x[1] * x[1]);
      const double Hgoal = fabs(x[2] - p.g2);
      const double dVgoal = fabs(x[4] - p.g3);
      if ((Dgoal <= 1) && (Hgoal <= 0.05) && (dVgoal <= 0.1)) goal[k] = 1;
      Roll r;
      r.x0 = x[0]; r.x1 = x[1]; r.x2 = x[2]; r.x6 = x[6];
      glibc::sincos(r.x2, r.s2, r.c2);
      uint32_t tests = 0;
      const double Dobs = obs_distance<true>(r, p, ov, tests);
      if (Dobs == 0) s_coll = 1;
      const double kappa = glibc::tan(x[3]) / p.L;
      double term = p.W0 * x[4] * p.dt + p.W1 * fabs(kappa);
      if (p.use_exp) term = term + p.W2 * glibc::exp(-p.W3 * Dobs);  // glibc's exp, restated
      double* t = a.terms + (a.koff[k] + i) * 2;
      t[0] = term;
      t[1] = p.bend ? p.W4 * dist_to_lane(x[0], x[1], p.lane_shift0, p.Cxy1, p.Cxy2) : 0.0;
    }
  }
  __syncthreads();
  if (s_coll) {
    if (tid == 0) {
      init_root(a.car, a.tree, a.nn, a.arena, a.rank);
      a.out[0] = CLRRT_REINIT_COLLISION;
      a.out[1] = 1; a.out[2] = 1;
    }
    return;
  }
  if (kept > a.max_nodes || rows > a.max_rows) {  // the host checks the path's totals; kept fits
    if (tid == 0) { a.out[0] = -1; a.out[1] = kept; a.out[2] = rows; }
    return;
  }
  // :84-87 cost recurrence
  if (tid == 0) {
    double parent = 0;
    for (int k = 0; k < kept; k++) {
      const clrrt_node& h = a.pn[a.kidx[k]];
      double cost = parent;
      const double* t = a.terms + a.koff[k] * 2;
      for (int i = 0; i < h.nrows; i++) {
        cost += t[2 * i];
        if (p.bend) cost += t[2 * i + 1];
      }
      a.costs[k] = (float)cost;
      parent = (double)a.costs[k];
    }
  }
  __syncthreads();
  // :90-93 the chain, rows into the arena
  for (int k = tid; k < kept; k += blockDim.x) {
    clrrt_node h = a.pn[a.kidx[k]];
    h.parent = k - 1;
    h.goal = goal[k];
    h.costS = a.costs[k];
    h.row_offset = a.koff[k];
    h.owner = a.rank;
    a.tree[k] = h;
    a.nn[k] = nn_record(h, k);
  }
  for (int k = 0; k < kept; k++) {
    const clrrt_node& h = a.pn[a.kidx[k]];
    const double* src = a.prow + h.row_offset * 10;
    double* dst = a.arena + a.koff[k] * 10;
    for (int e = tid; e < h.nrows * 10; e += blockDim.x) dst[e] = src[e];
  }
  if (tid == 0) { a.out[0] = CLRRT_REINIT_KEPT; a.out[1] = kept; a.out[2] = rows; }
}

// Elementary functions as the kernels evaluate them (test hook: bit-compared with the host libm).
__global__ void k_selftest_math(int fn, const double* __restrict__ a, const double* __restrict__ b, int n,
                                double* __restrict__ out) {
  glibc::stage_tables();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = a[i], y = b[i];
  const float xf = (float)x, yf = (float)y;
  double r;
  switch (fn) {
    case 0: r = glibc::sin(x); break;
    case 1: r = glibc::cos(x); break;
    case 2: r = glibc::tan(x); break;
    case 3: r = sqrt(x); break;
    case 4: r = fmod(x, y); break;
    case 5: r = glibc::atan2(x, y); break;
    case 6: r = glibc::exp(x); break;
    case 7: r = x / y; break;
    case 8: { float sf, cf; glibc::sincosf(xf, sf, cf); r = (double)cf; } break;
    case 9: r = (double)glibc::sinf(xf); break;
    case 10: r = (double)glibcf::atan2f(xf, yf); break;
    case 11: r = (double)glibcf::acosf(xf); break;
    case 12: r = (double)glibcf::asinf(xf); break;
    case 13: r = (double)sqrtf(xf); break;
    case 14: r = (double)(xf / yf); break;
    case 15: r = round(x); break;
    case 16: { double sx, cx; glibc::sincos(x, sx, cx); r = sx; } break;
    case 17: { double sx, cx; glibc::sincos(x, sx, cx); r = cx; } break;
    case 24: case 25: case 26: case 27: case 28: {  // glibc::step_trig (x2 = x, x3 = y): s2, c2, swp, cwp, t3
      double v[5];
      if (!glibc::step_trig(x, y, v[0], v[1], v[2], v[3], v[4])) {
        glibc::sincos_sel(x, v[0], v[1]);
        glibc::sin_cos_fma_sel(x, v[2], v[3]);
        v[4] = glibc::tan(y);
      }
      r = v[fn - 24];
    } break;
    case 20: { double sx, cx; glibc::sincos_sel(x, sx, cx); r = sx; } break;
    case 21: { double sx, cx; glibc::sincos_sel(x, sx, cx); r = cx; } break;
    case 22: { double sx, cx; glibc::sin_cos_fma_sel(x, sx, cx); r = sx; } break;
    case 23: { double sx, cx; glibc::sin_cos_fma_sel(x, sx, cx); r = cx; } break;
    case 18: {  // diagnostics: latency of a rollout step's trig (sincos, cos, sin, tan), y[0] iterations
      double z = x;
      for (int it = 0; it < (int)y; it++) {
        double sx, cx;
        glibc::sincos(z, sx, cx);
        const double c2 = glibc::cos(z), s2 = glibc::sin(z), t3 = glibc::tan(0.5 * sx);
        z = z + 1e-3 * (sx + cx + c2 + s2 + t3);
      }
      r = z;
    } break;
    case 19: {  // diagnostics: the same loop with FP64 multiply-adds only (no table, no branch)
      double z = x;
      for (int it = 0; it < (int)y; it++) {
        double q = z;
#pragma unroll 1
        for (int k = 0; k < 100; k++) q = q * 0.999999 + 1e-9;
        z = z + 1e-3 * q;
      }
      r = z;
    } break;
    default: r = 0.0; break;
  }
  out[i] = r;
}

// Hot-path units exactly as the kernels evaluate them, one case per lane (test hook: bit-compared with
// the reference's own code through tests/golden/ref_units.npz).  Formats: clrrt_selftest_units.
__global__ void k_selftest_units(int unit, const double* __restrict__ in, const BakedObs* __restrict__ obs, int n,
                                 DevParams p, const DevParams* __restrict__ cp, double* __restrict__ out) {
  glibc::stage_tables();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (unit) {
    case CLRRT_UNIT_DUBINS: {  // the nearest-node record's rotation (nn_record) + dubins_key
      const double* a = in + 6 * (int64_t)i;
      clrrt_node d;
      d.state[0] = a[2]; d.state[1] = a[3]; d.state[2] = a[4];
      d.ref_back[0] = 0.0; d.ref_back[1] = 0.0;
      d.ang_par = 0.0;
      d.costE = (float)a[5];
      const NnRec r = nn_record(d, 0);
      const float key = dubins_key(a[0], a[1], r.x, r.y, r.c, r.s);
      out[2 * (int64_t)i] = (double)key;
      out[2 * (int64_t)i + 1] = (double)(r.costE + key);
    } break;
    case CLRRT_UNIT_FEASIBLE: {  // angPar as the node records carry it, then the three deciders
      const double* a = in + 7 * (int64_t)i;
      const DevParams& q = cp[i];
      clrrt_node d;
      d.state[0] = 0.0; d.state[1] = 0.0; d.state[2] = 0.0;
      d.ref_back[0] = a[4]; d.ref_back[1] = a[5];
      d.ang_par = node_ang_par(a[4], a[5], a[2], a[3]);
      d.costE = 0.f;
      const NnRec r = nn_record(d, 0);
      const bool exact = feasible_node(r.bx, r.by, r.ang_par, a[0], a[1], q.feas_len);
      const bool search = feasible_search(a[0], a[1], r.bx, r.by, r.ca, r.sa, r.ang_par, q.feas_len);
      const float qx = (float)(a[0] - r.x), qy = (float)(a[1] - r.y);
      const float feas2 = nn_feas2(q.feas_len);
      const bool pre = nn_prefilter(a[0], a[1], qx, qy, r.c, r.s, r.ca, r.sa, r.bx, r.by, 0.f, 1,
                                    __builtin_inff(), feas2);
      out[3 * (int64_t)i] = exact ? 1.0 : 0.0;
      out[3 * (int64_t)i + 1] = search ? 1.0 : 0.0;
      out[3 * (int64_t)i + 2] = pre ? 1.0 : 0.0;
    } break;
    case CLRRT_UNIT_GOALBIAS: {
      const double* a = in + 8 * (int64_t)i;
      const double st[2] = {a[4], a[5]};
      out[i] = feasible_goal_bias(cp[i], st, a[6], a[7]) ? 1.0 : 0.0;
    } break;
    case CLRRT_UNIT_GOALREF: {  // getGoalReference's two segments + the goal-biased profile
      const double* a = in + 8 * (int64_t)i;
      const DevParams& q = cp[i];
      RefD R = make_goal_ref(a[4], a[5], q);
      double* row = out + (int64_t)(1 + 3 * CLRRT_UNIT_PROFILE_NMAX) * i;
      row[0] = (double)R.N;
      double x = R.a1x, y = R.a1y;
      for (int j = 0; j < R.N; j++) {
        if (j < CLRRT_UNIT_PROFILE_NMAX) {
          row[1 + CLRRT_UNIT_PROFILE_NMAX + j] = x;
          row[1 + 2 * CLRRT_UNIT_PROFILE_NMAX + j] = y;
        }
        if (j == R.N - 1) { R.bx = x; R.by = y; }
        ref_next(R, j, x, y);
      }
      const Prof P = make_profile(R, a[6], q, true);
      for (int j = 0; j < R.N && j < CLRRT_UNIT_PROFILE_NMAX; j++) row[1 + j] = prof_v(P, j);
    } break;
    case CLRRT_UNIT_CTRL: {  // Simulation ctor's controller + profile, then getControls per state
      const int K = CLRRT_UNIT_CTRL_K;
      const double* a = in + (int64_t)(12 + 6 * K) * i;
      double* o = out + (int64_t)(4 + 8 * K) * i;
      const DevParams& q = cp[i];
      const bool GB = a[0] != 0.0;
      const RefD R = GB ? make_goal_ref(a[1], a[2], q) : make_ref(a[1], a[2], a[3], a[4], q);
      const double* st = a + 12;
      double s0[10];
      for (int k = 0; k < 10; k++) s0[k] = k < 6 ? st[k] : 0.0;
      Roll r;
      double Px, Py;
      roll_init(r, s0, R, a[9], GB, q, &Px, &Py);
      o[0] = (double)r.wp; o[1] = (double)r.endr; o[2] = Px; o[3] = Py;
      for (int j = 0; j < K; j++) {
        const double* x = st + 6 * j;
        r.x0 = x[0]; r.x1 = x[1]; r.x2 = x[2]; r.x3 = x[3]; r.x4 = x[4]; r.x5 = x[5];
        glibc::sincos(r.x2, r.s2, r.c2);
        r.cwp = glibc::cos(r.x2);
        r.swp = glibc::sin(r.x2);
        const double dla = update_waypoint(r, q, Px, Py, false);
        const double ym = lateral_error(r, Px, Py);
        const double dc = steer_cmd(r, q, dla, ym);
        const double ac = accel_cmd(r, q, prof_v(r.P, r.wp + 2));
        double* w = o + 4 + 8 * j;
        w[0] = (double)r.wp; w[1] = (double)r.endr; w[2] = Px; w[3] = Py;
        w[4] = ym; w[5] = dc; w[6] = ac; w[7] = r.iE;
      }
    } break;
    case CLRRT_UNIT_OBB: {  // checkObsDistance's vehicle box vs one obstacle (getOBBdist)
      const double* a = in + 11 * (int64_t)i;
      double s2, c2;
      glibc::sincos(a[2], s2, c2);
      Box4 veh;
      veh_box(a[0] + 1.424 * c2, a[1] + 1.424 * s2, a[2], veh);
      out[i] = (double)obs_sat_baked(veh, obs[i], a[3]);
    } break;
    case CLRRT_UNIT_ODE: {  // VehicleODE + IntegrateEuler
      const double* a = in + 9 * (int64_t)i;
      Roll r;
      r.x0 = a[0]; r.x1 = a[1]; r.x2 = a[2]; r.x3 = a[3]; r.x4 = a[4]; r.x5 = a[5]; r.x6 = a[6];
      r.cwp = glibc::cos(r.x2);
      r.swp = glibc::sin(r.x2);
      r.t3 = glibc::tan(r.x3);
      const double d2 = ode_euler(r, p, a[7], a[8]);
      double* o = out + 8 * (int64_t)i;
      o[0] = r.x0; o[1] = r.x1; o[2] = r.x2; o[3] = r.x3; o[4] = r.x4; o[5] = r.x5; o[6] = r.x6; o[7] = d2;
    } break;
    case CLRRT_UNIT_LATERAL: {  // transformToVehicle + interpolate
      const double* a = in + 9 * (int64_t)i;
      double s, c;
      glibc::sincos(a[8], s, c);
      out[i] = transform_interp(a, a + 3, a[6], a[7], c, s);
    } break;
    case CLRRT_UNIT_PROFILE: {  // getReference's line + generateVelocityProfile
      const double* a = in + 12 * (int64_t)i;
      DevParams q = p;
      q.ref_res = a[4]; q.vmax = a[6];
      q.g0 = a[7]; q.g1 = a[8]; q.g2 = a[9]; q.g3 = a[10];
      RefD R = make_ref(a[0], a[1], a[2], a[3], q);
      double* row = out + (int64_t)(1 + 3 * CLRRT_UNIT_PROFILE_NMAX) * i;
      row[0] = (double)R.N;
      double x = R.a1x, y = R.a1y;
      for (int j = 0; j < R.N; j++) {
        if (j < CLRRT_UNIT_PROFILE_NMAX) {
          row[1 + CLRRT_UNIT_PROFILE_NMAX + j] = x;
          row[1 + 2 * CLRRT_UNIT_PROFILE_NMAX + j] = y;
        }
        if (j == R.N - 1) { R.bx = x; R.by = y; }
        ref_next(R, j, x, y);
      }
      const Prof P = make_profile(R, a[5], q, a[11] != 0.0);
      for (int j = 0; j < R.N && j < CLRRT_UNIT_PROFILE_NMAX; j++) row[1 + j] = prof_v(P, j);
    } break;
    case CLRRT_UNIT_ANGLE: {  // angleDiff, wrapToPi
      const double* a = in + 2 * (int64_t)i;
      out[2 * (int64_t)i] = angle_diff(a[0], a[1]);
      out[2 * (int64_t)i + 1] = wrap_pi(a[0]);
    } break;
    default: break;
  }
}

// checkObsDistance(x) (collision.h:41; stub collisioncheck.cpp:6-8 or the OBB form
// old_collisioncheck.cpp:24-51 under CLRRT_COLLISION_OBB) for n states of 10 doubles: the documented
// collision hook, evaluated by the rollout kernels' own collision code (every obstacle, gap value kept).
__global__ void k_obs_distance(DevParams p, const BakedObs* __restrict__ obs, const double* __restrict__ st, int n,
                               double* __restrict__ out) {
  glibc::stage_tables();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ObsView ov{obs, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                   p.coll_mode == CLRRT_COLLISION_OBB ? p.n_obs : 0, 0, 0, 0, 0.f, 0.f, 0.f};
  const double* x = st + 10 * (int64_t)i;
  Roll r;
  r.x0 = x[0]; r.x1 = x[1]; r.x2 = x[2]; r.x6 = x[6];
  glibc::sincos(r.x2, r.s2, r.c2);
  uint32_t tests = 0;
  out[i] = obs_distance<true>(r, p, ov, tests);
}

// ============================================================================================
// launch wrappers (host)
// ============================================================================================
#define LAUNCH_CHECK()                                   \
  do {                                                   \
    hipError_t e__ = hipGetLastError();                  \
    if (e__ != hipSuccess) return e__;                   \
  } while (0)

static hipError_t launch_nn_brute(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                  const DevParams& p, const NnFrame& fr, float* pk, int* pi, int* cand,
                                  float* ckey, int* ncand, int* ctie, int max_chunks, const float* seed = nullptr,
                                  unsigned long long* tstat = nullptr);

hipError_t launch_nn(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                     const DevParams& p, float* pk, int* pi, int* cand, float* ckey, int* ncand, int* ctie,
                     int max_chunks, KeyId* exact_scratch, float* seed, unsigned long long* stats, const NnFrame& fr) {
  {
    // shared per-sample key caps start at +inf (order-preserving encoding of +inf = 0xff800000)
    hipError_t e = seed ? hipMemsetD32Async((hipDeviceptr_t)seed, 0xff800000u, B, st) : hipSuccess;
    if (e != hipSuccess) return e;
    e = launch_nn_brute(st, S, B, nodes, N, p, fr, pk, pi, cand, ckey, ncand, ctie, max_chunks, seed,
                        stats ? stats + 5 : nullptr);
    if (e != hipSuccess) return e;
  }
  if (exact_scratch) return launch_nn_exact_any(st, S, B, nodes, N, p, ctie, exact_scratch, cand, ckey, ncand);
  return hipSuccess;
}

hipError_t launch_nn_exact_small(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                 const DevParams& p, int* cand, float* ckey, int* ncand, int* ctie) {
  if (N > NN_EXACT_LDS_MAX || B <= 0) return hipErrorInvalidValue;
  const size_t lds = sizeof(KeyId) * (size_t)N + sizeof(int2) * (size_t)(N / 2 + 64);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)&k_nn_exact_fused, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_nn_exact_fused, dim3(B), dim3(64), lds, st, S, B, nodes, N, p, cand, ckey, ncand, ctie);
  return hipGetLastError();
}

int nn_exact_small_max() { return NN_EXACT_LDS_MAX; }

// The round's new nodes in commit order (sample k's regular node, then its goal-biased one) as the tree's
// nearest-node records will hold them (ids base, base + 1, ...).  One lane: a round has a few dozen samples.
__global__ void k_build_xrec(const clrrt_node* __restrict__ reg, const clrrt_node* __restrict__ gbn,
                             const SampleOut* __restrict__ so, int n, int64_t base, NnRec* __restrict__ xrec) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t pos = 0;
  for (int k = 0; k < n; k++) {
    if (so[k].k < 0) continue;
    xrec[pos] = nn_record(reg[k], base + pos);
    pos++;
    if (so[k].gb_ok) {
      xrec[pos] = nn_record(gbn[k], base + pos);
      pos++;
    }
  }
}

hipError_t launch_nn_exact_x(hipStream_t st, const clrrt_sample* S, const NnRec* nodes, int N, const DevParams& p,
                             const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, int n, NnRec* xrec,
                             const int* slist, const int* xcnt, int nlist, int xmax, int* cand, float* ckey,
                             int* ncand, int* ctie) {
  if (nlist <= 0) return hipSuccess;
  const int Nl = N + xmax;
  if (Nl > NN_EXACT_LDS_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_build_xrec, dim3(1), dim3(64), 0, st, reg, gbn, so, n, (int64_t)N, xrec);
  LAUNCH_CHECK();
  const size_t lds = sizeof(KeyId) * (size_t)Nl + sizeof(int2) * (size_t)(Nl / 2 + 64);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)&k_nn_exact_fused, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_nn_exact_fused, dim3(nlist), dim3(64), lds, st, S, nlist, nodes, N, p, cand, ckey, ncand, ctie,
                     (const NnRec*)xrec, xcnt, slist, Nl);
  return hipGetLastError();
}

hipError_t launch_nn_delta(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int first, int count,
                           const DevParams& p, const NnFrame& fr, float* pk, int* pi, int max_chunks, int* cand,
                           float* ckey, int* ncand, int* ctie, float* seed) {
  if (count <= 0 || B <= 0) return hipSuccess;
  // (the seed / merge kernels and the index build run one-wave blocks: they run beside the lag-2 walk, whose
  // waves fill the CUs and free one slot at a time; priorities order dispatch but do not preempt)
  const int groups = (B + CLRRT_PATH_BLK - 1) / CLRRT_PATH_BLK;
  int nchunks = (count + 255) / 256;
  const int want = max(1, 2048 / max(1, groups));
  nchunks = max(1, min(nchunks, min(want, max_chunks)));
  int chunk = (count + nchunks - 1) / nchunks;
  chunk = (chunk + 255) & ~255;
  nchunks = (count + chunk - 1) / chunk;
  hipLaunchKernelGGL(k_nn_delta_seed, dim3((B + 63) / 64), dim3(64), 0, st, B, p.sort_limit, ckey, ncand, seed);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_nn_partial, dim3(groups, nchunks), dim3(CLRRT_PATH_BLK), 0, st, S, B, nodes + first, count, chunk,
                     nchunks, p, fr, pk, pi, seed, nullptr, nullptr);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_nn_merge_delta, dim3((B + 63) / 64), dim3(64), 0, st, B, nchunks, p.sort_limit, pk, pi,
                     first, cand, ckey, ncand, ctie);
  LAUNCH_CHECK();
  return hipSuccess;
}

// The appended-node search in two halves, for callers that split it (expand_lag2 with nn_split_delta): the partial
// lists of samples S over nodes [first, first + count) -- the chunks' shared key caps in gcap seeded from the samples'
// older list (ckey / ncand, the walk's: no node above its sort_limit-th key can enter; +inf without one, which costs
// ~4x: k_nn_partial 4.9 vs 1.15 ms per cfg3 launch, profiles/r06l_*) -- and the merge of such partial lists (ids
// relative to id0) into a list.  seeded: gcap already holds caps (no seed kernel).
hipError_t launch_nn_delta_partial(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int first,
                                   int count, const DevParams& p, const NnFrame& fr, float* pk, int* pi, int max_chunks,
                                   const float* ckey, const int* ncand, float* gcap, bool seeded, int* order,
                                   int* nchunks_out) {
  *nchunks_out = 0;
  if (count <= 0 || B <= 0) return hipSuccess;
  const int* sord = nullptr;
  if (order) {  // optimize samples on their own lanes (one 1024-thread block: a stable partition of the batch)
    hipLaunchKernelGGL(k_nn_order, dim3(1), dim3(1024), 0, st, S, B, order);
    LAUNCH_CHECK();
    sord = order;
  }
  const int groups = (B + CLRRT_PATH_BLK - 1) / CLRRT_PATH_BLK;
  int nchunks = (count + 255) / 256;
  const int want = max(1, 2048 / max(1, groups));
  nchunks = max(1, min(nchunks, min(want, max_chunks)));
  int chunk = (count + nchunks - 1) / nchunks;
  chunk = (chunk + 255) & ~255;
  nchunks = (count + chunk - 1) / chunk;
  if (!seeded) {  // (seeded: the caller's caps, e.g. k_walk_seed's)
    hipLaunchKernelGGL(k_nn_delta_seed, dim3((B + 63) / 64), dim3(64), 0, st, B, ckey ? p.sort_limit : 0, ckey, ncand,
                       gcap);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_nn_partial, dim3(groups, nchunks), dim3(CLRRT_PATH_BLK), 0, st, S, B, nodes + first, count, chunk,
                     nchunks, p, fr, pk, pi, gcap, nullptr, sord);
  LAUNCH_CHECK();
  *nchunks_out = nchunks;
  return hipSuccess;
}
hipError_t launch_nn_delta_merge(hipStream_t st, int B, int nchunks, const DevParams& p, const float* pk, const int* pi,
                                 int id0, int* cand, float* ckey, int* ncand, int* ctie) {
  if (nchunks <= 0 || B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nn_merge_delta, dim3((B + 63) / 64), dim3(64), 0, st, B, nchunks, p.sort_limit, pk, pi, id0, cand,
                     ckey, ncand, ctie);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_nn_exact_only(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                const DevParams& p, const int* ctie, KeyId* scratch, int* cand, float* ckey,
                                int* ncand) {
  return launch_nn_exact_any(st, S, B, nodes, N, p, ctie, scratch, cand, ckey, ncand);
}

static hipError_t launch_nn_brute(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                  const DevParams& p, const NnFrame& fr, float* pk, int* pi, int* cand,
                                  float* ckey, int* ncand, int* ctie, int max_chunks, const float* seed,
                                  unsigned long long* tstat) {
  int threads = 256;
  int groups = (B + 255) / 256;
  int nchunks = (N + 255) / 256;
  int want = max(1, 2048 / max(1, groups));  // aim for >= 2048 blocks of 4 waves
  nchunks = max(1, min(nchunks, min(want, max_chunks)));

  int chunk = (N + nchunks - 1) / nchunks;
  chunk = (chunk + 255) & ~255;  // tiles of 256 nodes never straddle chunks
  nchunks = (N + chunk - 1) / chunk;
  hipLaunchKernelGGL(k_nn_partial, dim3(groups, nchunks), dim3(threads), 0, st, S, B, nodes, N, chunk, nchunks,
                     p, fr, pk, pi, seed, tstat, nullptr);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_nn_merge, dim3((B + 255) / 256), dim3(256), 0, st, B, nchunks, p.sort_limit, pk, pi,
                     cand, ckey, ncand, ctie);
  LAUNCH_CHECK();
  return hipSuccess;
}

static size_t roll_lds_bytes(const RollArgs& a) {
  size_t lds = 0;
  if (a.p.coll_mode == CLRRT_COLLISION_OBB) {
    lds = (size_t)a.p.n_obs * (6 * sizeof(float4) + sizeof(float));
    if (a.grid.gw > 0)
      lds += sizeof(uint32_t) * ((size_t)a.grid.gw * a.grid.gh + 1) +
             sizeof(uint16_t) * ((size_t)a.grid.nitems + a.grid.nmov);
  }
  return lds;
}

template <int SRC>
static hipError_t launch_roll_t(hipStream_t st, const RollArgs& a) {
  if (a.njobs <= 0) return hipSuccess;
  const size_t lds = roll_lds_bytes(a);
  const int64_t threads = (int64_t)a.njobs * (a.job_stride > 1 ? a.job_stride : 1);
  dim3 grid((unsigned)((threads + 255) / 256)), block(256);
  if (a.p.need_gap)
    hipLaunchKernelGGL((k_rollout<SRC, true>), grid, block, 0, st, a);
  else
  {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)&k_rollout<SRC, false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_rollout<SRC, false>), grid, block, lds, st, a);
  }
  LAUNCH_CHECK();
  return hipSuccess;
}

// The queue order from k_roll_flag's flags: perm = flagged positions, then the others (both ascending).
// a.pflag's buffer holds [njobs flags][njobs exclusive-scan positions][scan scratch].
size_t roll_order_scratch_bytes(int n) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int*)nullptr, (int*)nullptr, n);
  return bytes;
}
static hipError_t roll_order(hipStream_t st, const RollArgs& a) {
  if (!a.perm || !a.pflag) return hipSuccess;
  int* ppos = a.pflag + a.njobs;
  void* tmp = (void*)(((uintptr_t)(a.pflag + 2 * (size_t)a.njobs) + 255) & ~(uintptr_t)255);  // 256 B spare
  size_t bytes = roll_order_scratch_bytes(a.njobs);
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, bytes, a.pflag, ppos, a.njobs, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_roll_order, dim3((a.njobs + 63) / 64), dim3(64), 0, st, a.pflag, ppos, a.njobs, a.perm);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_fill_ints(FillInts f) {
  const int stride = gridDim.x * blockDim.x;
  for (int q = 0; q < f.nj; q++)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < f.n[q]; i += stride) f.p[q][i] = f.v[q];
}
hipError_t launch_fill_ints(hipStream_t st, const FillInts& f) {
  if (f.nj <= 0) return hipSuccess;
  int mx = 0;
  for (int q = 0; q < f.nj; q++) mx = f.n[q] > mx ? f.n[q] : mx;
  const int blocks = (mx + 255) / 256 < 64 ? (mx + 255) / 256 : 64;
  hipLaunchKernelGGL(k_fill_ints, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, f);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_rollout_persistent(hipStream_t st, const RollArgs& a0, int B, int* qnext, int* best, int blocks,
                                     bool prefilled) {
  hipError_t e;
  if (!prefilled && a0.ncarry_out && (e = hipMemsetAsync(a0.ncarry_out, 0, sizeof(int), st)) != hipSuccess) return e;
  if (a0.njobs <= 0 && a0.nrep <= 0 && a0.ncarry <= 0) return hipSuccess;
  if (!prefilled) {
    if ((e = hipMemsetAsync(qnext, 0, sizeof(int), st)) != hipSuccess) return e;
    if (B > 0 && (e = hipMemsetAsync(best + a0.sbase, 0x7f, sizeof(int) * B, st)) != hipSuccess) return e;
  }
  RollArgs a = a0;
  a.B = B;
  // dynamic LDS of k_roll_run: the obstacle tables (not with NEED_GAP), then (COOP) the cooperative
  // collision check's per-wave scratch, when the static grid is built and the whole fits the 160 KB a
  // workgroup may use beside the glibc tables' static LDS (~12 KB)
  const size_t obs_lds = a.p.need_gap ? 0 : (roll_lds_bytes(a0) + 15) / 16 * 16;
  const bool coop = a.coop_enable && !a.p.need_gap && a.p.coll_mode == CLRRT_COLLISION_OBB && a.p.n_obs > 0 && a.grid.gw > 0 &&
                    obs_lds + 4 * kCoopLdsPerWave <= 148 * 1024;
  a.coop_off = (int)obs_lds;
  const size_t lds = obs_lds + (coop ? 4 * kCoopLdsPerWave : 0);
  const bool carry = a.cap > 0 || a.ncarry > 0;  // deferred samples: the CARRY instantiation
  const void* fn = a.p.need_gap ? (carry ? (const void*)&k_roll_run<true, false, true> : (const void*)&k_roll_run<true, false, false>)
                   : coop       ? (carry ? (const void*)&k_roll_run<false, true, true> : (const void*)&k_roll_run<false, true, false>)
                                : (carry ? (const void*)&k_roll_run<false, false, true> : (const void*)&k_roll_run<false, false, false>);
  if (lds > 64 * 1024 && (e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess)
    return e;
  const int nqueue = a0.njobs + a0.nrep + a0.ncarry;
  // a queue shorter than the grid's lanes is spread over its waves (lanes per wave = ceil(queue / waves))
  int lpw = a0.lanes_per_wave > 0 && a0.lanes_per_wave < 64 ? a0.lanes_per_wave : 64;
  if (a0.lanes_per_wave <= 0) {
    const int waves = 4 * blocks;
    lpw = (nqueue + waves - 1) / waves;
    lpw = lpw < 1 ? 1 : (lpw > 64 ? 64 : lpw);
  }
  a.lanes_per_wave = lpw;
  const int nb = blocks < (nqueue + 4 * lpw - 1) / (4 * lpw) ? blocks : (nqueue + 4 * lpw - 1) / (4 * lpw);
  if (a.njobs > 0 && a.perm && a.pflag) {  // queue order: the likely-long jobs first
    hipLaunchKernelGGL(k_roll_flag, dim3((a.njobs + 63) / 64), dim3(64), 0, st, a);
    LAUNCH_CHECK();
    if ((e = roll_order(st, a)) != hipSuccess) return e;
  } else {
    a.perm = nullptr;
  }
  if (carry) {
    if (a.p.need_gap)
      hipLaunchKernelGGL((k_roll_run<true, false, true>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
    else if (coop)
      hipLaunchKernelGGL((k_roll_run<false, true, true>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
    else
      hipLaunchKernelGGL((k_roll_run<false, false, true>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
  } else if (a.p.need_gap) {
    hipLaunchKernelGGL((k_roll_run<true, false, false>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
  } else if (coop) {
    hipLaunchKernelGGL((k_roll_run<false, true, false>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
  } else {
    hipLaunchKernelGGL((k_roll_run<false, false, false>), dim3(nb), dim3(256), lds, st, a, qnext, best, B);
  }
  LAUNCH_CHECK();
  return hipSuccess;
}


hipError_t launch_rollout(hipStream_t st, int src, const RollArgs& a) {
  if (src == SRC_SPEC) return launch_roll_t<SRC_SPEC>(st, a);
  if (src == SRC_EXPL) return launch_roll_t<SRC_EXPL>(st, a);
  return launch_roll_t<SRC_LIST>(st, a);
}

hipError_t launch_select(hipStream_t st, const SelArgs& a) {
  hipLaunchKernelGGL(k_select, dim3((a.B + CLRRT_SEL_BLK - 1) / CLRRT_SEL_BLK), dim3(CLRRT_SEL_BLK), 0, st, a);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_copy_rows(hipStream_t st, const Job* jobs, const clrrt_node* recs, int n, const double* slots,
                            int slot_rows, int slot_jobs, double* arena) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_rows, dim3(n), dim3(256), 0, st, jobs, recs, slots, slot_rows, slot_jobs, arena);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_conflict_fix(hipStream_t st, const DevParams& p, int B, const clrrt_sample* S,
                               const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, const int* ctie,
                               const int* ncand, const float* ckey, const RollRes* res, int* fix_n, int* fix_ids,
                               int* fix_adj) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conflict_fix, dim3((B + 63) / 64), dim3(64), 0, st, p, B, S, reg, gbn, so, ctie, ncand, ckey,
                     res, fix_n, fix_ids, fix_adj);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_conflict(hipStream_t st, const DevParams& p, int B, const clrrt_sample* S,
                           const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, const int* ctie,
                           int* first) {
  hipLaunchKernelGGL(k_conflict, dim3((B + 63) / 64), dim3(64), 0, st, p, B, S, reg, gbn, so, ctie, first);
  LAUNCH_CHECK();
  return hipSuccess;
}

// Deferred samples: the ring indices gv[v] of the views still pending after a commit, in view order (the
// oldest round first, then this round's in sample order), into out[0 .. *n_out) -- the next commit's views.
size_t defer_select_bytes(int n) {
  size_t bytes = 0;
  hipcub::DeviceSelect::Flagged(nullptr, bytes, (const int*)nullptr, (const uint8_t*)nullptr, (int*)nullptr,
                                (int*)nullptr, n);
  return bytes;
}
hipError_t launch_defer_select(hipStream_t st, const int* gv, const uint8_t* pend, int n, int* out, int* n_out,
                               void* tmp, size_t tmp_bytes) {
  if (n <= 0) return hipMemsetAsync(n_out, 0, sizeof(int), st);
  size_t bytes = tmp_bytes;
  return hipcub::DeviceSelect::Flagged(tmp, bytes, gv, pend, out, n_out, n, st);
}

size_t compact_scan_bytes(int n) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, n);
  return bytes;
}

// Sharded rounds (clrrt_set_shards) with deferred samples: the exchanged union of every rank's records (each
// rank's in (age desc, sample) order, ranks holding contiguous slices) into the global commit order, the
// oldest round first, by a stable sort on the age tag; the tag is cleared.  The appended records' goal
// flags are counted into *goal.
__global__ void k_xorder_keys(const clrrt_node* __restrict__ recs, int n, uint32_t* __restrict__ keys,
                              uint32_t* __restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = 255u - (((uint32_t)recs[i].goal >> 8) & 0xffu);
  idx[i] = (uint32_t)i;
}
__global__ void k_xgather(const clrrt_node* __restrict__ recs, const uint32_t* __restrict__ idx, int n,
                          clrrt_node* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  clrrt_node r = recs[idx ? idx[i] : i];
  r.goal &= 0xff;
  out[i] = r;
}
__global__ void k_goal_count(const clrrt_node* __restrict__ recs, int n, unsigned long long* goal) {
  unsigned long long c = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) c += recs[i].goal & 1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(goal, c);
}
size_t xorder_sort_bytes(int n) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, 8);
  return bytes;
}
hipError_t launch_xorder(hipStream_t st, const clrrt_node* recs, int n, bool sort, uint32_t* keys, void* tmp,
                         size_t tmp_bytes, clrrt_node* out, unsigned long long* goal) {
  if (n <= 0) return hipSuccess;
  const unsigned g = (unsigned)((n + 255) / 256);
  uint32_t* idx = nullptr;
  if (sort) {
    hipLaunchKernelGGL(k_xorder_keys, dim3(g), dim3(256), 0, st, recs, n, keys, keys + n);
    LAUNCH_CHECK();
    size_t bytes = tmp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, keys, keys + 2 * n, keys + n, keys + 3 * n, n, 0, 8, st);
    if (e != hipSuccess) return e;
    idx = keys + 3 * n;
  }
  hipLaunchKernelGGL(k_xgather, dim3(g), dim3(256), 0, st, recs, idx, n, out);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_goal_count, dim3(g < 1024 ? g : 1024), dim3(256), 0, st, out, n, goal);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_compact(hipStream_t st, int L, const clrrt_sample* S, const int* cand, const clrrt_node* reg,
                          const clrrt_node* gbn, const SampleOut* so, int64_t row_base, int rank,
                          clrrt_node* out, Job* jobs, int64_t* totals, CompactBufs& cb, int tag_slot, int tag_R,
                          int tag_B, bool totals_zeroed) {
  hipError_t e = totals_zeroed ? hipSuccess : hipMemsetAsync(totals, 0, sizeof(int64_t) * 8, st);
  if (e != hipSuccess) return e;
  if (L <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compact_count, dim3((L + 255) / 256), dim3(256), 0, st, L, so, reg, gbn, cb.packed, totals);
  LAUNCH_CHECK();
  size_t bytes = cb.tmp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(cb.tmp, bytes, cb.packed, cb.scanned, L, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_compact_scatter, dim3((L + 255) / 256), dim3(256), 0, st, L, so, reg, gbn, cb.packed, cb.scanned,
                     row_base, rank, out, jobs, totals, tag_slot, tag_R, tag_B);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bbox(hipStream_t st, const clrrt_node* recs, const int64_t* n_dev, int n_host, double* out4) {
  hipLaunchKernelGGL(k_bbox, dim3(1), dim3(256), 0, st, recs, n_dev, n_host, out4);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_append(hipStream_t st, const clrrt_node* in, int n, int64_t base, clrrt_node* tree, NnRec* nn) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_append, dim3((n + 255) / 256), dim3(256), 0, st, in, n, base, tree, nn);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_selftest_math(hipStream_t st, int fn, const double* a, const double* b, int n, double* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, st, fn, a, b, n, out);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_selftest_units(hipStream_t st, int unit, const double* in, const BakedObs* obs, int n,
                                 const DevParams& p, const DevParams* cp, double* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_units, dim3((n + 255) / 256), dim3(256), 0, st, unit, in, obs, n, p, cp, out);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_obs_distance(hipStream_t st, const DevParams& p, const BakedObs* obs, const double* states, int n,
                               double* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_obs_distance, dim3((n + 255) / 256), dim3(256), 0, st, p, obs, states, n, out);
  LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_goal_gather(hipStream_t st, const clrrt_node* tree, int64_t n, GoalRec* out, int* cnt) {
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int), st);
  if (e != hipSuccess || n == 0) return e;
  const int64_t want = (n + 255) / 256;
  const int blocks = (int)std::min<int64_t>(want, 4096);
  hipLaunchKernelGGL(k_goal_gather, dim3(blocks), dim3(256), 0, st, tree, n, out, cnt);
  return hipGetLastError();
}

hipError_t launch_backtrack(hipStream_t st, const clrrt_node* tree, int64_t n, int start, int cap, int* path,
                            int* len) {
  hipLaunchKernelGGL(k_backtrack, dim3(1), dim3(64), 0, st, tree, n, start, cap, path, len);
  return hipGetLastError();
}

hipError_t launch_gather_nodes(hipStream_t st, const clrrt_node* tree, const int* ids, int n, clrrt_node* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_nodes, dim3((n + 255) / 256), dim3(256), 0, st, tree, ids, n, out);
  return hipGetLastError();
}

hipError_t launch_path_transform(hipStream_t st, clrrt_node* nodes, int n, double* rows, int64_t nrows, int to_world,
                                 const double pose[3]) {
  const int64_t total = (int64_t)n + nrows;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_path_transform, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, nodes, n, rows,
                     nrows, to_world, pose[0], pose[1], pose[2]);
  return hipGetLastError();
}

hipError_t launch_tree_reinit(hipStream_t st, const ReinitArgs& a) {
  hipLaunchKernelGGL(k_tree_reinit, dim3(1), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_init_root(hipStream_t st, const double* state, clrrt_node* tree, NnRec* nn, double* arena) {
  hipLaunchKernelGGL(k_init_root, dim3(1), dim3(64), 0, st, state, tree, nn, arena);
  LAUNCH_CHECK();
  return hipSuccess;
}

}  // namespace clrrt
