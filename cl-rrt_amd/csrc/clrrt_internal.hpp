// clrrt_internal.hpp — records shared between the kernels and the host orchestration of libclrrt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clrrt.h"
#include "clrrt_dev.hpp"
#include "clrrt_stdsort.hpp"

namespace clrrt {

// Result of one rollout (what Simulation exposes after propagate).
struct RollRes {
  double st[10];       // stateArray.back()
  double costE, costS; // Simulation::costE / costS
  double bx, by;       // ref.x/y.back()
  double fx, fy;       // ref.x/y.front()
  double vback;        // ref.v.back()
  int32_t outcome;     // CLRRT_ROLL_*, -1 = no job
  int32_t nrows;       // stateArray.size()
  int32_t refN;
  int32_t pad;
};

// Algorithmic work of rollouts (SURVEY §8(d) roofline basis): simulated steps, reference points
// scanned by findClosestPoint, OBB box tests.
struct WorkCtr {
  uint32_t steps, scan, box;
};

// Explicit rollout job (parity entry, row replay).
struct Job {
  int32_t parent;   // tree node id, or sample index into the regular-node buffer when from_reg
  int32_t from_reg;
  int32_t gb;
  int32_t pad;
  double sx, sy;
  int64_t row_off;  // >= 0: write stateArray rows at arena[row_off*10 ...]
};

// Per-sample outcome of one expandTree iteration.
struct SampleOut {
  float thr;        // EXACT-mode conflict threshold
  int32_t k;        // accepted candidate index, -1 = none
  int32_t gb_ok;    // goal-biased node accepted
  int32_t nrows_reg, nrows_gb;
  int32_t rollouts, steps, f_col, f_acc, f_it;
};

// Job sources:
//   SRC_SPEC : job j -> (sample s = j / K, candidate k = j % K), parent = tree node cand[s][k]
//   SRC_GB   : job s -> goal-biased rollout from the regular node built for sample s (gbflag[s])
//   SRC_LIST : explicit Job records (parity entry and row replay), parent = tree node or record
enum { SRC_SPEC = 0, SRC_GB = 1, SRC_LIST = 2 };

struct RollArgs {
  DevParams p;
  const clrrt_node* __restrict__ tree;     // tree headers
  const clrrt_sample* __restrict__ samples;
  const int* __restrict__ cand;            // [B][K]
  const clrrt_node* __restrict__ regnodes; // [B] regular nodes built by k_select
  const int* __restrict__ gbflag;          // [B]
  const Job* __restrict__ jobs;
  const BakedObs* __restrict__ obs;
  double* __restrict__ arena;              // rows destination (LIST with row_off >= 0)
  RollRes* __restrict__ res;
  unsigned long long* ctr;  // [3] steps, scan points, box tests (nullable)
  int njobs;
};

struct SelArgs {
  DevParams p;
  const clrrt_node* __restrict__ tree;
  const int* __restrict__ cand;
  const float* __restrict__ ckey;
  const int* __restrict__ ncand;
  const RollRes* __restrict__ res;   // [B][K]
  clrrt_node* regnodes;              // [B]
  int* gbflag;                       // [B]
  SampleOut* so;                     // [B]
  int B;
};

// Nearest-node search.  exact_scratch != nullptr (EXACT mode, B*N KeyId entries): samples whose
// selection involves equal keys are re-sorted with the replay of std::sort.
hipError_t launch_nn(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                     const DevParams& p, float* pk, int* pi, int* cand, float* ckey, int* ncand, int* ctie,
                     int max_chunks, KeyId* exact_scratch);
hipError_t launch_rollout(hipStream_t st, int src, const RollArgs& a);
hipError_t launch_select(hipStream_t st, const SelArgs& a);
hipError_t launch_gb_select(hipStream_t st, int B, const clrrt_node* reg, const int* gbflag,
                            const RollRes* gbres, clrrt_node* gbnodes, SampleOut* so);
hipError_t launch_conflict(hipStream_t st, const DevParams& p, int B, const clrrt_sample* S,
                           const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, const int* ctie,
                           int* first);
hipError_t launch_compact(hipStream_t st, int L, const clrrt_sample* S, const int* cand, const clrrt_node* reg,
                          const clrrt_node* gbn, const SampleOut* so, int64_t row_base, int rank,
                          clrrt_node* out, Job* jobs, int64_t* totals);
hipError_t launch_append(hipStream_t st, const clrrt_node* in, int n, int64_t base, clrrt_node* tree, NnRec* nn);
hipError_t launch_selftest_math(hipStream_t st, int fn, const double* a, const double* b, int n, double* out);
hipError_t launch_init_root(hipStream_t st, const double* state, clrrt_node* tree, NnRec* nn, double* arena);

}  // namespace clrrt
