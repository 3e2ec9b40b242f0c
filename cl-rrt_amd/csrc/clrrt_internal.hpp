// clrrt_internal.hpp — records shared between the kernels and the host orchestration of libclrrt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clrrt.h"
#include "clrrt_dev.hpp"
#include "clrrt_stdsort.hpp"

namespace clrrt {

// RollRes::outcome of a rollout suspended at its chain's cap (deferred samples): not known yet.
#define CLRRT_ROLL_PENDING (-2)

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

// A parent state passed by value so that it stays in registers.
struct St10 {
  double v[10];
};

// Explicit rollout job (parity entry) or row-copy job (commit: parent = slot job, gb = pass).
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
  int32_t g;        // ring index of the sample (job of candidate k: g K + k)
  int32_t pend;     // 1: a rollout the result depends on is still suspended (deferred sample)
};

// Job sources:
//   SRC_SPEC : job j -> (sample s = j / K, candidate k = j % K), parent = tree node cand[s][k];
//              a successful regular rollout is followed in the same lane by the goal-biased one
//   SRC_LIST : explicit Job records (parity entry), parent = tree node
//   SRC_EXPL : explicit SimJob records (clrrt_simulate): parent state, reference generator and Vstart
//              given directly; rows to arena[row_off], the reference (x, y, v) to refv[ref_off]
enum { SRC_SPEC = 0, SRC_LIST = 2, SRC_EXPL = 3 };

// Simulation::Simulation for an explicit state and reference (clrrt_simulate): gb = 0: the n points
// a + i h (accumulated, getReference's LinearSpacedVector); gb = 1: getGoalReference from a.
struct SimJob {
  double st[10];
  double ax, ay, hx, hy, vstart;
  int32_t n, gb;
  int64_t row_off;  // >= 0: stateArray rows at arena[row_off * 10 ...]
  int64_t ref_off;  // >= 0: x[ref_cap], y[ref_cap], v[ref_cap] at refv[ref_off ...]
};

// Uniform grid over the static obstacles (built on the host by clrrt_set_obstacles): cell
// (gx, gy) lists, ascending, every static obstacle whose inflated bounding circle (radius + vehicle
// radius + margin, the kernel's cull test) comes within a small tolerance of the cell.
struct ObsGrid {
  const uint32_t* start;  // [gw*gh + 1]
  const uint16_t* items;
  const uint16_t* mov;    // moving obstacles (tested at every step)
  int gw, gh, nitems, nmov;
  float x0, y0, inv;
};

struct RollArgs {
  DevParams p;
  ObsGrid grid;
  const clrrt_node* __restrict__ tree;     // tree headers
  const clrrt_sample* __restrict__ samples;
  const int* __restrict__ cand;            // [B][K]
  const Job* __restrict__ jobs;
  const SimJob* __restrict__ sims;         // SRC_EXPL
  double* __restrict__ refv;               // SRC_EXPL: generated references
  int ref_cap;
  const BakedObs* __restrict__ obs;
  double* __restrict__ arena;              // rows destination (LIST with row_off >= 0)
  double* __restrict__ slots;              // SPEC rows, see k_rollout (job-major, rows contiguous)
  int slot_rows, slot_jobs;
  RollRes* __restrict__ res;               // regular rollout of each job
  RollRes* __restrict__ res_gb;            // SPEC: goal-biased rollout (outcome -1 = not run)
  unsigned long long* ctr;  // [3] steps, scan points, box tests (nullable)
  int njobs;
  // persistent rollouts: queue order (nullable).  k_roll_flag flags the jobs likely to run long
  // (pflag[q], q = k B + s), the queue serves them first (perm[position] = q); results do not depend
  // on the order
  int* perm;
  int* pflag;
  int B;
  int coop_off;     // k_roll_run's cooperative collision scratch: byte offset in the dynamic LDS
  int coop_enable;  // option "roll_coop": use it where it applies (launch_rollout_persistent)
  // k_roll_run: replays of committed rollouts (deferred rows, see Replay in clrrt_kernels.hip), served
  // before the round's jobs; slots == nullptr: the speculative rollouts store no rows
  const void* rep;
  int nrep;
  // k_roll_run lanes per wave that take jobs: <= 0 spreads the queue over the grid's waves (set by
  // launch_rollout_persistent), 64 fills every lane (option "roll_spread" 0)
  int lanes_per_wave;
  // Deferred samples (BATCH option "defer_steps" = cap > 0, see k_roll_run): a rollout chain (a regular
  // rollout + its goal-biased follow-up) runs at most `cap` more steps per launch; one that reaches its cap
  // is suspended into carry_out (count *ncarry_out) and resumed from carry_in[0 .. ncarry) -- the queue's
  // first positions -- by the next launch.  res / res_gb / best are rings over the rounds in flight: this
  // launch's job j = s K + k writes res[jbase + j] and its sample's first success best[sbase + s].
  int cap;
  const void* carry_in;
  int ncarry;
  void* carry_out;
  int* ncarry_out;
  int carry_cap;
  int jbase, sbase;
  unsigned long long* dbg;  // diagnostics (CLRRT_DEBUG_SYNC): per-wave heartbeat in host-mapped memory, or null
  // SRC_LIST jobs whose parent is a node of the round being committed (Job::from_reg 1: xreg[parent], 2:
  // xgb[parent]; EXACT fix-up rollouts), and the lanes that take jobs (job_stride 64: one job per wave, each at
  // the lone lane's step latency; 0 or 1: every lane)
  const clrrt_node* __restrict__ xreg;
  const clrrt_node* __restrict__ xgb;
  int job_stride;
};

// k_select over B "views": view v < nd is the still unresolved sample view[v] of an earlier round (deferred
// samples), view v >= nd is sample v - nd of this round; a sample is addressed by its ring index g (cand,
// ncand, res, res_gb at g K + k); without deferred samples nd = 0 and sbase = 0 (the round's own arrays).
struct SelArgs {
  DevParams p;
  const clrrt_node* __restrict__ tree;
  const int* __restrict__ cand;
  const float* __restrict__ ckey;
  const int* __restrict__ ncand;
  const RollRes* __restrict__ res;   // [.][K]
  const RollRes* __restrict__ res_gb; // [.][K]
  clrrt_node* regnodes;              // [B]
  clrrt_node* gbnodes;               // [B]
  SampleOut* so;                     // [B]
  int B;
  const int* view;                   // [nd] ring indices of the deferred samples (oldest round first)
  int nd, sbase;
  int* gv;                           // [B] ring index of view v (null: not needed)
  uint8_t* pend;                     // [B] 1 = view v is not resolved yet (null: every sample resolves)
  int* new_pend;                     // counts this round's samples (views >= nd) left pending (null: no count)
};

// Frame of the brute-force search's float prune: positions relative to (ox, oy) in float are within
// delta of the exact differences for every node and sample of the round.
struct NnFrame {
  double ox, oy;
  float delta;
  int debug;  // diagnostics only (results change!): 1 = skip the exact pass
};
// Bounds of a tile (64 place-ordered records) or super-tile (1024) of the walk search
// (clrrt_nnwalk.hip), frame coordinates.
struct WalkTile {
  float pcx, pcy, pr;  // disc holding the node positions (pr < 0: no records)
  float rcx, rcy, rr;  // disc holding the ref.back() points
  float thx, thy, thh; // arc of node headings: unit centre, half width [rad] (>= 3: unbounded)
  float apx, apy, aph; // arc of ang_par directions
  float cemin;         // min costE
  float aopt;          // min (costE - |position - (pcx, pcy)|)
  int32_t nonfinite;   // a record with a non-finite field: no bound
  float eroot;         // min (costE - |position - R|), R = node 0's position (the tree root)
};
static_assert(sizeof(WalkTile) == 64, "WalkTile layout");
struct WalkBufs {
  uint32_t *keys, *keys2;  // [2 max_nodes] 64-bit sort keys (radix sort in/out; samples: 32-bit)
  int *vals, *vals2;       // [max(max_nodes, max_batch)] node ids (vals2 = place order)
  int* sorder;             // [max_batch] samples in place order
  void* tmp;               // radix sort scratch
  size_t tmp_bytes;
  float4 *P, *Q;           // [max_nodes + 1024] (x, y, c, s), (bx, by, ca, sa) relative to the frame origin
  float* CE;               // costE
  int* ID;                 // node id (-1: padding)
  int* HEAD;               // first record of the run of records with equal Dubins-key inputs
  int2* trun;              // per tile: (run head, smallest id) of a tile inside one run, else (-1, -1)
  WalkTile *tiles, *supers;
  // overflow of the walk: a sample whose walk passes the budget (tiles visited / exact keys) hands
  // its search to nch waves over interleaved super-tile subsets with the list's 11th entry as the
  // bound, then a merge wave (k_walk_split / k_walk_merge); budget 0 = off
  int bud_tiles, bud_ex, max_over, nch;
  int half_max = 4096;  // fp16 LDS bounds up to this many super-tiles, coded bytes (+ inside bracket) beyond
  int lds_floor = 0;    // bytes of LDS each walk wave reserves at least (caps the walk's waves per CU)
  int waves = 0;        // > 0: a persistent walk grid of this many waves (samples from per-XCD counters)
  int waves_min_batch = 0;  // ... used for batches of at least this many samples
  // place order of the index (option "nn_walk_index"): 0 = ang_par sector, then the 2D Morton code of the
  // position; 1 = 3D Morton code of (x, y, rho * heading) in one metric scale (the Dubins key is bounded below by
  // max(|q|, rho * beta), so tiles compact in that space prune by heading as well as by distance); 2 = the same
  // with rho * ang_par; 3 / 4 = the ang_par sector first, then kind 1's / 2's code; 5 = kind 3 with records of
  // equal position, heading and cost in ref.back() order (k_walk_keys).  The context's default (clrrt_ctx::nnw_index)
  // is kind 5 since round 6 (2.8 M nodes 10.82 -> 10.35 ms per 16384-sample search, cfg3 +1.6 %,
  // profiles/r06g_nn_large_k*.txt); kind 3 was 0-5% faster than kind 0 at 1.1-16 M nodes (round 5,
  // profiles/r05c_nn_large_index_ab2.txt; kinds 1 / 2 double the tiles per sample, r05a_nn_large_index_ab.txt)
  int index_kind = 0;
  int hscale_pct = 100;  // the 3D codes' heading axis: percent of rho metres per radian (option nn_walk_hscale)
  int* wctr = nullptr;  // [8] the per-XCD sample counters
  int lpt = 0;          // the persistent grid's eighths: optimize samples first (k_walk_lpt, option nn_walk_lpt)
  // set by the caller around one launch_nn_walk_search: [B] key caps for the appended-node search written right after
  // the main grid (k_walk_seed), and an event recorded there (before the overflow split); null: neither
  float* seed_out = nullptr;
  hipEvent_t ev_main = nullptr;
  int* ovf_n;    // [1] overflow records claimed
  int4* ovf;     // [max_over] (sample, kth bits, idk + 1, 0)
  float* pk;     // [max_over * nch * 11] partial lists
  int* pi;
  // the index's sort result, kept for the next build: skeys/sids = the sorted (key, node) pairs of nodes
  // [0, sorted_n) in the frame (sorted_x0, sorted_y0, sorted_scale); sorted_n = -1: none
  uint64_t* skeys;
  int* sids;
  int64_t sorted_n;
  double sorted_x0, sorted_y0, sorted_scale;
  int sorted_kind;
  int64_t cap_nodes;  // the buffers hold an index of up to this many nodes (checked at every launch)
  int cap_batch;      // and searches of up to this many samples
};
size_t walk_sort_bytes(int n);
// Tile / super-tile records an index of up to n nodes needs (WalkBufs::tiles, ::supers).
int64_t walk_tile_count(int64_t n);
int64_t walk_super_count(int64_t n);
// Candidate lists of samples S[0 .. B) (same output as the brute force: cand, ckey, ncand, ctie);
// (x0, y0, x1, y1) = box holding every finite node position (the Morton frame).
hipError_t launch_nn_walk(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N, const DevParams& p,
                          const NnFrame& fr, double x0, double y0, double x1, double y1, WalkBufs& w, int* cand,
                          float* ckey, int* ncand, int* ctie, unsigned long long* stats, bool stateless);
// launch_nn_walk's two halves: the index of nodes [0, N), then the search of samples over it
hipError_t launch_nn_walk_build(hipStream_t st, const NnRec* nodes, int N, const NnFrame& fr, double x0, double y0,
                                double x1, double y1, WalkBufs& w, const WalkBufs* prev = nullptr);
hipError_t launch_nn_walk_search(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                 const DevParams& p, const NnFrame& fr, double x0, double y0, double x1, double y1,
                                 WalkBufs& w, int* cand, float* ckey, int* ncand, int* ctie, unsigned long long* stats,
                                 bool stateless);
// Diagnostics: per sample, the tiles / records any search over the index in w must touch (k_walk_audit)
hipError_t launch_walk_audit(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N, const DevParams& p,
                             const NnFrame& fr, const WalkBufs& w, int* out);
// Pipelined BATCH rounds: merges into (cand, ckey, ncand) -- the lists over nodes [0, first) -- the
// nodes [first, first + count) appended since (k_nn_partial over them + k_nn_merge_delta).
hipError_t launch_nn_delta(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int first, int count,
                           const DevParams& p, const NnFrame& fr, float* pk, int* pi, int max_chunks, int* cand,
                           float* ckey, int* ncand, int* ctie, float* seed);
// launch_nn_delta split in two: the partial lists over the appended nodes (caps shared between chunks from +inf in
// gcap[B], no older list needed; *nchunks_out lists per sample in pk / pi), and their merge into a list.
hipError_t launch_nn_delta_partial(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int first,
                                   int count, const DevParams& p, const NnFrame& fr, float* pk, int* pi, int max_chunks,
                                   const float* ckey, const int* ncand, float* gcap, bool seeded, int* order,
                                   int* nchunks_out);
hipError_t launch_nn_delta_merge(hipStream_t st, int B, int nchunks, const DevParams& p, const float* pk, const int* pi,
                                 int id0, int* cand, float* ckey, int* ncand, int* ctie);
// Nearest-node search.  exact_scratch != nullptr (EXACT mode, B*N KeyId entries): samples whose
// selection involves equal keys are re-sorted with the replay of std::sort.  seed: [B] scratch for the
// chunks' shared key caps (or null).
hipError_t launch_nn(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                     const DevParams& p, float* pk, int* pi, int* cand, float* ckey, int* ncand, int* ctie,
                     int max_chunks, KeyId* exact_scratch, float* seed, unsigned long long* stats, const NnFrame& fr);
// EXACT mode after a search that filled ctie: std::sort replay for the tied samples.
hipError_t launch_nn_exact_only(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                const DevParams& p, const int* ctie, KeyId* scratch, int* cand, float* ckey,
                                int* ncand);
hipError_t launch_rollout(hipStream_t st, int src, const RollArgs& a);
// EXACT-mode lists of a tree of at most nn_exact_small_max() nodes, one wave per sample (k_nn_exact_fused:
// keys, list, tie flag and the std::sort replay of tied samples in one kernel)
hipError_t launch_nn_exact_small(hipStream_t st, const clrrt_sample* S, int B, const NnRec* nodes, int N,
                                 const DevParams& p, int* cand, float* ckey, int* ncand, int* ctie);
int nn_exact_small_max();
// Round rollouts (and the pending replays a.rep[0..nrep)) as the persistent k_roll_run, behind k_roll_flag +
// k_roll_order when a.perm / a.pflag are set (see clrrt_kernels.hip); best B ints, qnext one int.
// prefilled: the round's prologue (launch_fill_ints) already reset *a.ncarry_out, *qnext and best[sbase, sbase + B)
hipError_t launch_rollout_persistent(hipStream_t st, const RollArgs& a, int B, int* qnext, int* best, int blocks,
                                     bool prefilled = false);
// Up to 8 int ranges set to one value each in ONE launch (a round's counter resets, which were one fill each)
struct FillInts {
  int* p[8];
  int n[8];
  int v[8];
  int nj = 0;
  void add(int* ptr, int count, int value) {
    if (ptr && count > 0) { p[nj] = ptr; n[nj] = count; v[nj] = value; nj++; }
  }
};
hipError_t launch_fill_ints(hipStream_t st, const FillInts& f);
size_t roll_order_scratch_bytes(int n);  // k_roll_order's scan scratch for n jobs
size_t replay_bytes();
size_t carry_bytes();  // one suspended rollout (deferred samples)
// deferred rows: the committed rollouts' start states (jobs/recs from launch_compact, prep and res of the
// round's lists / k_roll_run results) into out[0..n) for the next persistent launch's replays
hipError_t launch_replay_gather(hipStream_t st, const Job* jobs, const clrrt_node* recs, int n, const clrrt_node* tree,
                                const int* cand, const clrrt_sample* S, const RollRes* res, void* out);
hipError_t launch_select(hipStream_t st, const SelArgs& a);
hipError_t launch_copy_rows(hipStream_t st, const Job* jobs, const clrrt_node* recs, int n, const double* slots,
                            int slot_rows, int slot_jobs, double* arena);
// EXACT fix-ups (k_conflict_fix): per sample j of the round, the nodes appended earlier in the round that enter
// its candidate list before its result (fix_n[j] = their count m, fix_ids[j * FIX_MAX + i] = 2 k + (0 regular, 1
// goal-biased) of sample k), or -1 when the conflict cannot be resolved by rolling them out (see the kernel)
#define FIX_MAX 4
// EXACT fix-ups of the samples k_conflict_fix could not resolve: their lists over the tree they will see (the N
// tree nodes + the round's new nodes before them, xcnt[i] for sample slist[i]), one wave each (k_nn_exact_fused
// with std::sort's tie order), into rows 0 .. nlist of cand / ckey / ncand / ctie; xrec: [2 n] scratch
hipError_t launch_nn_exact_x(hipStream_t st, const clrrt_sample* S, const NnRec* nodes, int N, const DevParams& p,
                             const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, int n, NnRec* xrec,
                             const int* slist, const int* xcnt, int nlist, int xmax, int* cand, float* ckey,
                             int* ncand, int* ctie);
// fix_adj[j * 5 ..]: counters (rollouts, steps, collisions, acceleration limits, iteration limits) to add for old
// candidates of a sample without a result that the grown window pushes out (<= 0)
hipError_t launch_conflict_fix(hipStream_t st, const DevParams& p, int B, const clrrt_sample* S,
                               const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, const int* ctie,
                               const int* ncand, const float* ckey, const RollRes* res, int* fix_n, int* fix_ids,
                               int* fix_adj);
hipError_t launch_conflict(hipStream_t st, const DevParams& p, int B, const clrrt_sample* S,
                           const clrrt_node* reg, const clrrt_node* gbn, const SampleOut* so, const int* ctie,
                           int* first);
// Scratch of the multi-block compaction (k_compact_count / hipcub scan / k_compact_scatter).
struct CompactBufs {
  uint64_t* packed;   // [max_batch] per-sample (rows << 24 | nodes)
  uint64_t* scanned;  // [max_batch] exclusive prefix sums
  void* tmp;
  size_t tmp_bytes;
};
size_t compact_scan_bytes(int n);
size_t defer_select_bytes(int n);
hipError_t launch_defer_select(hipStream_t st, const int* gv, const uint8_t* pend, int n, int* out, int* n_out,
                               void* tmp, size_t tmp_bytes);
// tag_R > 0 (sharded rounds with deferred samples): each record's age in rounds relative to ring slot
// tag_slot (ring of tag_R slots of tag_B samples) in bits 8..15 of its goal field
hipError_t launch_compact(hipStream_t st, int L, const clrrt_sample* S, const int* cand, const clrrt_node* reg,
                          const clrrt_node* gbn, const SampleOut* so, int64_t row_base, int rank,
                          clrrt_node* out, Job* jobs, int64_t* totals, CompactBufs& cb, int tag_slot = 0,
                          int tag_R = 0, int tag_B = 1, bool totals_zeroed = false);
// The exchanged records (sort: by age tag, stable) into out in commit order, tags cleared; goal flags
// counted into *goal.  keys: [4 n] scratch.
size_t xorder_sort_bytes(int n);
hipError_t launch_xorder(hipStream_t st, const clrrt_node* recs, int n, bool sort, uint32_t* keys, void* tmp,
                         size_t tmp_bytes, clrrt_node* out, unsigned long long* goal);
// Bounding box (x0, y0, x1, y1) of the finite positions of recs[0 .. n), n = *n_dev when non-null.
hipError_t launch_bbox(hipStream_t st, const clrrt_node* recs, const int64_t* n_dev, int n_host, double* out4);
hipError_t launch_append(hipStream_t st, const clrrt_node* in, int n, int64_t base, clrrt_node* tree, NnRec* nn);
hipError_t launch_selftest_math(hipStream_t st, int fn, const double* a, const double* b, int n, double* out);
hipError_t launch_obs_distance(hipStream_t st, const DevParams& p, const BakedObs* obs, const double* states, int n,
                               double* out);
// cp: per-case parameters (units CLRRT_UNIT_FEASIBLE .. CLRRT_UNIT_CTRL), else null
hipError_t launch_selftest_units(hipStream_t st, int unit, const double* in, const BakedObs* obs, int n,
                                 const DevParams& p, const DevParams* cp, double* out);
// extractBestPath helpers: goal nodes (id, costS) appended in any order (count in *cnt), and the
// ancestor chain of `start` (start first) into path[0 .. cap) with its full length in *len.
struct GoalRec { int32_t id; float cost; };
hipError_t launch_goal_gather(hipStream_t st, const clrrt_node* tree, int64_t n, GoalRec* out, int* cnt);
hipError_t launch_backtrack(hipStream_t st, const clrrt_node* tree, int64_t n, int start, int cap, int* path,
                            int* len);
// initializeTree (rrtplanner.cpp:39-95) from the committed path pn[0 .. n) / prow (path-local rows).
struct ReinitArgs {
  DevParams p;
  const BakedObs* obs;
  const clrrt_node* pn;
  int n;
  const double* prow;
  double car[10];      // carState with the four appended zeros
  clrrt_node* tree;
  NnRec* nn;
  double* arena;
  int* kidx;           // [n] kept path index per new node; then [n] goal flag
  int64_t* koff;       // [n] new row offset per kept node
  double* terms;       // [2 * path rows] per-row cost term and lane term
  float* costs;        // [n]
  int64_t* out;        // [3] outcome, nodes, rows
  int rank;
  int64_t max_nodes, max_rows;
};
hipError_t launch_gather_nodes(hipStream_t st, const clrrt_node* tree, const int* ids, int n, clrrt_node* out);
hipError_t launch_path_transform(hipStream_t st, clrrt_node* nodes, int n, double* rows, int64_t nrows, int to_world,
                                 const double pose[3]);
hipError_t launch_tree_reinit(hipStream_t st, const ReinitArgs& a);
hipError_t launch_init_root(hipStream_t st, const double* state, clrrt_node* tree, NnRec* nn, double* arena);

}  // namespace clrrt
