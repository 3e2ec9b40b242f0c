// clrrt_capi.hip — host side of libclrrt: the C-ABI of include/clrrt.h.
//
// Round structure of one batch of expandTree iterations (rrtplanner.cpp:123-174) on the GPU:
//   1. nearest-node search for every sample against the frozen tree        (k_nn_partial/merge)
//   2. every candidate rollout of every sample, speculatively in parallel; a successful candidate
//      that passes the goal-bias gate continues in the same lane with the goal-biased rollout;
//      rows go to per-job slots                                              (k_rollout SPEC)
//   3. first success per sample -> regular node (+ goal-biased node)         (k_select)
//   4. EXACT mode only: first sample whose candidate list a node of an earlier sample of the round
//      would reorder (k_conflict) -> commit the prefix before it, re-draw nothing, retry the rest
//   5. scan committed samples -> node records, arena offsets, counters       (k_compact)
//   6. copy the accepted trajectories from their slots into the arena        (k_copy_rows)
//   7. append the records to the tree                                        (k_append)
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <climits>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <optional>
#include <string>
#include <vector>

#include "../../include/clrrt.h"
#include "clrrt_dev.hpp"
#include "clrrt_internal.hpp"

static const int kWalkMaxOver = 2048, kWalkMaxChunks = 64;  // walk overflow records, split waves per record

using namespace clrrt;

#define CAND_K 10
#define NN_K 11

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct clrrt_ctx {
  int device = 0;
  int rank = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  clrrt_params params;
  DevParams dp;
  clrrt_capacity cap;
  std::string err;
  // tree
  clrrt_node* tree = nullptr;
  NnRec* nn = nullptr;
  double* arena = nullptr;
  int64_t n_nodes = 0, n_rows = 0;
  // obstacles
  BakedObs* obs = nullptr;
  int n_obs = 0;
  ObsGrid grid{};              // device view of the static-obstacle grid
  void* grid_buf = nullptr;    // start | items | mov
  size_t grid_bytes = 0;
  // round buffers (capacity cap.max_batch samples)
  clrrt_sample* d_samples = nullptr;
  float* pk = nullptr;
  int* pi = nullptr;
  int64_t partial_cap = 0;  // entries (samples * chunks * K)
  int* cand = nullptr;
  float* ckey = nullptr;
  int* ncand = nullptr;
  int* ctie = nullptr;
  KeyId* sort_scratch = nullptr;
  int64_t sort_cap = 0;  // KeyId entries
  RollRes* res_spec = nullptr;
  clrrt_node* regnodes = nullptr;
  RollRes* res_gb = nullptr;
  double* slots = nullptr;  // rollout rows of one round, [2][max_batch * CAND_K][slot_rows][10] (allocated
                            // only when rows are not deferred: option "rows_deferred" 0 or the non-persistent path)
  int slot_rows = 0;
  // deferred rows (option "rows_deferred", default 1): the persistent rollouts store no rows; each commit
  // gathers its accepted rollouts' start states into rep_buf and the next persistent launch replays them
  // into the arena (flush_replays runs them alone when rows are needed before that)
  int rows_deferred = 1;
  void* rep_buf = nullptr;  // [2 max_batch] Replay
  int rep_n = 0;            // pending replays
  bool eval_deferred = false;  // the last eval_samples ran with deferred rows
  clrrt_node* gbnodes = nullptr;
  SampleOut* so = nullptr;
  int* first_conflict = nullptr;
  clrrt_node* out_nodes = nullptr;
  Job* jobs = nullptr;
  int64_t* totals = nullptr;
  bool totals_zeroed = false;  // the round's prologue fill reset totals (launch_compact skips its own fill)
  unsigned long long* work_ctr = nullptr;  // [3] algorithmic rollout work; [8..15] nn search statistics
  // spatial index of the tree (nearest-node search)
  float* nn_seed = nullptr;  // [max_batch] the brute-force chunks' shared per-sample key caps
  // bounding box of the tree's finite node positions (x0, y0, x1, y1), maintained on the host
  double bbox[4] = {HUGE_VAL, HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  double* d_bbox = nullptr;  // [4] device result of launch_bbox
  double* h_bbox = nullptr;  // [4] pinned
  int64_t nnw_min_nodes = 8192;       // walk search (clrrt_nnwalk.hip) from this tree size ("nn_walk_min")
  bool nnw_stateless = false;          // "nn_walk_stateless": the large-tree variant at every size (tests)
  // walk overflow ("nn_walk_budget_tiles", "nn_walk_budget_keys", 0 = off; "nn_walk_chunks" <= 64;
  // "nn_walk_max_over" records <= 2048); defaults from the cfg3 bench sweeps (round 3
  // with lag 2: 3072 tiles 1.039 vs 2048 1.031 M nodes/s, 8192 keys 1.008, 12 chunks 1.030)
  int nnw_bud_tiles = 3072, nnw_bud_ex = 4096, nnw_chunks = 16, nnw_max_over = 1024;
  // "nn_walk_max_over" unset: 1024 records, 2048 on trees of >= 6 Mi nodes (at 8 M nodes 1024 records ran out
  // and the samples past them searched alone: 31.7 -> 24.1 ms per 16384-sample round, profiles/r04u)
  bool nnw_max_over_set = false;
  // "nn_walk_budget_tiles" unset: max(3072, N / 2048) tiles (16 M nodes: 3072 overflowed 2048 samples per
  // round, 8192 -> 45.6 vs 58-59 ms; 8 M: 3072 stays best, 25.8 vs 29.9 ms at 8192, profiles/r04as)
  bool nnw_bud_tiles_set = false;
  int nnw_half_max = 4096;  // option "nn_walk_half_max": super-tiles up to which the walk keeps fp16 LDS bounds
  // option "nn_walk_hscale": the 3D index codes' heading axis, percent of rho per radian (round 6: 25 / 50 / 100 / 200
  // -> cfg3 1.289 / 1.293 / 1.274 / 1.232 M nodes/s, profiles/r06k_*)
  int nnw_hscale = 50;
  int nnw_lpt = 0;          // option "nn_walk_lpt": optimize samples first in each XCD's eighth (k_walk_lpt)
  int nnw_index = 5;        // option "nn_walk_index": the index's place order (WalkBufs::index_kind); 5 since round 6
  int nnw_lds_floor = 0;    // option "nn_walk_lds_floor": LDS bytes each walk wave reserves at least
  // option "nn_walk_waves": the walk's persistent grid (waves taking samples from per-XCD counters; 0 = one
  // wave per sample; -1, the default: 9 per CU).  A fixed grid leaves wave slots to the kernels that run
  // beside the lag-2 walk (the commit's k_select waited ~1.2 ms per round for slots behind ~1 ms walk waves)
  // and balances the walk's own tail: cfg3 1.164 -> 1.203 M nodes/s (round 4 sweep: 1024 / 1536 / 2048 /
  // 2560 waves -> 1.07 / 1.17 / 1.202 / 1.203 M), the 16 M-node search alone 62 -> 58 ms at 3072; the default
  // grid is used for batches of >= 4x its waves (below, one wave per sample).  Round 6: 8 per CU -- with the
  // rollout waves at 320 registers a walk wave fits beside them, and the rollout kernel gains more from the slots a
  // smaller walk grid leaves than the walk loses (cfg3, kind 5: 1536 / 1792 / 2048 / 2304 / 2560 waves -> 1.238 /
  // 1.257 / 1.275 / 1.256 / ~1.23 M nodes/s, profiles/r06i_*); then 9 per CU with the walk kernels at 96 VGPRs
  // (CLRRT_WALK_WAVES 5, clrrt_nnwalk.hip: two walk waves fit beside a rollout wave; 2048 / 2304 / 2560 / 2816 /
  // 3072 waves -> 1.285 / 1.310, 1.306 / 1.292, 1.303 / 1.287, 1.288 / 1.269 M against 1.288-1.290 M for the
  // 128-VGPR walk at 2048, profiles/r06r_*, r06s_*)
  int nnw_waves = -1;
  int nnw_double = 1;  // "nn_walk_double": build the next round's index while the side search runs
  WalkBufs nnw{};                      // allocated on first use
  // pipelined rounds: a second index set, so the next round's index is built while the side stream's
  // search still reads this one (swapped in after each commit); nnw_built: the tree size and frame the
  // current set's index was built for (n = -1: none)
  WalkBufs nnw_alt{};
  struct { int64_t n = -1; double ox, oy, x0, y0, x1, y1; float delta; } nnw_built;
  CompactBufs cmp{};                   // round compaction scratch
  // persistent rollouts (k_roll_run; k_roll_flag + k_roll_order for the queue order)
  int roll_persistent = 1;
  int nn_debug = 0;
  int roll_blocks = 0;       // persistent blocks (0: 5/8 of the CUs)
  int n_cu = 256;
  int* roll_q = nullptr;      // [1] queue head
  int* roll_best = nullptr;   // [max_batch] first successful candidate per sample
  int roll_priority = 1;      // option "roll_priority": likely-long rollouts first (k_roll_order)
  int roll_coop = 1;          // option "roll_coop": wave-cooperative collision checks in k_roll_run
  int roll_spread = 1;        // option "roll_spread": a short queue is spread over the persistent waves
  int roll_lanes = 0;         // option "roll_lanes": lanes per wave that take jobs (0: 64, or fewer by roll_spread)
  int nn_exact_fused = 1;     // option "nn_exact_fused": EXACT lists of small trees by k_nn_exact_fused
  int exact_min_width = 8;    // option "exact_min_width": EXACT rounds speculate at least this many samples
  // option "exact_fixup" (default 1): EXACT rounds resolve a conflict by rolling out the conflicting new nodes for
  // the sample (k_conflict_fix) instead of ending the committed prefix there, when that decides it
  int exact_fixup = 1;
  // option "exact_fixup_cap": fix-up rollouts run at most this many steps (0: to their end); one that reaches it is
  // undecided and ends the prefix at its sample (re-evaluated next round), so a round never waits for a long one
  int exact_fix_cap = 0;
  int* fix_n = nullptr;        // [max_batch]
  int* fix_ids = nullptr;      // [max_batch * FIX_MAX]
  int* fix_adj = nullptr;      // [max_batch * 5]
  NnRec* fix_xrec = nullptr;   // [2 max_batch] the round's new nodes as nearest-node records
  int* fix_xi = nullptr;       // [2 max_batch] samples whose list is recomputed, their new-node counts
  int* fix_xcand = nullptr;    // [max_batch * K] recomputed lists
  float* fix_xkey = nullptr;   // [max_batch * K]
  int* fix_xn = nullptr;       // [2 max_batch] list lengths, tie flags
  std::vector<int> h_fix_cand;
  std::vector<RollRes> h_fix_spec;
  Job* fix_jobs = nullptr;     // [max_batch * CAND_K]
  RollRes* fix_res = nullptr;  // [max_batch * CAND_K]
  std::vector<int> h_fix;      // fix_n then fix_ids
  std::vector<clrrt_sample> h_fix_smp;
  std::vector<Job> h_fix_jobs;
  std::vector<int> h_fix_owner;
  std::vector<RollRes> h_fix_res;
  std::vector<SampleOut> h_fix_so;
  // EXACT: rounds, conflicts resolved, fix-up rollouts, rounds ended by a conflict; then why the ending conflicts
  // were not resolved: a fix-up succeeded, tie, key equal to the threshold, > FIX_MAX nodes, k pushed out, full
  // window without a result
  int64_t ex_stats[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int* roll_perm = nullptr;   // [max_batch * CAND_K] queue order
  int* roll_pflag = nullptr;  // [2 max_batch * CAND_K + scratch] flags, scan positions, scan scratch
  // extractBestPath scratch (allocated on first use, max_nodes entries each)
  GoalRec* goal_recs = nullptr;
  int* bp_path = nullptr;  // [max_nodes + 2]: chain, then count and length
  // committed path (MotionPlanner::bestNodes) + initializeTree scratch
  clrrt_node* path_nodes = nullptr;
  double* path_rows = nullptr;
  int path_cap = 0;
  int64_t path_rows_cap = 0;
  int path_n = 0;
  int64_t path_nrows = 0;
  int* ri_int = nullptr;       // [2 * path_cap + ...] ids, kept index, goal flags
  int64_t* ri_off = nullptr;   // [path_cap] new row offsets, then [3] outcome / nodes / rows
  float* ri_cost = nullptr;    // [path_cap]
  double* ri_terms = nullptr;  // [2 * path_rows_cap]
  double reg_x0 = 0, reg_y0 = 0, reg_x1 = 0, reg_y1 = 0;  // sampling region + margin
  // pipelined BATCH rounds (clrrt_expand): while a round's rollouts run on `stream`, the walk search
  // of the next round's samples over the same tree runs on `side` into the *2 buffers; the round
  // then merges in the nodes it appended (launch_nn_delta) and the buffers swap
  int nn_pipeline = 1;  // option "nn_pipeline"
  hipStream_t side = nullptr;
  // option "cu_split" (k = 1..7): the rollouts run on their own stream restricted to k/8 of the CUs and
  // the side stream (the next round's search) on the other CUs, so no search wave shares a SIMD with a
  // rollout wave; 0: one unrestricted main stream for both (default)
  int cu_split = 0;
  hipStream_t roll_st = nullptr;
  hipEvent_t ev_rs0 = nullptr, ev_rs1 = nullptr;
  hipEvent_t ev_tree = nullptr, ev_walk = nullptr, ev_commit = nullptr;
  clrrt_sample* d_samples2 = nullptr;
  clrrt_sample* h_samples2 = nullptr;
  int* cand2 = nullptr;
  float* ckey2 = nullptr;
  int* ncand2 = nullptr;
  int* ctie2 = nullptr;
  // option "nn_lag" (1 or 2; 0 = by query length): how many rounds ahead the pipelined BATCH rounds search
  // (2: expand_lag2).  The default picks 2 for long queries (a budget of >= 1 s or >= 64 rounds), 1 for
  // short ones: round-3 A/B, cfg3 (2 s) 1.031 vs 1.015 M nodes/s for lag 2; cfg2 (200 ms) 0.551 vs 0.565 M
  // for lag 1; cfg5 (200 ms) equal.  (With round 2's rollout kernel lag 1 was ahead on cfg3 too.)
  // Lag 2 keeps a third list set (*3), a third walk index set and a second side stream (allocated on
  // first use).
  int nn_lag = 0;
  clrrt_sample* d_samples3 = nullptr;
  clrrt_sample* h_samples3 = nullptr;
  int* cand3 = nullptr;
  float* ckey3 = nullptr;
  int* ncand3 = nullptr;
  int* ctie3 = nullptr;
  WalkBufs nnw3{};
  hipStream_t side2 = nullptr;
  // lag 2: the appended-node merges run on their own stream (mst), behind the commit and the slot's walk
  // (events ev_lagw); with option "stream_prio" (default 1) the main and merge streams have the device's
  // highest priority and the walk streams (side, side2) its lowest, so the commit and merge kernels are
  // not queued behind thousands of walk waves (kernel trace: k_select 16 us -> 1.9 ms late in a query)
  hipStream_t mst = nullptr;
  // option "nn_split_delta" (default 0, round 6): the appended-node search of a slot is split by commit.  The
  // nodes a commit appends are searched for the round-after-next's samples (slot B) on mst as soon as that slot's
  // walk is done (its list seeds the chunk caps: unseeded, the search costs ~4x, profiles/r06l_*), beside the next
  // round's rollouts; after the next commit only that commit's nodes remain, and the walk list, the first partial
  // lists and the second are merged.  Round 5's single search of both commits' nodes started after the walk and
  // was ~1.2 ms of the round's critical path (profiles/r06j_*).  (A fifth stream of its own for the first searches
  // made every rollout kernel ~60% slower, split or not -- 4.1 vs 2.6 ms per round, profiles/r06n_*; not the
  // hardware queue count: GPU_MAX_HW_QUEUES 2 / 4 / 8 / 16 leave the default build unchanged, r06p_*.)  On mst the lists are
  // the same and the round is not faster (cfg3 1.281 / 1.275 vs 1.292 M nodes/s, list wait 1.06 / 0.95 vs 1.08 ms,
  // profiles/r06o_*): the lists wait for the walk, not for this search.
  int nn_split_delta = 0;
  // option "nn_delta_early" (default 1, round 6): the appended-node search of a slot starts after its walk's main grid
  // (key caps from k_walk_seed, per slot in wseed) instead of after the overflow split and its merge, so it runs beside
  // the split (a cfg3 trace: main grid done 1.7 ms before the rollout kernel, split until 0.6 ms after it, the search
  // after that until 1.9 ms, profiles/r06w_cfg3_list_crit.txt); the merge still waits for the whole walk.
  int nn_delta_early = 1;
  // option "nn_lane_order" (default 1, round 6): the lag-2 appended-node search puts optimize samples on their own
  // lanes (k_nn_order), so explore lanes do not idle while optimize lanes compute exact keys
  int nn_lane_order = 1;
  int* nn_order = nullptr;  // [max_batch]
  float* wseed[3] = {nullptr, nullptr, nullptr};      // per slot: [max_batch] caps taken after the main walk grid
  hipEvent_t ev_wm[3] = {nullptr, nullptr, nullptr};  // per slot: recorded after the main walk grid (and wseed)
  float* nn_seed2 = nullptr;                   // [max_batch] the first searches' chunk caps
  float* d1pk[3] = {nullptr, nullptr, nullptr};  // per slot: the first partial lists (partial_cap entries)
  int* d1pi[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_d1[3] = {nullptr, nullptr, nullptr};  // recorded after a slot's first partial search
  hipEvent_t ev_s[3] = {nullptr, nullptr, nullptr};   // recorded after a slot's samples reached the device
  hipEvent_t ev_lagw[3] = {nullptr, nullptr, nullptr};
  int stream_prio = 1;
  int walk_cu_reserve = 0;  // option "walk_cu_reserve" k = 1..7: lag-2 walk streams kept off k/8 of the CUs
  hipEvent_t ev_lag[3] = {nullptr, nullptr, nullptr};
  int stream_prio_applied = 0;  // the priority setting the current streams were created with
  bool side_prio_set = false;   // option "side_priority" made the side stream (apply_stream_prio keeps it)
  // clrrt_round_prefetch: declared next samples; pf_state 1 = their walk was launched (lists in the
  // *2 buffers, merge pending), 2 = merged and swapped in for pf_samples
  std::vector<clrrt_sample> pf_next, pf_samples;
  int pf_state = 0;
  // Deferred samples (BATCH option "defer_steps" T > 0; see Carry in clrrt_kernels.hip): every rollout chain
  // runs at most T more steps per launch; suspended chains resume at the front of the next launch and a
  // sample commits at the first commit after which nothing its result depends on is still running.  The
  // per-job results, lists and first-success flags of the rounds in flight live in rings of R round slots
  // (a chain of at most 2 n_steps_max steps resolves within ceil(2 n_steps_max / T) launches, so a slot is
  // free again when the ring comes round); the commit buffers hold vcap views (deferred + this round's).
  struct {
    int T = 0;                    // option value (0: off)
    bool active = false;          // the current expansion defers
    int R = 0;                    // ring slots allocated (for T_alloc / n_steps_alloc)
    int T_alloc = 0, n_steps_alloc = 0;
    int64_t vcap = 0;             // views the commit buffers hold
    RollRes* res = nullptr;       // [R][B][K]
    RollRes* res_gb = nullptr;    // [R][B][K]
    int* cand = nullptr;          // [R][B][K]
    int* ncand = nullptr;         // [R][B]
    clrrt_sample* samp = nullptr; // [R][B]
    int* best = nullptr;          // [R][B]
    int* dlist[2] = {nullptr, nullptr};  // ring indices of the deferred samples (views 0 .. nd)
    int cur_dl = 0, nd = 0;
    int nd_eval = -1;             // nd when the current round's views were selected (-1: no views)
    int* gv = nullptr;            // [vcap]
    uint8_t* pend = nullptr;      // [vcap]
    void* sel_tmp = nullptr;
    size_t sel_bytes = 0;
    int* d_cnt = nullptr;         // [3] selected views, suspended chains, this round's samples left pending (device)
    void* carry[2] = {nullptr, nullptr};
    int cur_c = 0, ncarry = 0, carry_cap = 0;
    int64_t round = 0;            // rounds of the current expansion
    int slot = 0;                 // ring slot of the current round
    int64_t deferred_total = 0;   // samples deferred at least once (statistics)
  } def;
  // Sharded BATCH expansion (clrrt_set_shards): this rank's slice of every round, one exchange of the
  // accepted-node records per round through the caller's collective
  struct {
    int rank = 0, world = 1;
    void* dev_local = nullptr;     // the caller's buffer the local records go to
    int cap_local = 0;
    clrrt_exchange_fn fn = nullptr;
    void* user = nullptr;
    double max_ms = 0;             // largest elapsed query time over the ranks at the last exchange
    int64_t nd_global = 0;         // deferred samples pending on all ranks after the last exchange
    int64_t rows_stop = 0;         // ranks whose arena cannot take another round (the same stop everywhere)
    int last_nb = 0;               // this rank's slice of the last round
    clrrt_node* xbuf = nullptr;    // the exchanged records in commit order (deferred samples: by age)
    uint32_t* xkey = nullptr;      // [2 xcap] sort keys (age), [2 xcap] record indices
    void* xtmp = nullptr;
    size_t xtmp_bytes = 0;
    int64_t xcap = 0;
    unsigned long long* d_goal = nullptr;  // goal nodes among the appended records (device counter)
    // errors are collective: a rank that fails sends an error flag through the exchange's aux word (bit 48) in
    // the exchange the other ranks make next -- a round's, or the closing exchange every sharded expansion ends
    // with -- so every rank leaves the expansion instead of waiting in a collective the failed rank never joins
    bool poison_seen = false;      // an exchange of this expansion reported another rank's failure
    bool fn_failed = false;        // the exchange hook itself failed (the collective is broken: no more calls)
  } sh;
  // option "fail_at_round" k (fault injection, tests): the k-th commit from now fails with CLRRT_ECAPACITY
  // after the round's deferred-sample bookkeeping, as the "trajectory arena full" check does
  int fail_at_round = 0;
  // option "fail_after_exchange" k (fault injection, tests): the k-th exchange from now fails after the hook
  // returned (as a failure of the work that follows the round's exchange would)
  int fail_after_exchange = 0;
  // CLRRT_DEBUG_SYNC (diagnostics, read once at clrrt_create): a heartbeat buffer the rollout kernel's waves
  // write, polled while waiting for the launch
  bool debug_sync = false;
  unsigned long long* dbg_host = nullptr;
  // clrrt_iteration_log: one record per committed iteration (EXACT / non-deferred BATCH rounds)
  bool iter_log = false;
  // the tree size after each commit of the last clrrt_expand (its rounds, then the drain of deferred samples when it
  // appended anything): clrrt_round_sizes
  std::vector<int64_t> round_sizes;
  std::vector<clrrt_iteration> iters;
  std::vector<SampleOut> iter_tmp;
  // host staging (pinned)
  clrrt_sample* h_samples = nullptr;
  int64_t* h_totals = nullptr;
  int* h_int = nullptr;
  // last round_eval bookkeeping
  int64_t last_eval_rows = 0;
  int64_t last_goal_nodes = 0;
  // counters
  clrrt_counters counters{};
  int64_t nn_bf_keys = 0, nn_samples = 0;  // search work: brute-force-equivalent keys, samples searched
  int64_t nn_super_bounds = 0;             // walk searches' phase-1 super-tile bounds (samples x super-tiles)
  // timing
  bool timing = false;
  // per class: 0 nearest-node search (index builds, walks, merges), 1 rollouts, 2 select / commit,
  // 3 the walk searches alone (launch_nn_walk_search: sample order, k_walk_search, split + merge; within class 0),
  // 4 the main stream's wait for a round's lists (the side streams' walk + merge running past the work queued
  // before it: the search's share of the round's critical path), 5 sharded exchanges (the stream span from the
  // records' copy to the gathered records' availability: the collective on the critical path)
  static constexpr int kKtClasses = 6;
  double kt_ms[kKtClasses] = {};
  int64_t kt_n[kKtClasses] = {};
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
};

// ------------------------------------------------------------------------------------------ util
static void pf_reset(clrrt_ctx* c);
static int flush_replays(clrrt_ctx* c);
static int append_nodes(clrrt_ctx* c, const clrrt_node* dev_nodes, int n);
static int watchdog_check(clrrt_ctx* c);
static void defer_roll_args(clrrt_ctx* c, RollArgs& a, bool capped);
static int commit_round(clrrt_ctx* c, int nn, double elapsed_ms, int* n_app);
static int ensure_slots(clrrt_ctx* c);

static int fail(clrrt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPC(c, call)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail((c), CLRRT_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));        \
  } while (0)

template <typename T>
static hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc((void**)p, count * sizeof(T));
}

static hipEvent_t ev_get(clrrt_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct KTimer {
  clrrt_ctx* c;
  int which;
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  KTimer(clrrt_ctx* c_, int w, hipStream_t s_ = nullptr) : c(c_), which(w), s(s_ ? s_ : c_->stream) {
    if (!c->timing) return;
    a = ev_get(c);
    b = ev_get(c);
    if (a) hipEventRecord(a, s);
  }
  ~KTimer() {
    if (!c->timing || !a || !b) return;
    hipEventRecord(b, s);
    c->ev_pending.push_back({which, {a, b}});
  }
};

static void drain_timers(clrrt_ctx* c) {
  for (auto& pe : c->ev_pending) {
    float ms = 0;
    hipEventSynchronize(pe.second.second);
    if (hipEventElapsedTime(&ms, pe.second.first, pe.second.second) == hipSuccess) {
      c->kt_ms[pe.first] += ms;
      c->kt_n[pe.first] += 1;
    }
    c->ev_pool.push_back(pe.second.first);
    c->ev_pool.push_back(pe.second.second);
  }
  c->ev_pending.clear();
}

// ------------------------------------------------------------------------------------------ params
static void derive(const clrrt_params& q, DevParams& d, int n_obs) {
  memset(&d, 0, sizeof(d));
  d.dmax = q.veh.dmax; d.ddmax = q.veh.ddmax; d.Td = q.veh.Td; d.Ta = q.veh.Ta;
  d.amin = q.veh.amin; d.amax = q.veh.amax; d.L = q.veh.L; d.Vch = q.veh.Vch; d.Kus = q.veh.Kus;
  d.dt = q.sim_dt; d.tla = q.ctrl_tla; d.mindla = q.ctrl_mindla;
  d.dla_c = q.ctrl_mindla - q.ctrl_tla * q.ctrl_dlavmin;  // controller.cpp:14
  d.Kp = q.ctrl_Kp; d.Ki = q.ctrl_Ki; d.ref_res = q.ref_res; d.vmax = q.vmax; d.ay_road_max = q.ay_road_max;
  d.g0 = q.goal[0]; d.g1 = q.goal[1]; d.g2 = q.goal[2]; d.g3 = q.goal[3];
  d.W0 = q.Wcost[0]; d.W1 = q.Wcost[1]; d.W2 = q.Wcost[2]; d.W3 = q.Wcost[3]; d.W4 = q.Wcost[4];
  d.lane_shift0 = q.lane_shift0; d.Cxy1 = q.Cxy[1]; d.Cxy2 = q.Cxy[2];
  d.feas_len = 2.1 * q.ref_res;
  // getGoalReference reference.cpp:27-50 (query constants)
  double dla_end = std::max(q.ctrl_mindla, d.dla_c + q.ctrl_tla * std::abs(q.goal[3]));
  double Dext = dla_end, Dal = 1;
  const double* g = q.goal;
  double sg2, cg2;
  ::sincos(g[2], &sg2, &cg2);  // getGoalReference: cos and sin of one argument -> glibc sincos
  d.gbP1x = g[0] + Dal * cg2; d.gbP1y = g[1] + Dal * sg2;
  d.gbP2x = g[0] - Dal * cg2; d.gbP2y = g[1] - Dal * sg2;
  d.gbF1x = d.gbP1x + (Dext + Dal) * cg2; d.gbF1y = d.gbP1y + (Dext + Dal) * sg2;
  d.gbF2x = d.gbP2x + (Dext + Dal) * cg2; d.gbF2y = d.gbP2y + (Dext + Dal) * sg2;
  // feasibleGoalBias rrtplanner.cpp:294-299 (the .y coordinates use cos, as the reference does)
  double R1 = 4.77;
  d.gbR2 = R1 - 0.3;
  d.gbLx = g[0] + R1 * cos(g[2] - M_PI_2); d.gbLy = g[1] + R1 * cos(g[2] - M_PI_2);
  d.gbRx = g[0] + R1 * cos(g[2] + M_PI_2); d.gbRy = g[1] + R1 * cos(g[2] + M_PI_2);
  d.bend = q.bend; d.obs_use_pred = q.obs_use_pred; d.sort_limit = std::min(q.sort_limit, CAND_K);
  d.coll_mode = q.collision_mode;
  int n = 0;
  while (n < (20 / q.sim_dt)) n++;  // `for(int i = 0; i<(20/sim_dt); i++)` simulation.cpp:58
  d.n_steps_max = n;
  d.use_exp = !(q.Wcost[2] == 0.0 && q.Wcost[3] >= 0.0);  // W2*exp(-W3*Dobs) is exactly +0 otherwise
  d.n_obs = n_obs;
  d.need_gap = (q.collision_mode == CLRRT_COLLISION_OBB) && d.use_exp;
}


static void bbox_reset(clrrt_ctx* c) {
  c->bbox[0] = c->bbox[1] = HUGE_VAL;
  c->bbox[2] = c->bbox[3] = -HUGE_VAL;
}
static void bbox_add(clrrt_ctx* c, double x0, double y0, double x1, double y1) {
  c->bbox[0] = std::min(c->bbox[0], x0); c->bbox[1] = std::min(c->bbox[1], y0);
  c->bbox[2] = std::max(c->bbox[2], x1); c->bbox[3] = std::max(c->bbox[3], y1);
}

// Region holding the samples (sampleAroundVehicle rrtplanner.cpp:187-201: rLong in [0, dGoal+10],
// rLat in [-7, 7] about the goal heading) and the goal, with a margin; nodes outside it go to the
// index's always-scanned overflow cell.
static void sample_region(const clrrt_params& q, double& x0, double& y0, double& x1, double& y1) {
  const double* g = q.goal;
  double dGoal = std::sqrt(g[0] * g[0] + g[1] * g[1]);
  double hd = std::atan2(g[1], g[0]);
  double ch = std::cos(hd), sh = std::sin(hd);
  x0 = y0 = 1e300; x1 = y1 = -1e300;
  for (double L : {0.0, dGoal + 10})
    for (double W : {-7.0, 7.0}) {
      double x = L * ch - W * sh, y = L * sh + W * ch;
      x0 = std::min(x0, x); x1 = std::max(x1, x); y0 = std::min(y0, y); y1 = std::max(y1, y);
    }
  x0 = std::min(x0, g[0]); x1 = std::max(x1, g[0]); y0 = std::min(y0, g[1]); y1 = std::max(y1, g[1]);
  const double m = 2.0;
  x0 -= m; y0 -= m; x1 += m; y1 += m;
}

// ------------------------------------------------------------------------------------------ C-ABI
extern "C" {

int clrrt_abi_version(void) { return CLRRT_ABI_VERSION; }
static_assert(sizeof(clrrt_exchange_io) == 128, "clrrt_exchange_io layout (clrrt/abi.py ExchangeIO)");

int clrrt_params_default(clrrt_params* p, double v0, const double goal[4], double vmax) {
  if (!p) return CLRRT_EINVAL;
  memset(p, 0, sizeof(*p));
  // Vehicle::setPrius vehicle.h:39-60
  p->veh.dmax = 0.52; p->veh.ddmax = 0.3294; p->veh.Td = 0.3; p->veh.Ta = 0.3;
  p->veh.amin = -6; p->veh.amax = 2; p->veh.L = 2.7;
  double lf = 1.0868, lr = 1.6132, Cf = 22201, Cr = 22201, m = 950 + 640;
  p->veh.Kus = (m / p->veh.L) * (lr / Cf - lf / Cr);
  p->veh.Vch = 20;
  // parameters.launch:3-20
  p->ctrl_tla = 1.4; p->ctrl_mindla = 3.2; p->ctrl_dlavmin = 3; p->ref_int = 0.02; p->ref_mindist = 0.2;
  p->sim_dt = 0.04; p->ctrl_Kp = 8; p->ctrl_Ki = 0.05;
  p->Wcost[0] = 10; p->Wcost[1] = 5; p->Wcost[2] = 0; p->Wcost[3] = 4; p->Wcost[4] = 1;
  // updateReferenceResolution controller.cpp:18-21 at the query's start velocity
  p->ref_res = std::max(std::abs(v0) * p->ref_int, p->ref_mindist);
  p->vmax = vmax;
  p->ay_road_max = 0;  // rrt_node.cpp:16, never assigned
  for (int i = 0; i < 4; i++) p->goal[i] = goal ? goal[i] : 0.0;
  p->bend = 0;
  p->obs_use_pred = 1;  // rrt_node.cpp:11
  p->sort_limit = 10;   // rrtplanner.cpp:13
  p->collision_mode = CLRRT_COLLISION_STUB;
  return CLRRT_OK;
}

// glibc random_r TYPE_3 (degree 31, separation 3), seeded like srandom_r: r[0..30] = state,
// r[31] = front index, r[32] = rear index.
void clrrt_rng_seed(clrrt_rng* g, uint32_t seed) {
  int32_t* s = g->r;
  int32_t word = (int32_t)(seed == 0 ? 1 : seed);
  s[0] = word;
  for (int i = 1; i < 31; i++) {
    int32_t hi = word / 127773, lo = word % 127773;
    word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    s[i] = word;
  }
  s[31] = 3;
  s[32] = 0;
  s[33] = 0;
  g->pos = 0;
  for (int i = 0; i < 310; i++) clrrt_rng_next(g);
}

int32_t clrrt_rng_next(clrrt_rng* g) {
  int32_t* s = g->r;
  int f = s[31], r = s[32];
  uint32_t v = (uint32_t)s[f] + (uint32_t)s[r];
  s[f] = (int32_t)v;
  int32_t out = (int32_t)(v >> 1);
  f = f + 1 == 31 ? 0 : f + 1;
  r = r + 1 == 31 ? 0 : r + 1;
  s[31] = f;
  s[32] = r;
  return out;
}

// sampleAroundVehicle rrtplanner.cpp:187-201 (rLong, rLat) + heuristic draw :142-143 (r).
int clrrt_draw_samples(const clrrt_params* p, clrrt_rng* rng, int32_t n, clrrt_sample* out) {
  if (!p || !rng || (n > 0 && !out)) return CLRRT_EINVAL;
  const double* g = p->goal;
  const double RM = 2147483647.0;  // RAND_MAX
  double dGoal = sqrt(g[0] * g[0] + g[1] * g[1]);
  double hd = atan2(g[1], g[0]);
  double latMin = -7, latMax = 7;
  float fl = (float)(RM / (dGoal + 10));
  float fw = (float)(RM / (latMax - latMin));
  double ch, sh, cq, sq;
  ::sincos(hd, &sh, &ch);  // sampleAroundVehicle: cos/sin pairs of one argument -> glibc sincos
  ::sincos(hd + M_PI / 2, &sq, &cq);
  for (int j = 0; j < n; j++) {
    double rLong = (float)clrrt_rng_next(rng) / fl;
    double rLat = latMin + (float)clrrt_rng_next(rng) / fw;
    out[j].x = rLong * ch + rLat * cq;
    out[j].y = rLong * sh + rLat * sq;
    double r = (double)clrrt_rng_next(rng) / (double)(2147483647 / 1);
    out[j].explore = r <= ((0 * 0.3) + (1 * 0.7));  // RRT.goalReached is never set
    out[j].pad = 0;
  }
  return CLRRT_OK;
}

const char* clrrt_last_error(const clrrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

static void free_all(clrrt_ctx* c) {
  if (c->side) hipStreamSynchronize(c->side);  // side-stream work (prefetched search) uses the *2 buffers
  void* ptrs[] = {c->tree, c->nn, c->arena, c->obs, c->d_samples, c->pk, c->pi, c->cand, c->ckey, c->ncand,
                  c->ctie, c->sort_scratch, c->res_spec, c->regnodes, c->res_gb, c->gbnodes, c->so, c->first_conflict,
                  c->out_nodes, c->jobs, c->slots, c->rep_buf, c->totals, c->work_ctr, c->grid_buf,
                  c->nn_seed, c->d_bbox, c->roll_q, c->roll_best, c->roll_perm, c->roll_pflag,
                  c->goal_recs, c->bp_path, c->path_nodes, c->path_rows, c->ri_int, c->ri_off, c->ri_cost,
                  c->ri_terms, c->nnw.keys, c->nnw.keys2, c->nnw.vals, c->nnw.vals2, c->nnw.tmp, c->nnw.P, c->nnw.Q,
                  c->nnw.CE, c->nnw.ID, c->nnw.tiles, c->nnw.supers, c->nnw.sorder, c->nnw.HEAD, c->nnw.ovf_n, c->nnw.ovf, c->nnw.pk, c->nnw.pi, c->nnw_alt.keys, c->nnw_alt.keys2, c->nnw_alt.vals, c->nnw_alt.vals2, c->nnw_alt.tmp, c->nnw_alt.P, c->nnw_alt.Q, c->nnw_alt.CE, c->nnw_alt.ID, c->nnw_alt.tiles, c->nnw_alt.supers, c->nnw_alt.sorder, c->nnw_alt.HEAD, c->nnw_alt.ovf_n, c->nnw_alt.ovf, c->nnw_alt.pk, c->nnw_alt.pi, c->nnw.skeys, c->nnw.sids, c->nnw_alt.skeys, c->nnw_alt.sids, c->cmp.packed, c->cmp.scanned,
                  c->cmp.tmp, c->d_samples2, c->cand2, c->ckey2, c->ncand2, c->ctie2, c->d_samples3, c->cand3, c->ckey3,
                  c->ncand3, c->ctie3, c->nnw3.keys, c->nnw3.keys2, c->nnw3.vals, c->nnw3.vals2, c->nnw3.tmp, c->nnw3.P,
                  c->nnw3.Q, c->nnw3.CE, c->nnw3.ID, c->nnw3.tiles, c->nnw3.supers, c->nnw3.sorder, c->nnw3.HEAD,
                  c->nnw3.ovf_n, c->nnw3.ovf, c->nnw3.pk, c->nnw3.pi, c->nnw3.skeys, c->nnw3.sids,
                  c->nnw.trun, c->nnw_alt.trun, c->nnw3.trun, c->nnw.wctr, c->nnw_alt.wctr, c->nnw3.wctr};
  for (void* p : ptrs)
    if (p) hipFree(p);
  void* sptrs[] = {c->sh.xbuf, c->sh.xkey, c->sh.xtmp, c->sh.d_goal, c->fix_n, c->fix_ids, c->fix_jobs, c->fix_res, c->fix_adj,
                   c->fix_xrec, c->fix_xi, c->fix_xcand, c->fix_xkey, c->fix_xn};
  for (void* p : sptrs)
    if (p) hipFree(p);
  void* dptrs[] = {c->def.res, c->def.res_gb, c->def.cand, c->def.ncand, c->def.samp, c->def.best, c->def.dlist[0],
                   c->def.dlist[1], c->def.gv, c->def.pend, c->def.sel_tmp, c->def.d_cnt, c->def.carry[0],
                   c->def.carry[1]};
  for (void* p : dptrs)
    if (p) hipFree(p);
  if (c->h_samples) hipHostFree(c->h_samples);
  if (c->h_samples2) hipHostFree(c->h_samples2);
  if (c->h_samples3) hipHostFree(c->h_samples3);
  if (c->side2) hipStreamSynchronize(c->side2);
  if (c->side2) hipStreamDestroy(c->side2);
  for (auto e : c->ev_lag)
    if (e) hipEventDestroy(e);
  for (auto e : c->ev_lagw)
    if (e) hipEventDestroy(e);
  if (c->mst) hipStreamSynchronize(c->mst);
  if (c->mst) hipStreamDestroy(c->mst);
  for (int q = 0; q < 3; q++) {
    if (c->ev_d1[q]) hipEventDestroy(c->ev_d1[q]);
    if (c->ev_s[q]) hipEventDestroy(c->ev_s[q]);
    if (c->d1pk[q]) hipFree(c->d1pk[q]);
    if (c->wseed[q]) hipFree(c->wseed[q]);
    if (q == 0 && c->nn_order) hipFree(c->nn_order);
    if (c->ev_wm[q]) hipEventDestroy(c->ev_wm[q]);
    if (c->d1pi[q]) hipFree(c->d1pi[q]);
  }
  if (c->nn_seed2) hipFree(c->nn_seed2);
  if (c->side) hipStreamSynchronize(c->side);
  if (c->ev_tree) hipEventDestroy(c->ev_tree);
  if (c->ev_walk) hipEventDestroy(c->ev_walk);
  if (c->ev_commit) hipEventDestroy(c->ev_commit);
  if (c->side) hipStreamDestroy(c->side);
  if (c->roll_st) hipStreamDestroy(c->roll_st);
  if (c->ev_rs0) hipEventDestroy(c->ev_rs0);
  if (c->ev_rs1) hipEventDestroy(c->ev_rs1);
  if (c->h_totals) hipHostFree(c->h_totals);
  if (c->h_int) hipHostFree(c->h_int);
  if (c->h_bbox) hipHostFree(c->h_bbox);
  if (c->dbg_host) hipHostFree(c->dbg_host);
  for (auto& pe : c->ev_pending) { hipEventDestroy(pe.second.first); hipEventDestroy(pe.second.second); }
  for (auto e : c->ev_pool) hipEventDestroy(e);
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
}

int clrrt_create(const clrrt_params* p, const clrrt_capacity* cap, int device, clrrt_ctx** out) {
  if (!p || !out) return CLRRT_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CLRRT_EHIP;
  if (device < 0 || device >= ndev) return CLRRT_EINVAL;
  clrrt_ctx* c = new clrrt_ctx();
  c->device = device;
  c->params = *p;
  c->debug_sync = getenv("CLRRT_DEBUG_SYNC") != nullptr;
  clrrt_capacity dc;
  dc.max_nodes = 1 << 20;
  dc.max_rows = 1 << 24;
  dc.max_batch = 4096;
  dc.max_obstacles = 4096;
  c->cap = cap ? *cap : dc;
  if (c->cap.max_nodes < 2 || c->cap.max_rows < 2 || c->cap.max_batch < 1 || c->cap.max_obstacles < 0) {
    delete c;
    return CLRRT_EINVAL;
  }
  derive(c->params, c->dp, 0);
  int rc = CLRRT_OK;
  auto chk = [&](hipError_t e) {
    if (e != hipSuccess && rc == CLRRT_OK) { rc = CLRRT_EHIP; c->err = hipGetErrorString(e); }
  };
  chk(hipSetDevice(device));
  chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  c->own_stream = true;
  const int64_t B = c->cap.max_batch;
  chk(dalloc(&c->tree, c->cap.max_nodes));
  chk(dalloc(&c->nn, c->cap.max_nodes));
  chk(dalloc(&c->arena, (size_t)c->cap.max_rows * 10));
  chk(dalloc(&c->obs, std::max<int64_t>(1, c->cap.max_obstacles)));
  chk(dalloc(&c->d_samples, B));
  c->partial_cap = std::max<int64_t>(B * 16, 4096) * NN_K;
  chk(dalloc(&c->pk, c->partial_cap));
  chk(dalloc(&c->pi, c->partial_cap));
  chk(dalloc(&c->cand, B * CAND_K));
  chk(dalloc(&c->ckey, B * CAND_K));
  chk(dalloc(&c->ncand, B));
  chk(dalloc(&c->ctie, B));
  chk(dalloc(&c->d_samples2, B));
  chk(dalloc(&c->cand2, B * CAND_K));
  chk(dalloc(&c->ckey2, B * CAND_K));
  chk(dalloc(&c->ncand2, B));
  chk(dalloc(&c->ctie2, B));
  chk(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  chk(hipEventCreateWithFlags(&c->ev_tree, hipEventDisableTiming));
  chk(hipEventCreateWithFlags(&c->ev_walk, hipEventDisableTiming));
  chk(hipEventCreateWithFlags(&c->ev_commit, hipEventDisableTiming));
  chk(dalloc(&c->res_spec, B * CAND_K));
  chk(dalloc(&c->regnodes, B));
  chk(dalloc(&c->res_gb, B * CAND_K));
  c->slot_rows = 0;  // slots allocated on first use (ensure_slots)
  chk(hipMalloc(&c->rep_buf, replay_bytes() * (size_t)2 * B));
  chk(dalloc(&c->gbnodes, B));
  chk(dalloc(&c->so, B));
  chk(dalloc(&c->first_conflict, 1));
  chk(dalloc(&c->out_nodes, 2 * B));
  chk(dalloc(&c->jobs, 2 * B));
  chk(dalloc(&c->totals, 8));
  chk(dalloc(&c->cmp.packed, B));
  chk(dalloc(&c->cmp.scanned, B));
  c->cmp.tmp_bytes = compact_scan_bytes((int)B);
  chk(hipMalloc(&c->cmp.tmp, std::max<size_t>(c->cmp.tmp_bytes, 256)));
  chk(dalloc(&c->nn_seed, B));
  chk(dalloc(&c->roll_q, 1));
  chk(dalloc(&c->roll_best, B));
  chk(dalloc(&c->roll_perm, (int64_t)B * CAND_K));
  chk(dalloc(&c->roll_pflag, 2 * (int64_t)B * CAND_K + (int64_t)(roll_order_scratch_bytes(B * CAND_K) / 4 + 64)));
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      c->n_cu = ncu;
  }
  chk(dalloc(&c->d_bbox, 4));
  chk(hipHostMalloc((void**)&c->h_bbox, sizeof(double) * 4, hipHostMallocDefault));
  chk(dalloc(&c->work_ctr, 64));
  if (rc == CLRRT_OK) chk(hipMemset(c->work_ctr, 0, 64 * sizeof(unsigned long long)));
  chk(hipHostMalloc((void**)&c->h_samples, sizeof(clrrt_sample) * B, hipHostMallocDefault));
  chk(hipHostMalloc((void**)&c->h_samples2, sizeof(clrrt_sample) * B, hipHostMallocDefault));
  chk(hipHostMalloc((void**)&c->h_totals, sizeof(int64_t) * 8, hipHostMallocDefault));
  chk(hipHostMalloc((void**)&c->h_int, sizeof(int) * 4, hipHostMallocDefault));
  if (rc != CLRRT_OK) {
    fprintf(stderr, "clrrt_create: %s\n", c->err.c_str());
    free_all(c);
    delete c;
    return rc;
  }
  *out = c;
  return CLRRT_OK;
}

void clrrt_destroy(clrrt_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  free_all(c);
  delete c;
}

int clrrt_set_stream(clrrt_ctx* c, void* s) {
  if (!c) return CLRRT_EINVAL;
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->own_stream) hipStreamDestroy(c->stream);
  if (s) {
    c->stream = (hipStream_t)s;
    c->own_stream = false;
  } else {
    HIPC(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  return CLRRT_OK;
}

int clrrt_set_rank(clrrt_ctx* c, int32_t rank) {
  if (!c || rank < 0) return CLRRT_EINVAL;
  c->rank = rank;
  return CLRRT_OK;
}

int clrrt_set_params(clrrt_ctx* c, const clrrt_params* p) {
  if (!c || !p) return CLRRT_EINVAL;
  pf_reset(c);
  DevParams d;
  derive(*p, d, c->n_obs);
  int rc = flush_replays(c);  // pending replays run under the parameters they were committed with
  if (rc != CLRRT_OK) return rc;
  if (c->slots && d.n_steps_max + 1 > c->slot_rows) {  // a smaller sim_dt needs longer rollout slots
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipFree(c->slots));
    c->slots = nullptr;
    c->slot_rows = 0;
    HIPC(c, dalloc(&c->slots, (size_t)2 * (d.n_steps_max + 1) * 10 * c->cap.max_batch * CAND_K));
    c->slot_rows = d.n_steps_max + 1;
  }
  c->params = *p;
  c->dp = d;
  return CLRRT_OK;
}

}  // extern "C"

// Uniform grid over the static obstacles for the rollout's collision cull (see ObsGrid).  The
// cell size starts near 1/1024 of the covered area and grows until the grid fits the LDS budget.
static const float kVehRad = 2.6220219f, kCullMargin = 0.05f;  // = VEH_RAD, CULL_MARGIN (kernels)
static int build_grid(clrrt_ctx* c, const std::vector<BakedObs>& b) {
  std::vector<int> stat, mov;
  for (int i = 0; i < (int)b.size(); i++) (b[i].moving ? mov : stat).push_back(i);
  const double tol = 0.05;
  double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
  std::vector<double> rr(b.size());
  for (int i : stat) {
    rr[i] = (double)(b[i].brad + kVehRad + kCullMargin);
    double cx = (double)(float)b[i].cx, cy = (double)(float)b[i].cy;
    x0 = std::min(x0, cx - rr[i] - tol); x1 = std::max(x1, cx + rr[i] + tol);
    y0 = std::min(y0, cy - rr[i] - tol); y1 = std::max(y1, cy + rr[i] + tol);
  }
  std::vector<uint32_t> start;
  std::vector<uint16_t> items;
  int gw = 0, gh = 0;
  float fx0 = 0, fy0 = 0, finv = 0;
  // dynamic LDS of the rollout kernels (36 B per obstacle + grid): the rollout kernels run one
  // 256-lane block per CU (256 VGPRs), so up to ~140 KiB of the CU's 160 KiB serve the grid
  // (launches raise hipFuncAttributeMaxDynamicSharedMemorySize accordingly)
#ifndef CLRRT_OBS_LDS_KB
#define CLRRT_OBS_LDS_KB 120
#endif
  const size_t lds_cap = CLRRT_OBS_LDS_KB * 1024;
  const size_t per_obs = 6 * 16 + 4;  // kernel LDS per obstacle: cull table + SAT geometry (roll_lds_bytes)
  const size_t lds_budget = b.size() * per_obs < lds_cap ? lds_cap - b.size() * per_obs : 0;
  if (!stat.empty() && std::isfinite(x0) && std::isfinite(x1) && std::isfinite(y0) && std::isfinite(y1) &&
      lds_budget >= 4 * 1024) {
    double W = x1 - x0, H = y1 - y0;
    double cs = std::max(0.25, std::sqrt(W * H / 8192.0));
    for (int attempt = 0; attempt < 40; attempt++, cs *= 1.25) {
      finv = (float)(1.0 / cs);
      fx0 = (float)x0; fy0 = (float)y0;
      // effective cell size seen by the kernel's float arithmetic
      double ecs = 1.0 / (double)finv;
      gw = (int)std::ceil((x1 - fx0) / ecs) + 1;
      gh = (int)std::ceil((y1 - fy0) / ecs) + 1;
      if ((int64_t)gw * gh > 16384) continue;
      start.assign((size_t)gw * gh + 1, 0);
      items.clear();
      for (int gy = 0; gy < gh; gy++)
        for (int gx = 0; gx < gw; gx++) {
          start[(size_t)gy * gw + gx] = (uint32_t)items.size();
          double rx0 = fx0 + gx * ecs - tol, rx1 = fx0 + (gx + 1) * ecs + tol;
          double ry0 = fy0 + gy * ecs - tol, ry1 = fy0 + (gy + 1) * ecs + tol;
          for (int i : stat) {
            double cx = (double)(float)b[i].cx, cy = (double)(float)b[i].cy;
            double dx = std::max(0.0, std::max(rx0 - cx, cx - rx1));
            double dy = std::max(0.0, std::max(ry0 - cy, cy - ry1));
            if (dx * dx + dy * dy > (rr[i] + tol) * (rr[i] + tol)) continue;
            // the kernel's second cull: the vehicle circle (VEH_RAD + margin) against the obstacle box.
            // A separating-axis gap between the cell and the (slackened) box bounds their distance from
            // below, so a gap beyond the circle radius proves no centre in the cell survives that cull.
            const double P = b[i].P, Q = b[i].Q, R = b[i].R, S = b[i].S;
            const double hh = std::sqrt(P * P + R * R), ww = std::sqrt(Q * Q + S * S);
            const double ux = hh > 0 ? P / hh : 1.0, uy = hh > 0 ? R / hh : 0.0;
            const double eh = hh * 1.0001 + 1e-3, ew = ww * 1.0001 + 1e-3;
            const double rcx = 0.5 * (rx0 + rx1), rcy = 0.5 * (ry0 + ry1);
            const double hx = 0.5 * (rx1 - rx0), hy = 0.5 * (ry1 - ry0);
            const double ex = std::fabs(ux) * eh + std::fabs(uy) * ew, ey = std::fabs(uy) * eh + std::fabs(ux) * ew;
            double gap = std::max(std::fabs(cx - rcx) - hx - ex, std::fabs(cy - rcy) - hy - ey);
            const double du = (cx - rcx) * ux + (cy - rcy) * uy, dv = -(cx - rcx) * uy + (cy - rcy) * ux;
            gap = std::max(gap, std::fabs(du) - eh - (hx * std::fabs(ux) + hy * std::fabs(uy)));
            gap = std::max(gap, std::fabs(dv) - ew - (hx * std::fabs(uy) + hy * std::fabs(ux)));
            if (gap > (double)(kVehRad + kCullMargin) + tol) continue;
            items.push_back((uint16_t)i);
          }
        }
      start[(size_t)gw * gh] = (uint32_t)items.size();
      size_t bytes = 4 * start.size() + 2 * (items.size() + mov.size());
      if (bytes <= lds_budget) break;
      gw = gh = 0;
    }
  }
  if (gw == 0) { start.clear(); items.clear(); }
  size_t need = 4 * start.size() + 2 * (items.size() + mov.size()) + 16;
  if (need > c->grid_bytes) {
    if (c->grid_buf) HIPC(c, hipFree(c->grid_buf));
    c->grid_buf = nullptr;
    c->grid_bytes = 0;
    HIPC(c, hipMalloc(&c->grid_buf, need));
    c->grid_bytes = need;
  }
  std::vector<uint8_t> host(need, 0);
  size_t o_items = 4 * start.size(), o_mov = o_items + 2 * items.size();
  if (!start.empty()) memcpy(host.data(), start.data(), 4 * start.size());
  if (!items.empty()) memcpy(host.data() + o_items, items.data(), 2 * items.size());
  for (size_t k = 0; k < mov.size(); k++) {
    uint16_t v = (uint16_t)mov[k];
    memcpy(host.data() + o_mov + 2 * k, &v, 2);
  }
  HIPC(c, hipMemcpyAsync(c->grid_buf, host.data(), need, hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  ObsGrid& g = c->grid;
  g.start = (const uint32_t*)c->grid_buf;
  g.items = (const uint16_t*)((const uint8_t*)c->grid_buf + o_items);
  g.mov = (const uint16_t*)((const uint8_t*)c->grid_buf + o_mov);
  g.gw = gw; g.gh = gh;
  g.nitems = (int)items.size();
  g.nmov = (int)mov.size();
  g.x0 = fx0; g.y0 = fy0; g.inv = finv;
  return CLRRT_OK;
}

// getOBBvector old_collisioncheck.cpp:14-16 + OBB::setVertices/setNorms :56-76 for one obstacle, hoisted
// out of the step loop: the float products (P, Q, R, S) always, the float SAT geometry of a static one.
static void bake_obstacle(const clrrt_obstacle& o, BakedObs& d) {
  memset(&d, 0, sizeof(d));
  float w = (float)(o.size_x / 2), h = (float)(o.size_y / 2), th = (float)o.theta;
  float cf, sf;
  ::sincosf(th, &sf, &cf);  // OBB::setVertices: float cos/sin of one argument -> glibc sincosf
  float hh = h / 2, ww = w / 2;
  d.P = cf * hh; d.Q = sf * ww; d.R = sf * hh; d.S = cf * ww;
  d.cx = o.cx; d.cy = o.cy; d.vlx = o.vx; d.vly = o.vy;
  d.moving = (o.vx != 0.0 || o.vy != 0.0);
  // static geometry: centre + 0*t (t >= 0) == centre + 0.0
  double px = o.cx + 0.0, py = o.cy + 0.0;
  d.vx[0] = (float)((px + (double)d.P) - (double)d.Q);
  d.vy[0] = (float)((py + (double)d.R) + (double)d.S);
  d.vx[1] = (float)((px + (double)d.P) - (double)(-d.Q));
  d.vy[1] = (float)((py + (double)d.R) + (double)(-d.S));
  d.vx[2] = (float)((px + (double)(-d.P)) - (double)(-d.Q));
  d.vy[2] = (float)((py + (double)(-d.R)) + (double)(-d.S));
  d.vx[3] = (float)((px + (double)(-d.P)) - (double)d.Q);
  d.vy[3] = (float)((py + (double)(-d.R)) + (double)d.S);
  for (int k = 0; k < 3; k++) {
    d.nx[k] = d.vy[k + 1] - d.vy[k];
    d.ny[k] = -(d.vx[k + 1] - d.vx[k]);
  }
  d.nx[3] = d.vy[0] - d.vy[3];
  d.ny[3] = -(d.vx[0] - d.vx[3]);
  d.bcx = (float)o.cx; d.bcy = (float)o.cy;
  d.brad = std::sqrt(hh * hh + ww * ww);
}

extern "C" {

// getOBBvector old_collisioncheck.cpp:6-22, evaluated once per query instead of once per step.
int clrrt_set_obstacles(clrrt_ctx* c, const clrrt_obstacle* o, int32_t m) {
  if (!c || m < 0 || (m > 0 && !o)) return CLRRT_EINVAL;
  if (m > c->cap.max_obstacles) return fail(c, CLRRT_ECAPACITY, "too many obstacles");
  if (m > 1400) return fail(c, CLRRT_ECAPACITY, "at most 1400 obstacles (rollout LDS cull table)");
  std::vector<BakedObs> b(m);
  for (int i = 0; i < m; i++) bake_obstacle(o[i], b[i]);
  HIPC(c, hipSetDevice(c->device));
  int frc = flush_replays(c);  // pending replays collide against the obstacles they were committed with
  if (frc != CLRRT_OK) return frc;
  if (m > 0) {
    HIPC(c, hipMemcpyAsync(c->obs, b.data(), sizeof(BakedObs) * m, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
  }
  c->n_obs = m;
  derive(c->params, c->dp, m);
  return build_grid(c, b);
}

int clrrt_tree_init(clrrt_ctx* c, const double root_state[10]) {
  if (!c || !root_state) return CLRRT_EINVAL;
  pf_reset(c);
  c->rep_n = 0;  // replays pending for the old tree's rows: the tree is replaced
  HIPC(c, hipSetDevice(c->device));
  double* d_state = nullptr;
  HIPC(c, hipMalloc((void**)&d_state, 10 * sizeof(double)));
  hipError_t e = hipMemcpyAsync(d_state, root_state, 10 * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = launch_init_root(c->stream, d_state, c->tree, c->nn, c->arena);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(d_state);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("tree_init: ") + hipGetErrorString(e));
  c->n_nodes = 1;
  c->n_rows = 1;
  bbox_reset(c);
  if (std::isfinite(root_state[0]) && std::isfinite(root_state[1]))
    bbox_add(c, root_state[0], root_state[1], root_state[0], root_state[1]);
  return CLRRT_OK;
}

int clrrt_tree_load(clrrt_ctx* c, const clrrt_node* nodes, int64_t n) {
  if (!c || n < 0 || (n > 0 && !nodes)) return CLRRT_EINVAL;
  pf_reset(c);
  c->rep_n = 0;  // the tree is replaced
  if (n > c->cap.max_nodes) return fail(c, CLRRT_ECAPACITY, "tree_load: too many nodes");
  HIPC(c, hipSetDevice(c->device));
  if (n > 0) {
    clrrt_node* tmp = nullptr;
    HIPC(c, hipMalloc((void**)&tmp, sizeof(clrrt_node) * n));
    hipError_t e = hipMemcpyAsync(tmp, nodes, sizeof(clrrt_node) * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_append(c->stream, tmp, (int)n, 0, c->tree, c->nn);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(tmp);
    if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("tree_load: ") + hipGetErrorString(e));
  }
  c->n_nodes = n;
  c->n_rows = 0;
  bbox_reset(c);
  for (int64_t i = 0; i < n; i++)
    if (std::isfinite(nodes[i].state[0]) && std::isfinite(nodes[i].state[1]))
      bbox_add(c, nodes[i].state[0], nodes[i].state[1], nodes[i].state[0], nodes[i].state[1]);
  return CLRRT_OK;
}

int clrrt_tree_truncate(clrrt_ctx* c, int64_t n) {
  if (!c || n < 1 || n > c->n_nodes) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  int rc = flush_replays(c);  // pending rows of committed nodes land first (the arena stays consistent)
  if (rc != CLRRT_OK) return rc;
  pf_reset(c);  // prefetched lists and kept walk sort results describe the longer tree
  if (n == c->n_nodes) return CLRRT_OK;
  clrrt_node h;
  HIPC(c, hipMemcpyAsync(&h, c->tree + n, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  c->n_nodes = n;
  if (h.row_offset >= 0 && h.row_offset <= c->n_rows) c->n_rows = h.row_offset;  // rows are appended in node order
  return CLRRT_OK;  // (the tree's box stays a superset: a valid search frame)
}

int clrrt_exact_stats(clrrt_ctx* c, int64_t out[10]) {
  if (!c || !out) return CLRRT_EINVAL;
  for (int i = 0; i < 10; i++) out[i] = c->ex_stats[i];
  return CLRRT_OK;
}

int clrrt_iteration_log(clrrt_ctx* c, int32_t on) {
  if (!c) return CLRRT_EINVAL;
  c->iter_log = on != 0;
  c->iters.clear();
  return CLRRT_OK;
}

int clrrt_iteration_records(clrrt_ctx* c, int64_t first, int64_t count, clrrt_iteration* out, int64_t* n_total) {
  if (!c || first < 0 || count < 0 || first + count > (int64_t)c->iters.size() || (count > 0 && !out))
    return CLRRT_EINVAL;
  if (n_total) *n_total = (int64_t)c->iters.size();
  for (int64_t i = 0; i < count; i++) out[i] = c->iters[first + i];
  return CLRRT_OK;
}

int clrrt_tree_size(clrrt_ctx* c, int64_t* n_nodes, int64_t* n_rows) {
  if (!c) return CLRRT_EINVAL;
  if (n_nodes) *n_nodes = c->n_nodes;
  if (n_rows) *n_rows = c->n_rows;
  return CLRRT_OK;
}

int clrrt_tree_download(clrrt_ctx* c, int64_t first, int64_t count, clrrt_node* out) {
  if (!c || first < 0 || count < 0 || first + count > c->n_nodes || (count > 0 && !out)) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (count == 0) return CLRRT_OK;
  HIPC(c, hipMemcpyAsync(out, c->tree + first, sizeof(clrrt_node) * count, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_tree_rows(clrrt_ctx* c, int64_t row_offset, int64_t nrows, double* out) {
  if (!c || row_offset < 0 || nrows < 0 || row_offset + nrows > c->n_rows || (nrows > 0 && !out))
    return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (nrows == 0) return CLRRT_OK;
  int rc = flush_replays(c);
  if (rc != CLRRT_OK) return rc;
  HIPC(c, hipMemcpyAsync(out, c->arena + row_offset * 10, sizeof(double) * 10 * nrows, hipMemcpyDeviceToHost,
                         c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_extract_best_path(clrrt_ctx* c, int32_t* path, int32_t cap, int32_t* n_path, float* best_cost,
                            int64_t* n_goal) {
  if (!c || !n_path || cap < 0 || (cap > 0 && !path)) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  *n_path = 0;
  if (best_cost) *best_cost = HUGE_VALF;
  if (n_goal) *n_goal = 0;
  const int64_t n = c->n_nodes;
  if (n == 0) return CLRRT_OK;
  if (!c->goal_recs) {
    HIPC(c, hipMalloc(&c->goal_recs, sizeof(GoalRec) * c->cap.max_nodes));
    HIPC(c, hipMalloc(&c->bp_path, sizeof(int) * (c->cap.max_nodes + 2)));
  }
  int* d_cnt = c->bp_path + c->cap.max_nodes;
  HIPC(c, launch_goal_gather(c->stream, c->tree, n, c->goal_recs, d_cnt));
  int cnt = 0;
  HIPC(c, hipMemcpyAsync(&cnt, d_cnt, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (n_goal) *n_goal = cnt;
  if (cnt == 0) return CLRRT_OK;  // "No feasible path found" (rrtplanner.cpp:361-366)
  std::vector<GoalRec> g(cnt);
  HIPC(c, hipMemcpyAsync(g.data(), c->goal_recs, sizeof(GoalRec) * cnt, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  // pair_vector in tree order (rrtplanner.cpp:330-335), then the reference's sort verbatim in
  // semantics: std::sort on (id, double(costS)) pairs by .second -- equal costs keep whatever
  // order introsort leaves them in, which depends on the input order, hence the id pass first.
  std::sort(g.begin(), g.end(), [](const GoalRec& a, const GoalRec& b) { return a.id < b.id; });
  std::vector<std::pair<int, double>> pv(cnt);
  for (int i = 0; i < cnt; i++) pv[i] = std::make_pair((int)g[i].id, (double)g[i].cost);
  std::sort(pv.begin(), pv.end(),
            [](const std::pair<int, double>& a, const std::pair<int, double>& b) { return a.second < b.second; });
  const int best = pv.front().first;
  if (best_cost) *best_cost = (float)pv.front().second;
  HIPC(c, launch_backtrack(c->stream, c->tree, n, best, (int)c->cap.max_nodes, c->bp_path, d_cnt + 1));
  int len = 0;
  HIPC(c, hipMemcpyAsync(&len, d_cnt + 1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (len <= 0) return fail(c, CLRRT_EINVAL, "extract_best_path: parent chain does not reach the root");
  const int m = std::min<int>(len, cap);
  if (m > 0) {
    std::vector<int> chain(len);  // goal -> root
    HIPC(c, hipMemcpyAsync(chain.data(), c->bp_path, sizeof(int) * len, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < m; i++) path[i] = chain[len - 1 - i];
  }
  *n_path = len;
  return CLRRT_OK;
}

// ------------------------------------------------------------------ committed path / re-init
// Grow the path buffers to hold n nodes and nrows rows (contents not preserved).
static int path_reserve(clrrt_ctx* c, int n, int64_t nrows) {
  if (n > c->path_cap) {
    const int cap = std::max(n, 2 * c->path_cap);
    for (void* p : {(void*)c->path_nodes, (void*)c->ri_int, (void*)c->ri_off, (void*)c->ri_cost})
      if (p) hipFree(p);
    c->path_nodes = nullptr; c->ri_int = nullptr; c->ri_off = nullptr; c->ri_cost = nullptr;
    c->path_cap = 0;
    HIPC(c, hipMalloc((void**)&c->path_nodes, sizeof(clrrt_node) * cap));
    HIPC(c, hipMalloc((void**)&c->ri_int, sizeof(int) * (3 * (size_t)cap)));
    HIPC(c, hipMalloc((void**)&c->ri_off, sizeof(int64_t) * ((size_t)cap + 3)));
    HIPC(c, hipMalloc((void**)&c->ri_cost, sizeof(float) * cap));
    c->path_cap = cap;
  }
  if (nrows > c->path_rows_cap) {
    const int64_t cap = std::max<int64_t>(nrows, 2 * c->path_rows_cap);
    if (c->path_rows) hipFree(c->path_rows);
    if (c->ri_terms) hipFree(c->ri_terms);
    c->path_rows = nullptr; c->ri_terms = nullptr;
    c->path_rows_cap = 0;
    HIPC(c, hipMalloc((void**)&c->path_rows, sizeof(double) * 10 * cap));
    HIPC(c, hipMalloc((void**)&c->ri_terms, sizeof(double) * 2 * cap));
    c->path_rows_cap = cap;
  }
  return CLRRT_OK;
}

int clrrt_path_commit(clrrt_ctx* c, const int32_t* ids, int32_t n, int32_t* n_remote) {
  if (!c || n < 0 || (n > 0 && !ids)) return CLRRT_EINVAL;
  for (int i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= c->n_nodes) return fail(c, CLRRT_EINVAL, "path_commit: node id outside the tree");
  HIPC(c, hipSetDevice(c->device));
  int frc = flush_replays(c);  // the path's rows are copied from the arena
  if (frc != CLRRT_OK) return frc;
  if (n_remote) *n_remote = 0;
  c->path_n = 0;
  c->path_nrows = 0;
  if (n == 0) return CLRRT_OK;
  int rc = path_reserve(c, n, 1);
  if (rc != CLRRT_OK) return rc;
  // headers of the path nodes, then path-local row offsets on the host
  HIPC(c, hipMemcpyAsync(c->ri_int, ids, sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
  HIPC(c, launch_gather_nodes(c->stream, c->tree, c->ri_int, n, c->path_nodes));
  std::vector<clrrt_node> h(n);
  HIPC(c, hipMemcpyAsync(h.data(), c->path_nodes, sizeof(clrrt_node) * n, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  std::vector<int64_t> src(n);
  int64_t rows = 0;
  int remote = 0;
  for (int i = 0; i < n; i++) {
    if (h[i].nrows < 1) return fail(c, CLRRT_EINVAL, "path_commit: node without trajectory rows");
    src[i] = h[i].row_offset;
    h[i].row_offset = rows;
    rows += h[i].nrows;
    if (h[i].owner != c->rank) remote++;
  }
  rc = path_reserve(c, n, rows);
  if (rc != CLRRT_OK) return rc;
  HIPC(c, hipMemcpyAsync(c->path_nodes, h.data(), sizeof(clrrt_node) * n, hipMemcpyHostToDevice, c->stream));
  for (int i = 0; i < n; i++) {
    double* dst = c->path_rows + h[i].row_offset * 10;
    const size_t bytes = sizeof(double) * 10 * h[i].nrows;
    if (h[i].owner == c->rank) {
      HIPC(c, hipMemcpyAsync(dst, c->arena + src[i] * 10, bytes, hipMemcpyDeviceToDevice, c->stream));
    } else {
      HIPC(c, hipMemsetAsync(dst, 0, bytes, c->stream));
    }
  }
  HIPC(c, hipStreamSynchronize(c->stream));
  c->path_n = n;
  c->path_nrows = rows;
  if (n_remote) *n_remote = remote;
  return CLRRT_OK;
}

int clrrt_path_load(clrrt_ctx* c, const clrrt_node* nodes, int32_t n, const double* rows, int64_t n_rows) {
  if (!c || n < 0 || n_rows < 0 || (n > 0 && (!nodes || !rows))) return CLRRT_EINVAL;
  for (int i = 0; i < n; i++)
    if (nodes[i].nrows < 1 || nodes[i].row_offset < 0 || nodes[i].row_offset + nodes[i].nrows > n_rows)
      return fail(c, CLRRT_EINVAL, "path_load: node rows outside the row buffer");
  HIPC(c, hipSetDevice(c->device));
  int rc = path_reserve(c, n, n_rows);
  if (rc != CLRRT_OK) return rc;
  if (n > 0) {
    HIPC(c, hipMemcpyAsync(c->path_nodes, nodes, sizeof(clrrt_node) * n, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->path_rows, rows, sizeof(double) * 10 * n_rows, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
  }
  c->path_n = n;
  c->path_nrows = n > 0 ? n_rows : 0;
  return CLRRT_OK;
}

int clrrt_path_size(clrrt_ctx* c, int32_t* n, int64_t* n_rows) {
  if (!c) return CLRRT_EINVAL;
  if (n) *n = c->path_n;
  if (n_rows) *n_rows = c->path_nrows;
  return CLRRT_OK;
}

int clrrt_path_download(clrrt_ctx* c, clrrt_node* nodes, double* rows) {
  if (!c) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (c->path_n > 0 && nodes)
    HIPC(c, hipMemcpyAsync(nodes, c->path_nodes, sizeof(clrrt_node) * c->path_n, hipMemcpyDeviceToHost, c->stream));
  if (c->path_nrows > 0 && rows)
    HIPC(c, hipMemcpyAsync(rows, c->path_rows, sizeof(double) * 10 * c->path_nrows, hipMemcpyDeviceToHost,
                           c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_path_transform(clrrt_ctx* c, int32_t dir, const double pose[3]) {
  if (!c || !pose || (dir != CLRRT_WORLD_TO_CAR && dir != CLRRT_CAR_TO_WORLD)) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (c->path_n == 0) return CLRRT_OK;
  HIPC(c, launch_path_transform(c->stream, c->path_nodes, c->path_n, c->path_rows, c->path_nrows,
                                dir == CLRRT_CAR_TO_WORLD, pose));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_tree_init_from_path(clrrt_ctx* c, const double car_state[6], int32_t* outcome) {
  if (!c || !car_state) return CLRRT_EINVAL;
  pf_reset(c);
  c->rep_n = 0;  // the tree is replaced by the committed path's survivors (their rows: the path buffer)
  HIPC(c, hipSetDevice(c->device));
  int rc = path_reserve(c, std::max(1, c->path_n), std::max<int64_t>(1, c->path_nrows));
  if (rc != CLRRT_OK) return rc;
  if (c->path_n > c->cap.max_nodes || c->path_nrows > c->cap.max_rows)
    return fail(c, CLRRT_ECAPACITY, "tree_init_from_path: committed path exceeds the tree capacity");
  ReinitArgs a;
  a.p = c->dp;
  a.obs = c->obs;
  a.pn = c->path_nodes;
  a.n = c->path_n;
  a.prow = c->path_rows;
  for (int k = 0; k < 10; k++) a.car[k] = k < 6 ? car_state[k] : 0.0;
  a.tree = c->tree;
  a.nn = c->nn;
  a.arena = c->arena;
  a.kidx = c->ri_int;
  a.koff = c->ri_off;
  a.terms = c->ri_terms;
  a.costs = c->ri_cost;
  a.out = c->ri_off + c->path_cap;
  a.rank = c->rank;
  a.max_nodes = c->cap.max_nodes;
  a.max_rows = c->cap.max_rows;
  HIPC(c, launch_tree_reinit(c->stream, a));
  int64_t out[3];
  HIPC(c, hipMemcpyAsync(out, a.out, sizeof(out), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (out[0] < 0) return fail(c, CLRRT_ECAPACITY, "tree_init_from_path: tree capacity");
  c->n_nodes = out[1];
  c->n_rows = out[2];
  bbox_reset(c);
  HIPC(c, launch_bbox(c->stream, c->tree, nullptr, (int)c->n_nodes, c->d_bbox));
  HIPC(c, hipMemcpyAsync(c->h_bbox, c->d_bbox, sizeof(double) * 4, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  bbox_add(c, c->h_bbox[0], c->h_bbox[1], c->h_bbox[2], c->h_bbox[3]);
  if (outcome) *outcome = (int32_t)out[0];
  return CLRRT_OK;
}

int clrrt_path_mpc_message(clrrt_ctx* c, int32_t filtered, double* out, int32_t cap, int32_t* n_points) {
  if (!c || !n_points || cap < 0 || (cap > 0 && !out)) return CLRRT_EINVAL;
  *n_points = 0;
  if (c->path_n == 0) return CLRRT_OK;
  std::vector<clrrt_node> h(c->path_n);
  std::vector<double> rows(10 * c->path_nrows);
  int rc = clrrt_path_download(c, h.data(), rows.data());
  if (rc != CLRRT_OK) return rc;
  // generateMPCmessage: rows 1 .. nrows-1 of every segment
  std::vector<std::array<double, 8>> msg;
  for (const clrrt_node& nd : h)
    for (int i = 1; i < nd.nrows; i++) {
      const double* r = &rows[(nd.row_offset + i) * 10];
      msg.push_back({r[0], r[1], r[2], r[3], r[4], r[5], r[8], r[9]});
    }
  if (filtered && !msg.empty()) {  // filterMPCmessage: keep index i when the distance since the last kept is 0
    std::vector<std::array<double, 8>> f;
    const double interval = 5;
    double d = 0;
    for (size_t i = 1; i != msg.size(); i++) {
      if (d == 0) {
        std::array<double, 8> p = msg[i];
        p[3] = NAN;
        f.push_back(p);
      }
      const double dx = msg[i][0] - msg[i - 1][0], dy = msg[i][1] - msg[i - 1][1];
      d += sqrt(dx * dx + dy * dy);
      if (d >= interval) d = 0;
    }
    msg.swap(f);
  }
  *n_points = (int32_t)msg.size();
  for (int i = 0; i < (int)msg.size() && i < cap; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = msg[i][k];
  return CLRRT_OK;
}

int clrrt_get_counters(clrrt_ctx* c, clrrt_counters* out) {
  if (!c || !out) return CLRRT_EINVAL;
  *out = c->counters;
  return CLRRT_OK;
}

int clrrt_reset_counters(clrrt_ctx* c) {
  if (!c) return CLRRT_EINVAL;
  memset(&c->counters, 0, sizeof(c->counters));
  c->nn_bf_keys = c->nn_samples = c->nn_super_bounds = 0;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemsetAsync(c->work_ctr, 0, 64 * sizeof(unsigned long long), c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_debug_counters(clrrt_ctx* c, int64_t out[64]) {
  if (!c || !out) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipStreamSynchronize(c->stream));
  unsigned long long h[64];
  HIPC(c, hipMemcpy(h, c->work_ctr, sizeof(h), hipMemcpyDeviceToHost));
  for (int i = 0; i < 64; i++) out[i] = (int64_t)h[i];
  return CLRRT_OK;
}

int clrrt_work_counters(clrrt_ctx* c, int64_t out[3]) {
  if (!c || !out) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  unsigned long long h[4];
  HIPC(c, hipMemcpyAsync(h, c->work_ctr, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < 3; i++) out[i] = (int64_t)h[i];
  return CLRRT_OK;
}

int clrrt_search_work(clrrt_ctx* c, int64_t out[4]) {
  if (!c || !out) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->side) HIPC(c, hipStreamSynchronize(c->side));
  unsigned long long h[19];
  HIPC(c, hipMemcpy(h, c->work_ctr + 8, sizeof(h), hipMemcpyDeviceToHost));
  out[0] = c->nn_bf_keys;
  out[1] = c->nn_samples;
  out[2] = (int64_t)h[11];
  out[3] = (int64_t)h[13];
  return CLRRT_OK;
}

int clrrt_search_work_ex(clrrt_ctx* c, int64_t out[8]) {
  if (!c || !out) return CLRRT_EINVAL;
  int64_t w[4];
  const int rc = clrrt_search_work(c, w);
  if (rc != CLRRT_OK) return rc;
  unsigned long long h[19];
  HIPC(c, hipMemcpy(h, c->work_ctr + 8, sizeof(h), hipMemcpyDeviceToHost));
  for (int i = 0; i < 4; i++) out[i] = w[i];
  out[4] = c->nn_super_bounds;
  out[5] = (int64_t)h[10];  // super-tile visits (32 tile bounds each)
  out[6] = (int64_t)h[12];  // records past the prefilter (queued for stage 1 / 2)
  out[7] = 0;
  return CLRRT_OK;
}

int clrrt_nn_stats(clrrt_ctx* c, int64_t out[19]) {
  if (!c || !out) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipStreamSynchronize(c->stream));
  unsigned long long h[19];
  HIPC(c, hipMemcpy(h, c->work_ctr + 8, sizeof(h), hipMemcpyDeviceToHost));
  for (int i = 0; i < 19; i++) out[i] = (int64_t)h[i];
  out[4] &= 0xffffffff;
  return CLRRT_OK;
}

int clrrt_set_option(clrrt_ctx* c, const char* key, int64_t value) {
  if (!c || !key) return CLRRT_EINVAL;
  const std::string k(key);
  if (k == "roll_persistent") c->roll_persistent = value != 0;
  else if (k == "nn_walk_min" && value >= 0) c->nnw_min_nodes = value;
  else if (k == "nn_walk_stateless") c->nnw_stateless = value != 0;
  else if (k == "nn_walk_budget_tiles" && value >= 0 && value < INT_MAX) {
    c->nnw_bud_tiles = (int)value;
    c->nnw_bud_tiles_set = true;
  }
  else if (k == "nn_walk_budget_keys" && value >= 0 && value < INT_MAX) c->nnw_bud_ex = (int)value;
  else if (k == "nn_walk_half_max" && value >= 0 && value < INT_MAX) c->nnw_half_max = (int)value;
  else if (k == "nn_walk_hscale" && value >= 1 && value <= 10000) {  // index order: scheduling only
    c->nnw_hscale = (int)value;
    c->nnw_built.n = -1;
    c->nnw.sorted_n = c->nnw_alt.sorted_n = c->nnw3.sorted_n = -1;
  }
  else if (k == "nn_walk_lpt") c->nnw_lpt = value != 0;  // scheduling only: same lists
  else if (k == "nn_walk_index" && value >= 0 && value <= 5) {
    c->nnw_index = (int)value;
    c->nnw_built.n = -1;  // the kept index and sort results have the old order
    c->nnw.sorted_n = c->nnw_alt.sorted_n = c->nnw3.sorted_n = -1;
  }
  else if (k == "nn_walk_lds_floor" && value >= 0 && value <= 65536) c->nnw_lds_floor = (int)value;
  else if (k == "nn_walk_waves" && value >= -1 && value <= 1 << 20) c->nnw_waves = (int)value;
  else if (k == "nn_walk_chunks" && value >= 1 && value <= kWalkMaxChunks) c->nnw_chunks = (int)value;
  else if (k == "nn_walk_max_over" && value >= 1 && value <= kWalkMaxOver) {
    c->nnw_max_over = (int)value;
    c->nnw_max_over_set = true;
  }
  else if (k == "nn_walk_double") c->nnw_double = value != 0;
  else if (k == "nn_lag" && (value == 0 || value == 1 || value == 2)) c->nn_lag = (int)value;
  else if (k == "nn_split_delta") c->nn_split_delta = value != 0 ? 1 : 0;  // scheduling only: same lists
  else if (k == "nn_delta_early") c->nn_delta_early = value != 0 ? 1 : 0;  // scheduling only: same lists
  else if (k == "nn_lane_order") c->nn_lane_order = value != 0 ? 1 : 0;  // scheduling only: same lists
  else if (k == "nn_debug" && value >= 0) c->nn_debug = (int)value;  // diagnostics: changes results
  else if (k == "fail_at_round" && value >= 0 && value < INT_MAX) c->fail_at_round = (int)value;  // fault injection
  else if (k == "fail_after_exchange" && value >= 0 && value < INT_MAX) c->fail_after_exchange = (int)value;
  else if (k == "roll_blocks" && value >= 0 && value < (1 << 20)) c->roll_blocks = (int)value;
  else if (k == "nn_pipeline") c->nn_pipeline = value != 0;
  else if (k == "roll_priority") c->roll_priority = value != 0;
  else if (k == "roll_coop") c->roll_coop = value != 0;
  else if (k == "roll_spread") c->roll_spread = value != 0;
  else if (k == "roll_lanes") c->roll_lanes = (int)std::max<int64_t>(0, std::min<int64_t>(64, value));
  else if (k == "nn_exact_fused") c->nn_exact_fused = value != 0;
  else if (k == "rows_deferred") {
    int rc = flush_replays(c);
    if (rc != CLRRT_OK) return rc;
    c->rows_deferred = value != 0;
  }
  else if (k == "exact_min_width" && value >= 1 && value <= 1 << 20) c->exact_min_width = (int)value;
  else if (k == "exact_fixup") c->exact_fixup = value != 0;
  else if (k == "exact_fixup_cap" && value >= 0 && value < INT_MAX) c->exact_fix_cap = (int)value;
  else if (k == "defer_steps" && value >= 0 && value <= 1 << 20) {
    // BATCH rounds with deferred samples (changes the BATCH tree: samples whose rollouts run past T steps
    // per launch commit in a later round, by a deterministic rule the oracle restates); 0 = off
    if (value > 0 && value < 8) return fail(c, CLRRT_EINVAL, "defer_steps must be 0 or >= 8");
    c->def.T = (int)value;
  }
  else if (k == "cu_split" && value >= 0 && value <= 7) {
    HIPC(c, hipStreamSynchronize(c->side));
    if (c->roll_st) HIPC(c, hipStreamSynchronize(c->roll_st));
    HIPC(c, hipStreamDestroy(c->side));
    c->side = nullptr;
    if (c->roll_st) HIPC(c, hipStreamDestroy(c->roll_st));
    c->roll_st = nullptr;
    c->cu_split = (int)value;
    c->stream_prio_applied = 0;  // the lag-2 streams are re-made for the new split
    if (value == 0) {
      HIPC(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    } else {
      // CU i goes to the rollouts when i mod 8 < k: k/8 of every run of 8 CU indices
      const int nw = (c->n_cu + 31) / 32;
      std::vector<uint32_t> mr(nw, 0u), ms(nw, 0u);
      for (int i = 0; i < c->n_cu; i++) ((i % 8) < value ? mr : ms)[i / 32] |= 1u << (i % 32);
      HIPC(c, hipExtStreamCreateWithCUMask(&c->roll_st, (uint32_t)nw, mr.data()));
      HIPC(c, hipExtStreamCreateWithCUMask(&c->side, (uint32_t)nw, ms.data()));
      if (!c->ev_rs0) HIPC(c, hipEventCreateWithFlags(&c->ev_rs0, hipEventDisableTiming));
      if (!c->ev_rs1) HIPC(c, hipEventCreateWithFlags(&c->ev_rs1, hipEventDisableTiming));
    }
  }
  else if (k == "stream_prio") c->stream_prio = value != 0;
  else if (k == "walk_cu_reserve" && value >= 0 && value <= 7) c->walk_cu_reserve = (int)value;
  else if (k == "side_priority") {  // -1: lower than the main stream's, 0: equal, 1: higher
    int lo = 0, hi = 0;
    HIPC(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPC(c, hipStreamSynchronize(c->side));
    HIPC(c, hipStreamDestroy(c->side));
    const int pr = value > 0 ? hi : value < 0 ? lo : 0;
    HIPC(c, hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, pr));
    c->side_prio_set = true;
    c->stream_prio_applied = 0;
    if (value < 0 && c->own_stream) {  // and the main stream gets the highest priority
      HIPC(c, hipStreamSynchronize(c->stream));
      HIPC(c, hipStreamDestroy(c->stream));
      HIPC(c, hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
    }
  }
  else return fail(c, CLRRT_EINVAL, "unknown option or value: " + k);
  return CLRRT_OK;
}

int clrrt_enable_timing(clrrt_ctx* c, int32_t on) {
  if (!c) return CLRRT_EINVAL;
  drain_timers(c);
  c->timing = on != 0;
  for (int i = 0; i < clrrt_ctx::kKtClasses; i++) { c->kt_ms[i] = 0; c->kt_n[i] = 0; }
  return CLRRT_OK;
}

int clrrt_kernel_time(clrrt_ctx* c, int32_t which, double* ms, int64_t* launches) {
  if (!c || which < 0 || which >= clrrt_ctx::kKtClasses) return CLRRT_EINVAL;
  drain_timers(c);
  if (ms) *ms = c->kt_ms[which];
  if (launches) *launches = c->kt_n[which];
  return CLRRT_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------ rounds
static RollArgs roll_args(clrrt_ctx* c, int njobs) {
  RollArgs a;
  memset(&a, 0, sizeof(a));
  a.p = c->dp;
  a.tree = c->tree;
  a.samples = c->d_samples;
  a.cand = c->cand;
  a.jobs = c->jobs;
  a.obs = c->obs;
  a.arena = c->arena;
  a.ctr = c->work_ctr;
  a.grid = c->grid;
  a.njobs = njobs;
  return a;
}

static int ensure_sort_scratch(clrrt_ctx* c, int64_t entries) {
  if (entries <= c->sort_cap) return CLRRT_OK;
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->sort_scratch) HIPC(c, hipFree(c->sort_scratch));
  c->sort_scratch = nullptr;
  c->sort_cap = 0;
  int64_t want = std::max<int64_t>(entries, 1 << 20);
  HIPC(c, hipMalloc((void**)&c->sort_scratch, sizeof(KeyId) * want));
  c->sort_cap = want;
  return CLRRT_OK;
}

// One walk-search buffer set, sized for the context's capacity.
static int alloc_walk(clrrt_ctx* c, WalkBufs& w) {
  if (w.P) return CLRRT_OK;
  const int64_t M = std::max<int64_t>(c->cap.max_nodes, c->cap.max_batch);
  const int64_t Mp = c->cap.max_nodes + 1024;
  HIPC(c, dalloc(&w.sorder, c->cap.max_batch));
  HIPC(c, dalloc(&w.keys, 2 * M));
  HIPC(c, dalloc(&w.keys2, 2 * M));
  HIPC(c, dalloc(&w.vals, std::max<int64_t>(M, Mp)));  // also the run markers of the padded records
  HIPC(c, dalloc(&w.vals2, M));
  w.tmp_bytes = walk_sort_bytes((int)M);
  HIPC(c, hipMalloc(&w.tmp, std::max<size_t>(w.tmp_bytes, 256)));
  HIPC(c, dalloc(&w.Q, Mp));
  HIPC(c, dalloc(&w.CE, Mp));
  HIPC(c, dalloc(&w.ID, Mp));
  HIPC(c, dalloc(&w.HEAD, Mp));
  HIPC(c, dalloc(&w.trun, walk_tile_count(c->cap.max_nodes) + 1));
  // one record per tile / super-tile of the padded index (launch_nn_walk_build)
  HIPC(c, dalloc(&w.tiles, walk_tile_count(c->cap.max_nodes) + 1));
  HIPC(c, dalloc(&w.supers, walk_super_count(c->cap.max_nodes) + 1));
  HIPC(c, dalloc(&w.ovf_n, 1));
  HIPC(c, dalloc(&w.ovf, kWalkMaxOver));
  HIPC(c, dalloc(&w.wctr, 8));
  HIPC(c, dalloc(&w.pk, (int64_t)kWalkMaxOver * kWalkMaxChunks * 11));
  HIPC(c, dalloc(&w.pi, (int64_t)kWalkMaxOver * kWalkMaxChunks * 11));
  HIPC(c, dalloc(&w.skeys, Mp));
  HIPC(c, dalloc(&w.sids, Mp));
  w.sorted_n = -1;
  w.cap_nodes = c->cap.max_nodes;
  w.cap_batch = (int)c->cap.max_batch;
  HIPC(c, dalloc(&w.P, Mp));  // last: marks the set complete
  return CLRRT_OK;
}

// Walk-search configuration of a set (+ its buffers on first use).
static int ensure_walk_set(clrrt_ctx* c, WalkBufs& w) {
  w.bud_tiles = c->nnw_bud_tiles_set || c->nnw_bud_tiles == 0
                    ? c->nnw_bud_tiles
                    : (int)std::max<int64_t>(c->nnw_bud_tiles, c->n_nodes >> 11);
  // the exact-key budget grows with the tree (denser trees: more near-tied keys per sample; the cfg3
  // sweeps: 4096 best at <= 1.6 M nodes, 8192 at 4.7 M, where 4096 overflows more samples than there
  // are records)
  w.bud_ex = c->nnw_bud_ex > 0 ? (int)std::max<int64_t>(c->nnw_bud_ex, c->n_nodes >> 9) : 0;
  w.max_over = c->nnw_max_over_set || c->n_nodes < (6 << 20) ? c->nnw_max_over : kWalkMaxOver;
  w.nch = c->nnw_chunks;
  w.half_max = c->nnw_half_max;
  w.index_kind = c->nnw_index;
  w.hscale_pct = c->nnw_hscale;
  w.lpt = c->nnw_lpt;
  w.lds_floor = c->nnw_lds_floor;
  w.waves = c->nnw_waves < 0 ? 9 * c->n_cu : c->nnw_waves;
  // the default grid serves batches of >= 4x its waves (cfg2's 4096-sample rounds run 4% faster with one
  // wave per sample: 1.237 vs 1.188 M nodes/s)
  w.waves_min_batch = c->nnw_waves < 0 ? 4 * w.waves : 0;
  return alloc_walk(c, w);
}
static int ensure_walk(clrrt_ctx* c) { return ensure_walk_set(c, c->nnw); }

// Search region (the sampling region and the tree's box) and the float frame of the searches.
struct NnSetup {
  NnFrame fr;
  double x0, y0, x1, y1;
  bool region_ok;
};
static NnSetup nn_setup(clrrt_ctx* c) {
  NnSetup su;
  double& x0 = su.x0; double& y0 = su.y0; double& x1 = su.x1; double& y1 = su.y1;
  sample_region(c->params, x0, y0, x1, y1);
  if (c->bbox[0] <= c->bbox[2]) {  // grid covers the samples and every finite node: no overflow
    x0 = std::min(x0, c->bbox[0] - 1.0); y0 = std::min(y0, c->bbox[1] - 1.0);
    x1 = std::max(x1, c->bbox[2] + 1.0); y1 = std::max(y1, c->bbox[3] + 1.0);
  }
  // float frame of the brute-force prune: |coordinate - origin| <= E for every sample and finite node
  // (samples of this round lie in the sample region, nodes in the tree's box); each float rounding
  // of a coordinate difference errs by <= 2^-24 E, a squared distance difference by a few of them
  NnFrame fr;
  fr.debug = c->nn_debug;
  fr.ox = 0.5 * (x0 + x1);
  fr.oy = 0.5 * (y0 + y1);
  {
    const double E = std::max(x1 - x0, y1 - y0) + 1.0;
    const double d = 16.0 * std::ldexp(E, -24) + 1e-5;
    fr.delta = std::isfinite(d) ? (float)d : HUGE_VALF;
  }
  su.fr = fr;
  const double W = x1 - x0, H = y1 - y0;
  su.region_ok = std::isfinite(W * H) && W * H > 0;
  return su;
}

// The walk search serves the tree as it is now (run_nn's choice).
static bool walk_serves(clrrt_ctx* c, const NnSetup& su) {
  return c->n_nodes >= c->nnw_min_nodes && su.region_ok;
}

// Any tree change other than clrrt_round_commit invalidates a prefetched search.
static void pf_reset(clrrt_ctx* c) {
  if (c->pf_state != 0 && c->side) hipStreamSynchronize(c->side);
  c->pf_state = 0;
  c->pf_next.clear();
  c->nnw_built.n = -1;
  c->nnw.sorted_n = -1;  // the kept sort results describe the old tree
  c->nnw_alt.sorted_n = -1;
  c->nnw3.sorted_n = -1;
}

// Launches the walk search of samples h2[0..n2) (host, pinned) over the current tree on the side
// stream into the *2 buffers; eval_samples records ev_tree before its rollouts.
// The index is built on the main stream before the rollouts (its radix sort's look-back passes starve
// beside the rollout kernel on large trees: 3+ ms instead of 0.2), the search runs on the side stream.
static bool walk_built_for(const clrrt_ctx* c, const NnSetup& su) {
  const auto& b = c->nnw_built;
  return b.n == c->n_nodes && b.ox == su.fr.ox && b.oy == su.fr.oy && b.delta == su.fr.delta && b.x0 == su.x0 &&
         b.y0 == su.y0 && b.x1 == su.x1 && b.y1 == su.y1;
}
static int pre_roll_build(clrrt_ctx* c, const NnSetup& su) {
  KTimer kt(c, 0, c->stream);
  const int rw = ensure_walk(c);
  if (rw != CLRRT_OK) return rw;
  if (walk_built_for(c, su)) return CLRRT_OK;  // built ahead (next_round_build)
  HIPC(c, launch_nn_walk_build(c->stream, c->nn, (int)c->n_nodes, su.fr, su.x0, su.y0, su.x1, su.y1, c->nnw,
                               c->nnw_alt.P ? &c->nnw_alt : nullptr));
  auto& b = c->nnw_built;
  b.n = c->n_nodes;
  b.ox = su.fr.ox; b.oy = su.fr.oy; b.delta = su.fr.delta;
  b.x0 = su.x0; b.y0 = su.y0; b.x1 = su.x1; b.y1 = su.y1;
  return CLRRT_OK;
}

// Pipelined rounds, right after a commit: the next round's index over the committed tree goes into
// the other buffer set on the main stream while the side stream's search still reads this one (it
// waits for nothing but the commit; the wait for the side search comes after it).
static int next_round_build(clrrt_ctx* c) {
  const NnSetup su = nn_setup(c);
  if (!walk_serves(c, su)) return CLRRT_OK;
  std::swap(c->nnw, c->nnw_alt);
  c->nnw_built.n = -1;
  return pre_roll_build(c, su);
}

static int launch_side_walk(clrrt_ctx* c, int n2, const NnSetup& su) {
  c->nn_bf_keys += (int64_t)n2 * c->n_nodes;
  c->nn_samples += n2;
  HIPC(c, hipStreamWaitEvent(c->side, c->ev_tree, 0));
  HIPC(c, hipMemcpyAsync(c->d_samples2, c->h_samples2, sizeof(clrrt_sample) * n2, hipMemcpyHostToDevice, c->side));
  c->nn_super_bounds += (int64_t)n2 * walk_super_count(c->n_nodes);
  {
    KTimer kt(c, 0, c->side), kt3(c, 3, c->side);
    HIPC(c, launch_nn_walk_search(c->side, c->d_samples2, n2, c->nn, (int)c->n_nodes, c->dp, su.fr, su.x0, su.y0,
                                  su.x1, su.y1, c->nnw, c->cand2, c->ckey2, c->ncand2, c->ctie2, c->work_ctr + 18,
                                  c->nnw_stateless));
  }
  HIPC(c, hipEventRecord(c->ev_walk, c->side));
  return CLRRT_OK;
}

// After the appended nodes [first_new, first_new + nn) are in the tree (queued on the main stream):
// their search for the next round's samples, merged into the side walk's lists, runs on the side
// stream behind the walk, so the main stream can build the next round's index meanwhile.
static int side_delta_launch(clrrt_ctx* c, int n2, int64_t first_new, int nn) {
  if (nn <= 0) return CLRRT_OK;
  HIPC(c, hipEventRecord(c->ev_commit, c->stream));
  HIPC(c, hipStreamWaitEvent(c->side, c->ev_commit, 0));
  {
    KTimer kt(c, 0, c->side);
    c->nn_bf_keys += (int64_t)n2 * nn;
    const NnSetup su2 = nn_setup(c);  // the box includes the appended nodes
    const int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)n2 * NN_K));
    HIPC(c, launch_nn_delta(c->side, c->d_samples2, n2, c->nn, (int)first_new, nn, c->dp, su2.fr, c->pk, c->pi,
                            max_chunks, c->cand2, c->ckey2, c->ncand2, c->ctie2, c->nn_seed));
  }
  HIPC(c, hipEventRecord(c->ev_walk, c->side));
  return CLRRT_OK;
}

// The main stream waits for the side stream's lists and swaps the *2 buffers in.
static int side_lists_join(clrrt_ctx* c) {
  {
    KTimer kt(c, 4);  // the lists' wait (time the main stream stalls on the side stream)
    HIPC(c, hipStreamWaitEvent(c->stream, c->ev_walk, 0));
  }
  std::swap(c->d_samples, c->d_samples2);
  std::swap(c->h_samples, c->h_samples2);
  std::swap(c->cand, c->cand2);
  std::swap(c->ckey, c->ckey2);
  std::swap(c->ncand, c->ncand2);
  std::swap(c->ctie, c->ctie2);
  return CLRRT_OK;
}

static int merge_side_lists(clrrt_ctx* c, int n2, int64_t first_new, int nn) {
  const int rc = side_delta_launch(c, n2, first_new, nn);
  return rc != CLRRT_OK ? rc : side_lists_join(c);
}

// Stage 1: candidate lists of samples c->d_samples[0..n) (spatial index for large trees).
static int run_nn(clrrt_ctx* c, int n, KeyId* scratch) {
  hipStream_t st = c->stream;
  KTimer kt(c, 0);
  c->nn_bf_keys += (int64_t)n * c->n_nodes;
  c->nn_samples += n;
  int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)n * NN_K));
  if (scratch && c->nn_exact_fused && c->n_nodes <= nn_exact_small_max()) {  // EXACT rounds on small trees
    HIPC(c, launch_nn_exact_small(st, c->d_samples, n, c->nn, (int)c->n_nodes, c->dp, c->cand, c->ckey, c->ncand,
                                  c->ctie));
    return CLRRT_OK;
  }
  const NnSetup su = nn_setup(c);
  if (walk_serves(c, su)) {
    int rc = ensure_walk(c);
    if (rc != CLRRT_OK) return rc;
    c->nnw_built.n = -1;
    HIPC(c, launch_nn_walk(st, c->d_samples, n, c->nn, (int)c->n_nodes, c->dp, su.fr, su.x0, su.y0, su.x1, su.y1,
                           c->nnw, c->cand, c->ckey, c->ncand, c->ctie, c->work_ctr + 18, c->nnw_stateless));
    if (scratch) HIPC(c, launch_nn_exact_only(st, c->d_samples, n, c->nn, (int)c->n_nodes, c->dp, c->ctie, scratch,
                                              c->cand, c->ckey, c->ncand));
    return CLRRT_OK;
  }
  HIPC(c, launch_nn(st, c->d_samples, n, c->nn, (int)c->n_nodes, c->dp, c->pk, c->pi, c->cand, c->ckey,
                    c->ncand, c->ctie, max_chunks, scratch, c->nn_seed, c->work_ctr + 8, su.fr));
  return CLRRT_OK;
}

// EXACT mode, stage 5 with fix-ups (k_conflict_fix): the committed prefix of the round's n samples runs up to the
// first sample whose result the reference would not reproduce.  A sample k_conflict_fix resolves takes the fix-up
// rollouts of the new nodes that enter its list before its result; a sample it cannot resolve (ties, thresholds,
// window changes) gets its list recomputed over the tree the reference's sort sees for it -- the N tree nodes and
// the round's new nodes before it, std::sort's tie order included (launch_nn_exact_x) -- and the candidates that
// list tries before its result which the speculative evaluation did not try (new nodes, or old ones it ordered
// after its result) become fix-ups too.  The fix-ups run in one launch (one job per wave); a sample stands when all
// of its fix-ups fail and its result is still the first success of its list; its counters become those of the
// list's tried candidates.  *L: the prefix.
static int exact_fixups(clrrt_ctx* c, int n, int* L) {
  hipStream_t st = c->stream;
  const int64_t B = c->cap.max_batch;
  const int K = CAND_K;
  if (!c->fix_n) {
    HIPC(c, dalloc(&c->fix_n, B));
    HIPC(c, dalloc(&c->fix_ids, B * FIX_MAX));
    HIPC(c, dalloc(&c->fix_adj, B * 5));
    HIPC(c, dalloc(&c->fix_jobs, B * K));
    HIPC(c, dalloc(&c->fix_res, B * K));
    HIPC(c, dalloc(&c->fix_xrec, 2 * B));
    HIPC(c, dalloc(&c->fix_xi, 2 * B));
    HIPC(c, dalloc(&c->fix_xcand, B * K));
    HIPC(c, dalloc(&c->fix_xkey, B * K));
    HIPC(c, dalloc(&c->fix_xn, 2 * B));
  }
  {
    KTimer kt(c, 2);
    HIPC(c, launch_conflict_fix(st, c->dp, n, c->d_samples, c->regnodes, c->gbnodes, c->so, c->ctie, c->ncand, c->ckey,
                                c->res_spec, c->fix_n, c->fix_ids, c->fix_adj));
  }
  c->h_fix.resize((size_t)n * (1 + FIX_MAX + 5));
  c->h_fix_smp.resize(n);
  c->h_fix_so.resize(n);
  c->h_fix_cand.resize((size_t)n * K);
  c->h_fix_spec.resize((size_t)n * K);
  HIPC(c, hipMemcpyAsync(c->h_fix.data(), c->fix_n, sizeof(int) * n, hipMemcpyDeviceToHost, st));
  HIPC(c, hipMemcpyAsync(c->h_fix.data() + n, c->fix_ids, sizeof(int) * n * FIX_MAX, hipMemcpyDeviceToHost, st));
  HIPC(c, hipMemcpyAsync(c->h_fix.data() + n * (1 + FIX_MAX), c->fix_adj, sizeof(int) * n * 5, hipMemcpyDeviceToHost,
                         st));
  HIPC(c, hipMemcpyAsync(c->h_fix_smp.data(), c->d_samples, sizeof(clrrt_sample) * n, hipMemcpyDeviceToHost, st));
  HIPC(c, hipMemcpyAsync(c->h_fix_so.data(), c->so, sizeof(SampleOut) * n, hipMemcpyDeviceToHost, st));
  HIPC(c, hipMemcpyAsync(c->h_fix_cand.data(), c->cand, sizeof(int) * n * K, hipMemcpyDeviceToHost, st));
  HIPC(c, hipMemcpyAsync(c->h_fix_spec.data(), c->res_spec, sizeof(RollRes) * n * K, hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  const int* fn = c->h_fix.data();
  const int* fid = c->h_fix.data() + n;
  const int* fadj = c->h_fix.data() + n * (1 + FIX_MAX);
  const int64_t N = c->n_nodes;
  // the round's new nodes in commit order: count before each sample, and (sample, 0 regular | 1 goal-biased) by position
  std::vector<int> xpre(n + 1, 0);
  std::vector<int> xpos;
  for (int k = 0; k < n; k++) {
    const SampleOut& o = c->h_fix_so[k];
    xpre[k + 1] = xpre[k];
    if (o.k >= 0) {
      xpos.push_back(2 * k);
      xpre[k + 1]++;
      if (o.gb_ok) { xpos.push_back(2 * k + 1); xpre[k + 1]++; }
    }
  }
  // the samples that need their list recomputed (and whether that fits the LDS kernel)
  const bool x_fits = N + xpre[n] <= nn_exact_small_max() && c->dp.sort_limit <= K;
  int stop = n;
  std::vector<int> xl;
  for (int j = 0; j < n; j++) {
    if (fn[j] >= 0) continue;
    if (!x_fits) { stop = j; if (-fn[j] >= 1 && -fn[j] <= 4) c->ex_stats[4 + -fn[j]]++; break; }
    xl.push_back(j);
  }
  const int nl = (int)xl.size();
  std::vector<int> xc, xn;
  if (nl > 0) {
    std::vector<int> xs(2 * nl);
    for (int i = 0; i < nl; i++) { xs[i] = xl[i]; xs[nl + i] = xpre[xl[i]]; }
    HIPC(c, hipMemcpyAsync(c->fix_xi, xs.data(), sizeof(int) * 2 * nl, hipMemcpyHostToDevice, st));
    {
      KTimer kt(c, 0);
      HIPC(c, launch_nn_exact_x(st, c->d_samples, c->nn, (int)N, c->dp, c->regnodes, c->gbnodes, c->so, n, c->fix_xrec,
                                c->fix_xi, c->fix_xi + nl, nl, xpre[n], c->fix_xcand, c->fix_xkey, c->fix_xn,
                                c->fix_xn + nl));
    }
    xc.resize((size_t)nl * K);
    xn.resize(nl);
    HIPC(c, hipMemcpyAsync(xc.data(), c->fix_xcand, sizeof(int) * nl * K, hipMemcpyDeviceToHost, st));
    HIPC(c, hipMemcpyAsync(xn.data(), c->fix_xn, sizeof(int) * nl, hipMemcpyDeviceToHost, st));
    HIPC(c, hipStreamSynchronize(st));
  }
  auto is_fail = [](int oc) { return oc >= 0 && oc != CLRRT_ROLL_END && oc != CLRRT_ROLL_GOAL; };
  auto add_res = [](SampleOut& d, const RollRes& r, int sign) {
    d.rollouts += sign;
    d.steps += sign * (r.nrows - 1);
    d.f_col += sign * (r.outcome == CLRRT_ROLL_COLLISION);
    d.f_acc += sign * (r.outcome == CLRRT_ROLL_ACCLIMIT);
    d.f_it += sign * (r.outcome == CLRRT_ROLL_ITERLIMIT);
  };
  // per sample: the fix-up jobs and the counters' change apart from them
  c->h_fix_jobs.clear();
  c->h_fix_owner.clear();
  std::vector<SampleOut> delta(n);
  auto job = [&](int j, int from, int parent) {
    Job jb;
    jb.parent = parent;
    jb.from_reg = from;
    jb.gb = 0;
    jb.pad = 0;
    jb.sx = c->h_fix_smp[j].x;
    jb.sy = c->h_fix_smp[j].y;
    jb.row_off = -1;
    c->h_fix_jobs.push_back(jb);
    c->h_fix_owner.push_back(j);
  };
  for (int j = 0, xi = 0; j < stop; j++) {
    SampleOut& d = delta[j];
    d = SampleOut{};
    if (fn[j] >= 0) {
      for (int i = 0; i < fn[j]; i++) {
        const int id = fid[j * FIX_MAX + i];
        job(j, 1 + (id & 1), id >> 1);
      }
      const int* ad = fadj + 5 * j;  // old candidates pushed out of the window (samples without a result)
      d.rollouts += ad[0]; d.steps += ad[1]; d.f_col += ad[2]; d.f_acc += ad[3]; d.f_it += ad[4];
      continue;
    }
    // the recomputed list
    const SampleOut& o = c->h_fix_so[j];
    const int* lst = xc.data() + (size_t)xi * K;
    const int ln = xn[xi];
    xi++;
    const int* spec = c->h_fix_cand.data() + (size_t)j * K;
    const RollRes* sres = c->h_fix_spec.data() + (size_t)j * K;
    const int acc = o.k >= 0 ? spec[o.k] : -1;
    // the speculative counters of the candidates tried before the result (all of them without one) come out ...
    for (int q = 0; q < K; q++) {
      if (spec[q] < 0 || (o.k >= 0 && q >= o.k)) break;
      add_res(d, sres[q], -1);
    }
    // ... and those of the recomputed list's candidates before the result go in (known failures, or fix-ups)
    bool found = false;
    for (int t = 0; t < ln; t++) {
      const int e = lst[t];
      if (e == acc) { found = true; break; }
      int q = -1;
      if (e < N)
        for (int r = 0; r < K && spec[r] >= 0; r++)
          if (spec[r] == e) { q = r; break; }
      if (q >= 0 && (o.k < 0 || q < o.k) && is_fail(sres[q].outcome)) {
        add_res(d, sres[q], +1);
      } else if (e < N) {
        job(j, 0, e);
      } else {
        const int pw = xpos[e - N];
        job(j, 1 + (pw & 1), pw >> 1);
      }
    }
    if (o.k >= 0 && !found) {  // the result is not its list's first success any more
      stop = j;
      c->ex_stats[8]++;
      while (!c->h_fix_owner.empty() && c->h_fix_owner.back() == j) {
        c->h_fix_owner.pop_back();
        c->h_fix_jobs.pop_back();
      }
      break;
    }
  }
  const int nj = (int)c->h_fix_jobs.size();
  c->h_fix_res.resize(nj);
  if (nj > 0) {
    HIPC(c, hipMemcpyAsync(c->fix_jobs, c->h_fix_jobs.data(), sizeof(Job) * nj, hipMemcpyHostToDevice, st));
    RollArgs a = roll_args(c, nj);
    a.jobs = c->fix_jobs;
    a.res = c->fix_res;
    a.res_gb = c->fix_res;  // (SRC_LIST runs no goal-biased pass)
    a.xreg = c->regnodes;
    a.xgb = c->gbnodes;
    a.job_stride = 64;  // one job per wave: the fix-ups run at the lone lane's step latency
    if (c->exact_fix_cap > 0 && c->exact_fix_cap < a.p.n_steps_max) a.p.n_steps_max = c->exact_fix_cap;
    {
      KTimer kt(c, 1);
      HIPC(c, launch_rollout(st, SRC_LIST, a));
    }
    HIPC(c, hipMemcpyAsync(c->h_fix_res.data(), c->fix_res, sizeof(RollRes) * nj, hipMemcpyDeviceToHost, st));
    HIPC(c, hipStreamSynchronize(st));
  }
  // in sample order: a fix-up that succeeds changes the sample's result (it ends the prefix)
  int Lr = stop, resolved = 0;
  bool patched = false;
  const int cap = c->exact_fix_cap > 0 && c->exact_fix_cap < c->dp.n_steps_max ? c->exact_fix_cap : 0;
  for (int j = 0, q = 0; j < stop; j++) {
    SampleOut add = delta[j];
    bool ok = true, any = fn[j] != 0;
    for (; q < nj && c->h_fix_owner[q] == j; q++) {
      const RollRes& r = c->h_fix_res[q];
      // (a capped rollout stopped at the cap: undecided -- the true iteration limit lies beyond it)
      if (!is_fail(r.outcome) || (cap && r.outcome == CLRRT_ROLL_ITERLIMIT)) ok = false;
      add_res(add, r, +1);
    }
    if (!ok) {
      Lr = j;
      c->ex_stats[4]++;
      break;
    }
    if (!any) continue;
    SampleOut& o = c->h_fix_so[j];
    o.rollouts += add.rollouts; o.steps += add.steps; o.f_col += add.f_col; o.f_acc += add.f_acc; o.f_it += add.f_it;
    patched = true;
    resolved++;
  }
  if (patched) HIPC(c, hipMemcpyAsync(c->so, c->h_fix_so.data(), sizeof(SampleOut) * Lr, hipMemcpyHostToDevice, st));
  c->ex_stats[0]++;
  c->ex_stats[1] += resolved;
  c->ex_stats[2] += nj;
  c->ex_stats[3] += Lr < n;
  *L = std::max(1, Lr);
  return CLRRT_OK;
}

// Stages 1-4 (+5 in EXACT mode) for n samples already in c->d_samples.  Returns the number of
// samples to commit (n in BATCH mode).  have_lists: the candidate lists are already in c->cand
// (pipelined rounds); during_roll runs right after the rollout kernel's launch.
static int eval_samples(clrrt_ctx* c, int n, bool exact, int* L_out, bool have_lists = false,
                        const std::function<int()>& during_roll = nullptr,
                        const std::function<int()>& pre_roll = nullptr) {
  hipStream_t st = c->stream;
  KeyId* scratch = nullptr;
  if (exact) {
    int rc = ensure_sort_scratch(c, (int64_t)n * c->n_nodes);
    if (rc != CLRRT_OK) return rc;
    scratch = c->sort_scratch;
  }
  if (!have_lists) {
    int rc = run_nn(c, n, scratch);
    if (rc != CLRRT_OK) return rc;
  }
  // the tree, this round's lists and the walk buffers are final here: work queued by during_roll on
  // another stream waits for this point only, not for the rollouts
  if (pre_roll) {
    int rc = pre_roll();
    if (rc != CLRRT_OK) return rc;
  }
  if (during_roll) HIPC(c, hipEventRecord(c->ev_tree, st));
  // the rollouts' stream: the main one, or (cu_split) their CU-restricted stream, ordered after the
  // main stream's work so far and joined back right after the launch
  hipStream_t rst = st;
  if (c->roll_st) {
    rst = c->roll_st;
    HIPC(c, hipEventRecord(c->ev_rs0, st));
    HIPC(c, hipStreamWaitEvent(rst, c->ev_rs0, 0));
  }
  const bool persistent = c->roll_persistent && c->dp.n_steps_max > 0;
  const bool deferred = persistent && c->rows_deferred;
  if (!deferred) {  // rows into job slots: replays pending from a deferred round run first
    int rc = flush_replays(c);
    if (rc == CLRRT_OK) rc = ensure_slots(c);
    if (rc != CLRRT_OK) return rc;
  }
  const bool defer = c->def.active && !exact && persistent && deferred;
  if (defer) {  // this round's lists and samples into its ring slot (k_select / the replays read them there)
    auto& d = c->def;
    d.slot = (int)(d.round % d.R);
    const int64_t B = c->cap.max_batch;
    HIPC(c, hipMemcpyAsync(d.cand + (int64_t)d.slot * B * CAND_K, c->cand, sizeof(int) * n * CAND_K,
                           hipMemcpyDeviceToDevice, st));
    HIPC(c, hipMemcpyAsync(d.ncand + (int64_t)d.slot * B, c->ncand, sizeof(int) * n, hipMemcpyDeviceToDevice, st));
    HIPC(c, hipMemcpyAsync(d.samp + (int64_t)d.slot * B, c->d_samples, sizeof(clrrt_sample) * n,
                           hipMemcpyDeviceToDevice, st));
    if (d.nd + (int64_t)n > d.vcap) return fail(c, CLRRT_ECAPACITY, "deferred samples exceed the commit buffers");
    if (rst != st) {  // the copies precede the rollouts' ring writes
      HIPC(c, hipEventRecord(c->ev_rs0, st));
      HIPC(c, hipStreamWaitEvent(rst, c->ev_rs0, 0));
    }
  }
  {
    KTimer kt(c, 1, rst);
    RollArgs a = roll_args(c, n * CAND_K);
    a.res = c->res_spec;
    a.res_gb = c->res_gb;
    if (defer) defer_roll_args(c, a, true);
    a.slots = deferred ? nullptr : c->slots;
    a.slot_rows = c->slot_rows;
    a.slot_jobs = (int)(c->cap.max_batch * CAND_K);
    if (deferred) {  // this launch also replays the previous commit's accepted rollouts
      a.rep = c->rep_buf;
      a.nrep = c->rep_n;
    }
    // persistent blocks (1 resident per CU: the step loop fills the register file).  The rollout kernel's
    // makespan is its longest chains, not its width, while the side stream's search of the next round
    // grows with the tree and takes the CUs the rollouts leave; so the grid narrows as the tree grows:
    // 7/8 of the CUs below 300 k nodes, 5/8 to 700 k, 1/2 to 1.1 M, 3/8 beyond (cfg3 round time by tree
    // size and width, tools/blocks_vs_size.py: each step the best or within 2% of it; a fixed 5/8 grid
    // was the best single width).  Scheduling only: results do not depend on the width.
    const int64_t nt = c->n_nodes;
    const int eighths = nt < 300000 ? 7 : nt < 700000 ? 5 : nt < 1100000 ? 4 : 3;
    const int blocks = c->roll_blocks > 0 ? std::min(c->roll_blocks, 4 * c->n_cu)
                       : c->cu_split > 0  ? std::max(1, (c->cu_split * c->n_cu) / 8)
                                          : std::max(1, (eighths * c->n_cu) / 8);
    a.coop_enable = c->roll_coop;
    a.lanes_per_wave = c->roll_lanes > 0 ? c->roll_lanes : c->roll_spread ? 0 : 64;
    if (c->roll_priority) {
      a.perm = c->roll_perm;
      a.pflag = c->roll_pflag;
    }
    unsigned long long*& dbg_host = c->dbg_host;  // diagnostics heartbeat (host-mapped)
    if (c->debug_sync) {  // diagnostics: which kernel of the round does not finish
      if (!dbg_host) HIPC(c, hipHostMalloc((void**)&dbg_host, sizeof(unsigned long long) * 8 * 4096, hipHostMallocMapped));
      memset(dbg_host, 0, sizeof(unsigned long long) * 8 * 4096);
      HIPC(c, hipHostGetDevicePointer((void**)&a.dbg, dbg_host, 0));
      HIPC(c, hipStreamSynchronize(rst));
      fprintf(stderr, "[dbg] pre-rollout work done (n %d, nrep %d, ncarry %d)\n", n, a.nrep, a.ncarry);
    }
    if (persistent && defer) {
      // the round's resets in one launch: the rollout queue / carry counters and the first-success array, the
      // count of this round's samples left pending (k_select) and the compaction's totals (launch_compact)
      FillInts f;
      f.add(a.ncarry_out, 1, 0);
      f.add(c->roll_q, 1, 0);
      f.add(c->def.best + a.sbase, n, 0x7f7f7f7f);
      f.add(c->def.d_cnt + 2, 1, 0);
      f.add((int*)c->totals, 16, 0);
      HIPC(c, launch_fill_ints(rst, f));
      c->totals_zeroed = true;
      HIPC(c, launch_rollout_persistent(rst, a, n, c->roll_q, c->def.best, blocks, true));
    } else if (persistent)
      HIPC(c, launch_rollout_persistent(rst, a, n, c->roll_q, defer ? c->def.best : c->roll_best, blocks));
    else
      HIPC(c, launch_rollout(rst, SRC_SPEC, a));
    if (c->debug_sync) {
      const auto t0 = std::chrono::steady_clock::now();
      while (hipStreamQuery(rst) == hipErrorNotReady) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 10.0) {
          fprintf(stderr, "[dbg] rollout kernel not done after 10 s; waves (iterations, busy, parked, qdone|first "
                          "busy lane, j|pass, steps|chain, wp|N, t):\n");
          unsigned long long tmax = 0;
          for (int w = 0; w < 4096; w++) tmax = std::max(tmax, dbg_host[w * 8 + 7]);
          int shown = 0;
          for (int w = 0; w < 4096 && shown < 40; w++) {
            const unsigned long long* d = dbg_host + w * 8;
            if (d[7] == 0 || tmax - d[7] < 100000000ull) continue;  // still beating in the last second
            if (d[1] == 0 && d[2] == 0 && (d[3] >> 32)) continue;      // finished
            fprintf(stderr, "  wave %d: it %llu busy %016llx parked %016llx qdone %llu lane %d j %d pass %d steps %d "
                            "chain %d wp %d N %d age %.3f s\n", w, d[0], d[1], d[2], d[3] >> 32, (int)(uint32_t)d[3],
                    (int)(d[4] >> 32), (int)(uint32_t)d[4], (int)(d[5] >> 32), (int)(uint32_t)d[5], (int)(d[6] >> 32),
                    (int)(uint32_t)d[6], (double)(tmax - d[7]) * 1e-8);
            shown++;
          }
          int alive = 0;
          for (int w = 0; w < 4096; w++) alive += dbg_host[w * 8 + 7] != 0 && tmax - dbg_host[w * 8 + 7] < 100000000ull;
          fprintf(stderr, "  waves still beating: %d\n", alive);
          abort();
        }
      }
      fprintf(stderr, "[dbg] rollout kernel done: %s\n", hipGetErrorString(hipStreamQuery(rst)));
    }
    if (deferred) c->rep_n = 0;
    c->eval_deferred = deferred;
  }
  if (c->roll_st) {
    HIPC(c, hipEventRecord(c->ev_rs1, rst));
    HIPC(c, hipStreamWaitEvent(st, c->ev_rs1, 0));
  }
  if (during_roll) {  // queued behind the rollout kernel, whose persistent blocks take the CUs first
    int rc = during_roll();
    if (rc != CLRRT_OK) return rc;
  }
  SelArgs s;
  memset(&s, 0, sizeof(s));
  s.p = c->dp; s.tree = c->tree; s.cand = c->cand; s.ckey = c->ckey; s.ncand = c->ncand; s.res = c->res_spec;
  s.res_gb = c->res_gb; s.regnodes = c->regnodes; s.gbnodes = c->gbnodes; s.so = c->so; s.B = n;
  if (defer) {  // views: the deferred samples of earlier rounds, then this round's
    auto& d = c->def;
    s.cand = d.cand; s.ncand = d.ncand; s.res = d.res; s.res_gb = d.res_gb;
    s.ckey = nullptr;  // the round's keys are not in the rings (EXACT's conflict threshold only)
    s.view = d.dlist[d.cur_dl];
    s.nd = d.nd;
    s.sbase = d.slot * (int)c->cap.max_batch;
    s.gv = d.gv;
    s.pend = d.pend;
    s.new_pend = d.d_cnt + 2;
    s.B = d.nd + n;  // (d_cnt[2] was reset by the round's prologue fill before the rollouts)
  }
  c->def.nd_eval = defer ? c->def.nd : -1;
  {
    KTimer kt(c, 2);
    HIPC(c, launch_select(st, s));
  }
  int L = n;
  if (exact && n > 1 && c->exact_fixup) {
    int rc = exact_fixups(c, n, &L);
    if (rc != CLRRT_OK) return rc;
  } else if (exact && n > 1) {
    c->h_int[0] = n;
    HIPC(c, hipMemcpyAsync(c->first_conflict, c->h_int, sizeof(int), hipMemcpyHostToDevice, st));
    {
      KTimer kt(c, 2);
      HIPC(c, launch_conflict(st, c->dp, n, c->d_samples, c->regnodes, c->gbnodes, c->so, c->ctie,
                              c->first_conflict));
    }
    HIPC(c, hipMemcpyAsync(c->h_int + 1, c->first_conflict, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(c, hipStreamSynchronize(st));
    L = std::max(1, std::min(n, c->h_int[1]));
  }
  *L_out = L;
  return CLRRT_OK;
}

// Stages 5-6: compact the first L samples into node records (c->out_nodes), reserve arena rows,
// copy the accepted trajectories into the arena.  *n_out = records.
static int compact_and_copy(clrrt_ctx* c, int L, int* n_out, bool merge_bbox) {
  hipStream_t st = c->stream;
  auto& d = c->def;
  const bool defer = d.nd_eval >= 0;  // eval_samples selected views (deferred samples + this round's)
  const int V = defer ? d.nd_eval + L : L;
  {
    KTimer kt(c, 2);
    const bool tag = defer && c->sh.world > 1;  // the exchange orders deferred samples by age
    HIPC(c, launch_compact(st, V, c->d_samples, c->cand, c->regnodes, c->gbnodes, c->so, c->n_rows, c->rank,
                           c->out_nodes, c->jobs, c->totals, c->cmp, tag ? d.slot : 0, tag ? d.R : 0,
                           (int)c->cap.max_batch, c->totals_zeroed));
    c->totals_zeroed = false;
    if (merge_bbox) HIPC(c, launch_bbox(st, c->out_nodes, c->totals, 0, c->d_bbox));
    // the views still pending, in view order: the next commit's deferred samples
    if (defer) HIPC(c, launch_defer_select(st, d.gv, d.pend, V, d.dlist[1 - d.cur_dl], d.d_cnt, d.sel_tmp, d.sel_bytes));
  }
  HIPC(c, hipMemcpyAsync(c->h_totals, c->totals, sizeof(int64_t) * 8, hipMemcpyDeviceToHost, st));
  if (merge_bbox) HIPC(c, hipMemcpyAsync(c->h_bbox, c->d_bbox, sizeof(double) * 4, hipMemcpyDeviceToHost, st));
  if (defer) {
    HIPC(c, hipMemcpyAsync(c->h_int, d.d_cnt, sizeof(int) * 2, hipMemcpyDeviceToHost, st));
    HIPC(c, hipMemcpyAsync(c->h_int + 3, d.d_cnt + 2, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(c, hipMemcpyAsync(c->h_int + 2, (const char*)(c->work_ctr + 62), sizeof(int), hipMemcpyDeviceToHost, st));
  }
  HIPC(c, hipStreamSynchronize(st));
  {
    const int rw = watchdog_check(c);
    if (rw != CLRRT_OK) return rw;
  }
  if (c->iter_log && !defer && L > 0) {  // the committed iterations' records, in sample order
    c->iter_tmp.resize(L);
    HIPC(c, hipMemcpy(c->iter_tmp.data(), c->so, sizeof(SampleOut) * L, hipMemcpyDeviceToHost));
    for (int j = 0; j < L; j++) {
      const SampleOut& o = c->iter_tmp[j];
      clrrt_iteration r;
      r.nodes = (o.k >= 0) + (o.k >= 0 && o.gb_ok);
      r.sim_count = o.steps; r.fail_collision = o.f_col; r.fail_acclimit = o.f_acc; r.fail_iterlimit = o.f_it;
      r.rollouts = o.rollouts;
      c->iters.push_back(r);
    }
  }
  if (merge_bbox) bbox_add(c, c->h_bbox[0], c->h_bbox[1], c->h_bbox[2], c->h_bbox[3]);
  if (defer) {
    if (c->h_int[2] != 0 || c->h_int[1] > d.carry_cap)
      return fail(c, CLRRT_ECAPACITY, "suspended rollouts exceed the carry buffer (raise defer_steps)");
    if (L > 0) d.deferred_total += c->h_int[3];  // this round's samples left pending (k_select)
    d.cur_dl ^= 1;
    d.nd = c->h_int[0];
    d.cur_c ^= 1;
    d.ncarry = c->h_int[1];
    d.round++;
    d.nd_eval = -1;
  }
  int64_t nn = c->h_totals[0], nr = c->h_totals[1];
  if (c->n_rows + nr > c->cap.max_rows) return fail(c, CLRRT_ECAPACITY, "trajectory arena full");
  if (c->fail_at_round > 0 && --c->fail_at_round == 0)
    return fail(c, CLRRT_ECAPACITY, "injected failure (option fail_at_round)");
  c->counters.sim_count += c->h_totals[2];
  c->counters.fail_collision += c->h_totals[3];
  c->counters.fail_acclimit += c->h_totals[4];
  c->counters.fail_iterlimit += c->h_totals[5];
  c->counters.rollouts += c->h_totals[6];
  c->last_goal_nodes = c->h_totals[7];
  if (c->eval_deferred) {  // the accepted rollouts are replayed into the arena by the next persistent launch
    if (c->rep_n > 0) {
      int rc = flush_replays(c);
      if (rc != CLRRT_OK) return rc;
    }
    KTimer kt(c, 2);
    if (defer)  // the committed samples' lists and results sit in the rings
      HIPC(c, launch_replay_gather(st, c->jobs, c->out_nodes, (int)nn, c->tree, d.cand, d.samp, d.res, c->rep_buf));
    else
      HIPC(c, launch_replay_gather(st, c->jobs, c->out_nodes, (int)nn, c->tree, c->cand, c->d_samples, c->res_spec,
                                   c->rep_buf));
    c->rep_n = (int)nn;
  } else {
    KTimer kt(c, 2);
    HIPC(c, launch_copy_rows(st, c->jobs, c->out_nodes, (int)nn, c->slots, c->slot_rows,
                             (int)(c->cap.max_batch * CAND_K), c->arena));
  }
  c->n_rows += nr;
  c->last_eval_rows = nr;
  *n_out = (int)nn;
  return CLRRT_OK;
}

// Deferred samples: the rings for the context's T and n_steps_max, the view-sized commit buffers and the
// carry buffers (allocated on the first expansion that defers, grown when T shrinks or sim_dt does).
static int ensure_defer(clrrt_ctx* c) {
  auto& d = c->def;
  const int64_t B = c->cap.max_batch;
  const int n = std::max(1, c->dp.n_steps_max);
  const int R = (int)((2LL * n + d.T - 1) / d.T) + 2;
  // sharded rounds carry a record's origin-round age in 8 bits (k_compact_scatter / k_xorder_keys)
  if (c->sh.world > 1 && R > 256)
    return fail(c, CLRRT_EINVAL, "defer_steps too small for sharded rounds (more than 256 rounds in flight)");
  if (!d.res || d.R < R) {
    HIPC(c, hipStreamSynchronize(c->stream));
    for (void* p : {(void*)d.res, (void*)d.res_gb, (void*)d.cand, (void*)d.ncand, (void*)d.samp, (void*)d.best})
      if (p) HIPC(c, hipFree(p));
    d.res = nullptr; d.res_gb = nullptr; d.cand = nullptr; d.ncand = nullptr; d.samp = nullptr; d.best = nullptr;
    d.R = 0;
    HIPC(c, dalloc(&d.res, (size_t)R * B * CAND_K));
    HIPC(c, dalloc(&d.res_gb, (size_t)R * B * CAND_K));
    HIPC(c, dalloc(&d.cand, (size_t)R * B * CAND_K));
    HIPC(c, dalloc(&d.ncand, (size_t)R * B));
    HIPC(c, dalloc(&d.samp, (size_t)R * B));
    HIPC(c, dalloc(&d.best, (size_t)R * B));
    d.R = R;
  }
  if (!d.gv || d.vcap < (int64_t)d.R * B) {
    // every commit path holds up to vcap views: the deferred samples (at most R - 1 earlier rounds' worth,
    // the ring) + one round
    const int64_t V = (int64_t)d.R * B;
    int rc = flush_replays(c);  // rep_buf is re-made below
    if (rc != CLRRT_OK) return rc;
    HIPC(c, hipStreamSynchronize(c->stream));
    for (void* p : {(void*)c->regnodes, (void*)c->gbnodes, (void*)c->so, (void*)c->out_nodes, (void*)c->jobs,
                    c->rep_buf, (void*)c->cmp.packed, (void*)c->cmp.scanned, c->cmp.tmp})
      if (p) HIPC(c, hipFree(p));
    c->regnodes = nullptr; c->gbnodes = nullptr; c->so = nullptr; c->out_nodes = nullptr; c->jobs = nullptr;
    c->rep_buf = nullptr; c->cmp.packed = nullptr; c->cmp.scanned = nullptr; c->cmp.tmp = nullptr;
    for (void* p : {(void*)d.dlist[0], (void*)d.dlist[1], (void*)d.gv, (void*)d.pend, d.sel_tmp, (void*)d.d_cnt,
                    d.carry[0], d.carry[1]})
      if (p) HIPC(c, hipFree(p));
    d.dlist[0] = d.dlist[1] = nullptr; d.gv = nullptr; d.pend = nullptr; d.sel_tmp = nullptr; d.d_cnt = nullptr;
    d.carry[0] = d.carry[1] = nullptr;
    HIPC(c, dalloc(&c->regnodes, V));
    HIPC(c, dalloc(&c->gbnodes, V));
    HIPC(c, dalloc(&c->so, V));
    HIPC(c, dalloc(&c->out_nodes, 2 * V));
    HIPC(c, dalloc(&c->jobs, 2 * V));
    HIPC(c, hipMalloc(&c->rep_buf, replay_bytes() * (size_t)2 * V));
    HIPC(c, dalloc(&c->cmp.packed, V));
    HIPC(c, dalloc(&c->cmp.scanned, V));
    c->cmp.tmp_bytes = compact_scan_bytes((int)V);
    HIPC(c, hipMalloc(&c->cmp.tmp, std::max<size_t>(c->cmp.tmp_bytes, 256)));
    HIPC(c, dalloc(&d.dlist[0], V));
    HIPC(c, dalloc(&d.dlist[1], V));
    HIPC(c, dalloc(&d.gv, V));
    HIPC(c, dalloc(&d.pend, V));
    d.sel_bytes = defer_select_bytes((int)V);
    HIPC(c, hipMalloc(&d.sel_tmp, std::max<size_t>(d.sel_bytes, 256)));
    HIPC(c, dalloc(&d.d_cnt, 3));
    // suspended chains: at most every job of the rounds in flight (a launch's chains all come from them)
    d.carry_cap = (int)std::min<int64_t>(V * CAND_K, 1 << 21);
    HIPC(c, hipMalloc(&d.carry[0], carry_bytes() * (size_t)d.carry_cap));
    HIPC(c, hipMalloc(&d.carry[1], carry_bytes() * (size_t)d.carry_cap));
    d.vcap = V;
  }
  return CLRRT_OK;
}

// The start of an expansion: deferral on for BATCH rounds when the option asks for it and the rollouts run
// persistent with deferred rows (the paths the carry records exist for).
static int defer_begin(clrrt_ctx* c, bool batch) {
  auto& d = c->def;
  d.active = batch && d.T > 0 && c->roll_persistent && c->rows_deferred && c->dp.n_steps_max > 0;
  d.nd = 0; d.ncarry = 0; d.round = 0; d.slot = 0; d.nd_eval = -1; d.deferred_total = 0;
  return d.active ? ensure_defer(c) : CLRRT_OK;
}

// Ring / carry fields of a rollout launch: this round's slot (cap T) or, for the drain (cap 0), no new jobs.
static void defer_roll_args(clrrt_ctx* c, RollArgs& a, bool capped) {
  auto& d = c->def;
  a.res = d.res;
  a.res_gb = d.res_gb;
  a.jbase = d.slot * (int)c->cap.max_batch * CAND_K;
  a.sbase = d.slot * (int)c->cap.max_batch;
  a.cap = capped ? d.T : 0;
  a.carry_in = d.carry[d.cur_c];
  a.ncarry = d.ncarry;
  a.carry_out = d.carry[1 - d.cur_c];
  a.ncarry_out = d.d_cnt + 1;
  a.carry_cap = d.carry_cap;
}

// Row slots for the paths that store speculative rows (option "rows_deferred" 0, non-persistent rollouts).
static int ensure_slots(clrrt_ctx* c) {
  const int need = c->dp.n_steps_max + 1;
  if (c->slots && c->slot_rows >= need) return CLRRT_OK;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->slots) HIPC(c, hipFree(c->slots));
  c->slots = nullptr;
  c->slot_rows = 0;
  HIPC(c, dalloc(&c->slots, (size_t)2 * need * 10 * c->cap.max_batch * CAND_K));
  c->slot_rows = need;
  return CLRRT_OK;
}

// k_roll_run's watchdog (work counters 56..59): a wave that loops far past any correct launch exits and
// records its state; reported as an error.
static int watchdog_check(clrrt_ctx* c) {
  unsigned long long h[4];
  HIPC(c, hipMemcpy(h, c->work_ctr + 56, sizeof(h), hipMemcpyDeviceToHost));
  if (h[0] == 0) return CLRRT_OK;
  char msg[256];
  snprintf(msg, sizeof(msg), "rollout kernel watchdog: %llu waves; j %d fin %d steps %d chain %d qdone %d busy %d",
           h[0], (int)(h[1] >> 32), (int)(uint32_t)h[1], (int)(h[2] >> 32), (int)(uint32_t)h[2], (int)(h[3] >> 32),
           (int)(uint32_t)h[3]);
  return fail(c, CLRRT_EHIP, msg);
}

// Every replay must run exactly as many steps as its committed node has rows (k_roll_run counts the
// ones that do not in work counter 61 and stores no row past the node's count).  Nonzero means the
// arena's rows are not the committed rollouts': reported as an error instead of a silently wrong tree.
static int replay_check(clrrt_ctx* c) {
  HIPC(c, hipMemcpyAsync(c->h_int + 2, (const char*)(c->work_ctr + 61), sizeof(int), hipMemcpyDeviceToHost,
                         c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->h_int[2] != 0) return fail(c, CLRRT_EHIP, "a deferred-row replay diverged from its committed rollout");
  return watchdog_check(c);
}

// Run the pending replays (the last commit's accepted rollouts, deferred rows) on their own: before
// anything reads the arena, changes what a replay depends on (parameters, obstacles), or at the end of
// an expansion.  Same kernel, no jobs of a round.
static int flush_replays(clrrt_ctx* c) {
  auto& d = c->def;
  if (c->rep_n <= 0 && d.ncarry <= 0) return CLRRT_OK;
  HIPC(c, hipSetDevice(c->device));
  KTimer kt(c, 1);
  RollArgs a = roll_args(c, 0);
  a.res = c->res_spec;
  a.res_gb = c->res_gb;
  a.rep = c->rep_buf;
  a.nrep = c->rep_n;
  a.coop_enable = c->roll_coop;
  a.lanes_per_wave = c->roll_spread ? 0 : 64;
  // chains resumed from the carry buffer index the ring's first-success flags (ring slot x max_batch), not
  // roll_best's max_batch entries
  int* best = c->roll_best;
  if (d.ncarry > 0) {  // suspended replays of a deferring expansion: run to their end
    defer_roll_args(c, a, false);
    best = d.best;
    d.ncarry = 0;
  }
  HIPC(c, launch_rollout_persistent(c->stream, a, 0, c->roll_q, best, c->n_cu));
  c->rep_n = 0;
  return replay_check(c);
}

// The end of a deferring expansion: one launch without a cap runs every suspended chain (and replay) to its
// end, the samples still pending commit in view order (the oldest round first), then their rows replay.
static int defer_drain(clrrt_ctx* c, int64_t* goal_nodes) {
  auto& d = c->def;
  if (!d.active) return CLRRT_OK;
  const bool sharded = c->sh.world > 1;  // every rank takes part in the drain's exchange
  if (d.nd > 0 || d.ncarry > 0 || sharded) {
    hipStream_t st = c->stream;
    {
      KTimer kt(c, 1);
      RollArgs a = roll_args(c, 0);
      a.rep = c->rep_buf;
      a.nrep = c->rep_n;
      a.coop_enable = c->roll_coop;
      a.lanes_per_wave = c->roll_spread ? 0 : 64;
      defer_roll_args(c, a, false);
      HIPC(c, launch_rollout_persistent(st, a, 0, c->roll_q, d.best, c->n_cu));
      c->rep_n = 0;
      d.ncarry = 0;
    }
    if (d.nd > 0 || sharded) {
      SelArgs s;
      memset(&s, 0, sizeof(s));
      s.p = c->dp; s.tree = c->tree; s.cand = d.cand; s.ckey = nullptr; s.ncand = d.ncand; s.res = d.res;
      s.res_gb = d.res_gb; s.regnodes = c->regnodes; s.gbnodes = c->gbnodes; s.so = c->so;
      s.view = d.dlist[d.cur_dl]; s.nd = d.nd; s.sbase = 0; s.gv = d.gv; s.pend = d.pend; s.B = d.nd;
      if (d.nd > 0) {
        KTimer kt(c, 2);
        HIPC(c, launch_select(st, s));
      }
      d.nd_eval = d.nd;
      int nn = 0, n_app = 0;
      int rc = compact_and_copy(c, 0, &nn, true);
      if (rc == CLRRT_OK) rc = commit_round(c, nn, c->sh.max_ms, &n_app);
      if (rc != CLRRT_OK) return rc;
      if (goal_nodes) *goal_nodes += c->last_goal_nodes;
      if (d.nd != 0 || d.ncarry != 0) return fail(c, CLRRT_EHIP, "deferred samples left after the drain");
    }
  }
  d.active = false;
  return flush_replays(c);
}

static int append_nodes(clrrt_ctx* c, const clrrt_node* dev_nodes, int n) {
  if (c->n_nodes + n > c->cap.max_nodes) return fail(c, CLRRT_ECAPACITY, "tree full");
  {
    KTimer kt(c, 2);
    HIPC(c, launch_append(c->stream, dev_nodes, n, c->n_nodes, c->tree, c->nn));
  }
  c->n_nodes += n;
  return CLRRT_OK;
}

extern "C" {

int clrrt_round_eval(clrrt_ctx* c, const clrrt_sample* samples, int32_t n, void* dev_out, int32_t* n_out) {
  if (!c || n < 0 || (n > 0 && !samples) || !n_out) return CLRRT_EINVAL;
  if (n > c->cap.max_batch) return fail(c, CLRRT_ECAPACITY, "batch larger than max_batch");
  if (c->n_nodes <= 0) return fail(c, CLRRT_ESTATE, "tree not initialised");
  HIPC(c, hipSetDevice(c->device));
  *n_out = 0;
  if (n == 0) return CLRRT_OK;
  // lists prefetched by the previous round (clrrt_round_prefetch) serve exactly the declared samples
  const bool have = c->pf_state == 2 && (int)c->pf_samples.size() == n &&
                    memcmp(c->pf_samples.data(), samples, sizeof(clrrt_sample) * n) == 0;
  if (!have) {
    if (c->pf_state != 0 && c->side) HIPC(c, hipStreamSynchronize(c->side));
    memcpy(c->h_samples, samples, sizeof(clrrt_sample) * n);
    HIPC(c, hipMemcpyAsync(c->d_samples, c->h_samples, sizeof(clrrt_sample) * n, hipMemcpyHostToDevice, c->stream));
  }
  c->pf_state = 0;
  const int n2 = (int)std::min<size_t>(c->pf_next.size(), (size_t)c->cap.max_batch);
  NnSetup su{};
  bool side = false;
  if (n2 > 0 && c->nn_pipeline) {
    su = nn_setup(c);
    side = walk_serves(c, su);
  }
  auto during = [&]() -> int {
    memcpy(c->h_samples2, c->pf_next.data(), sizeof(clrrt_sample) * n2);
    c->pf_samples.assign(c->pf_next.begin(), c->pf_next.begin() + n2);
    c->pf_state = 1;
    return launch_side_walk(c, n2, su);
  };
  c->pf_next.clear();
  int L = n, rc;
  auto build = [&]() -> int { return pre_roll_build(c, su); };
  if ((rc = eval_samples(c, n, false, &L, have, side ? std::function<int()>(during) : nullptr,
                         side ? std::function<int()>(build) : nullptr)) != CLRRT_OK)
    return rc;
  int nn = 0;
  if ((rc = compact_and_copy(c, L, &nn, false)) != CLRRT_OK) return rc;
  if (dev_out && nn > 0)
    HIPC(c, hipMemcpyAsync(dev_out, c->out_nodes, sizeof(clrrt_node) * nn, hipMemcpyDeviceToDevice, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  *n_out = nn;
  return CLRRT_OK;
}

int clrrt_round_commit(clrrt_ctx* c, const void* dev_nodes, int32_t n, int32_t local_first, int32_t local_count) {
  (void)local_first;
  (void)local_count;  // the local records' rows are only reserved by clrrt_round_eval: the next rollout
                      // launch (or clrrt_rows_flush) replays them into the arena (deferred rows)
  if (!c || n < 0 || (n > 0 && !dev_nodes)) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  const int64_t first_new = c->n_nodes;
  int rc = append_nodes(c, (const clrrt_node*)dev_nodes, n);
  if (rc != CLRRT_OK) return rc;
  if (n > 0) {
    HIPC(c, launch_bbox(c->stream, (const clrrt_node*)dev_nodes, nullptr, n, c->d_bbox));
    HIPC(c, hipMemcpyAsync(c->h_bbox, c->d_bbox, sizeof(double) * 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIPC(c, hipStreamSynchronize(c->stream));
  if (n > 0) bbox_add(c, c->h_bbox[0], c->h_bbox[1], c->h_bbox[2], c->h_bbox[3]);
  if (c->pf_state == 1) {  // the next round's search ran beside this round's rollouts
    // as in clrrt_expand: the appended nodes' search behind it on the side stream, the next round's
    // index into the other buffer set meanwhile
    if ((rc = side_delta_launch(c, (int)c->pf_samples.size(), first_new, n)) != CLRRT_OK) return rc;
    if (c->nnw_double && (rc = next_round_build(c)) != CLRRT_OK) return rc;
    if ((rc = side_lists_join(c)) != CLRRT_OK) return rc;
    c->pf_state = 2;
  }
  return CLRRT_OK;
}

int clrrt_rows_flush(clrrt_ctx* c) {
  if (!c) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  return flush_replays(c);
}

int clrrt_round_prefetch(clrrt_ctx* c, const clrrt_sample* next, int32_t n) {
  if (!c || n < 0 || (n > 0 && !next)) return CLRRT_EINVAL;
  if (n > c->cap.max_batch) return fail(c, CLRRT_ECAPACITY, "batch larger than max_batch");
  c->pf_next.assign(next, next + n);
  return CLRRT_OK;
}

// ---------------------------------------------------------------------------------------------
// Sharded rounds: goal nodes among the records appended since the last reset (every rank's), read once at
// the end of an expansion.
static int shard_goal_reset(clrrt_ctx* c) {
  HIPC(c, hipMemsetAsync(c->sh.d_goal, 0, sizeof(unsigned long long), c->stream));
  return CLRRT_OK;
}
static int shard_goal_count(clrrt_ctx* c, int64_t* out) {
  unsigned long long v = 0;
  HIPC(c, hipMemcpyAsync(c->h_totals, c->sh.d_goal, sizeof(v), hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  memcpy(&v, c->h_totals, sizeof(v));
  *out = (int64_t)v;
  return CLRRT_OK;
}

// Sharded rounds (clrrt_set_shards): this rank's contiguous slice [f, f + n) of a round of g samples.
static inline void shard_slice(const clrrt_ctx* c, int64_t g, int64_t* f, int* n) {
  const int64_t W = c->sh.world, r = c->sh.rank;
  *f = g * r / W;
  *n = (int)(g * (r + 1) / W - *f);
}

// The end of a sharded expansion: one closing exchange on every rank (no records), which carries this rank's
// failure (aux bit 48) to the others -- a failure in its last round's post-exchange work or in the drain included,
// when no round exchange is left for them to see it in -- and reports theirs.  Skipped when every rank already
// left at the same exchange (an error flag seen there) or the collective itself failed.  Returns the final status.
static int shard_expansion_end(clrrt_ctx* c, int rc) {
  auto& h = c->sh;
  if (h.world > 1 && !h.poison_seen && !h.fn_failed) {
    clrrt_exchange_io io;
    memset(&io, 0, sizeof(io));
    io.flags = 1;
    io.elapsed_ms = h.max_ms;
    io.aux_local = rc != CLRRT_OK ? (1ll << 48) : 0;
    io.bbox_local[0] = io.bbox_local[1] = HUGE_VAL;
    io.bbox_local[2] = io.bbox_local[3] = -HUGE_VAL;
    io.stream = (void*)c->stream;
    io.aux_sum = io.aux_local;
    const int r = h.fn(h.user, &io);
    if (rc == CLRRT_OK) {
      if (r != 0) rc = fail(c, CLRRT_EHIP, "the closing exchange of the sharded expansion failed");
      else if (io.aux_sum >> 48)
        rc = fail(c, CLRRT_EHIP, "sharded expansion: " + std::to_string(io.aux_sum >> 48) + " rank(s) failed");
    }
  }
  if (rc != CLRRT_OK) {  // the expansion's suspended chains and pending samples are dropped with its results
    c->def.ncarry = 0;
    c->def.nd = 0;
  }
  return rc;
}
static void shard_expansion_begin(clrrt_ctx* c) {
  c->sh.poison_seen = c->sh.fn_failed = false;
}

// The commit of a round's records (c->out_nodes[0 .. nn)): appended as they are (one rank), or exchanged
// with the other ranks and the union appended in the same order on every rank.  *n_app = records appended.
// Sharded, nothing here waits for the device besides the hook's read of the exchanged counts: the records go
// to dev_local on the engine's stream and the hook orders its collective after it (clrrt_exchange_io.stream);
// the ranks' position bounds travel with the counts (compact_and_copy read this rank's into h_bbox).
static int commit_round(clrrt_ctx* c, int nn, double elapsed_ms, int* n_app) {
  auto& h = c->sh;
  *n_app = 0;
  if (h.world <= 1) {
    *n_app = nn;
    const int rc = append_nodes(c, c->out_nodes, nn);
    if (rc == CLRRT_OK) c->round_sizes.push_back(c->n_nodes);
    return rc;
  }
  if (nn > h.cap_local) return fail(c, CLRRT_ECAPACITY, "the round's records exceed the exchange buffer");
  std::optional<KTimer> kt;
  kt.emplace(c, 5);  // the exchange's span on the engine's stream
  if (nn > 0)
    HIPC(c, hipMemcpyAsync(h.dev_local, c->out_nodes, sizeof(clrrt_node) * nn, hipMemcpyDeviceToDevice, c->stream));
  clrrt_exchange_io io;
  memset(&io, 0, sizeof(io));
  io.n_local = nn;
  io.elapsed_ms = elapsed_ms;
  // aux: this rank's pending deferred samples (low 32 bits) and whether its arena can take another round of
  // its slice (+ its deferred samples) -- summed over the ranks, so every rank takes the same stop decision
  const int64_t nd_loc = c->def.active ? c->def.nd : 0;
  const bool rows_full =
      c->n_rows + nn + 2 * ((int64_t)h.last_nb + nd_loc) * (c->dp.n_steps_max + 1) > c->cap.max_rows;
  io.aux_local = nd_loc + (rows_full ? (1ll << 32) : 0);
  for (int q = 0; q < 4; q++) io.bbox_local[q] = nn > 0 ? c->h_bbox[q] : (q < 2 ? HUGE_VAL : -HUGE_VAL);
  io.stream = (void*)c->stream;
  io.max_elapsed_ms = elapsed_ms;
  io.aux_sum = io.aux_local;
  if (h.fn(h.user, &io) != 0 || io.n_all < 0 || (io.n_all > 0 && !io.dev_all)) {
    h.fn_failed = true;
    return fail(c, CLRRT_EHIP, "the exchange of the round's records failed");
  }
  kt.reset();
  const int64_t aux_sum = io.aux_sum;
  if (aux_sum >> 48) {  // another rank failed (shard_poison): every rank leaves the expansion
    h.poison_seen = true;
    return fail(c, CLRRT_EHIP, "sharded expansion: " + std::to_string(aux_sum >> 48) + " rank(s) failed this round");
  }
  if (c->fail_after_exchange > 0 && --c->fail_after_exchange == 0)
    return fail(c, CLRRT_ECAPACITY, "injected failure (option fail_after_exchange)");
  h.max_ms = io.max_elapsed_ms;
  h.nd_global = aux_sum & 0xffffffffll;
  h.rows_stop = (aux_sum >> 32) & 0xffff;
  const int32_t n_all = io.n_all;
  void* all = io.dev_all;
  if (n_all > 0) {
    if (n_all > h.xcap) {
      HIPC(c, hipStreamSynchronize(c->stream));
      for (void* p : {(void*)h.xbuf, (void*)h.xkey, h.xtmp})
        if (p) HIPC(c, hipFree(p));
      h.xbuf = nullptr; h.xkey = nullptr; h.xtmp = nullptr;
      const int64_t cap = std::max<int64_t>(2 * (int64_t)n_all, 4096);
      HIPC(c, dalloc(&h.xbuf, cap));
      HIPC(c, dalloc(&h.xkey, 4 * cap));
      h.xtmp_bytes = xorder_sort_bytes((int)cap);
      HIPC(c, hipMalloc(&h.xtmp, std::max<size_t>(h.xtmp_bytes, 256)));
      h.xcap = cap;
    }
    HIPC(c, launch_xorder(c->stream, (const clrrt_node*)all, n_all, c->def.active, h.xkey, h.xtmp, h.xtmp_bytes,
                          h.xbuf, h.d_goal));
    int rc = append_nodes(c, h.xbuf, n_all);
    if (rc != CLRRT_OK) return rc;
    // the tree's bounding box takes every rank's records (the walk frame is then the same on every rank); the
    // union of the ranks' bounds is the bound of the union (min / max), so no pass over the gathered records
    bbox_add(c, io.bbox_all[0], io.bbox_all[1], io.bbox_all[2], io.bbox_all[3]);
  }
  *n_app = n_all;
  c->round_sizes.push_back(c->n_nodes);
  return CLRRT_OK;
}

// ---------------------------------------------------------------------------------------------
// Lag-2 pipelined BATCH rounds (option "nn_lag" 2).  BATCH rounds commit every sample, so the samples of
// the next rounds are known ahead.  The walk search of round r+2's samples runs over the tree T_r (the
// tree round r's rollouts start from) on a side stream, beside rounds r and r+1; after round r+1's
// commit the nodes those two rounds appended, [|T_r|, |T_{r+2}|), are searched and merged in
// (launch_nn_delta: every appended id is larger than every older one, so the merged lists equal a search
// over T_{r+2}).  A search thus has two rounds' time instead of one.  Three list sets rotate (this
// round's, round r+1's being merged, round r+2's being searched), three walk index sets (the one being
// searched by round r+1's walk, the one by round r+2's, the one being built for the next), and two side
// streams (round r+1's merge must not wait behind round r+2's walk).  Results are those of plain rounds.
struct LagSlot {
  clrrt_sample* d = nullptr;
  clrrt_sample* h = nullptr;
  int* cand = nullptr;
  float* ckey = nullptr;
  int* ncand = nullptr;
  int* ctie = nullptr;
  hipEvent_t ev = nullptr;  // recorded after its merge
  hipEvent_t evw = nullptr; // recorded after its walk (the merge waits for it on the merge stream)
  int n = 0;                // samples searched (0: none): this rank's slice
  int64_t g = 0;            // samples of the round (all ranks)
  int64_t tree_n = 0;       // size of the tree its walk searched
  int stream = 0;           // side stream index
  // nn_split_delta: the first partial search (the nodes of the commit after its walk's tree), its lists and events
  float* d1pk = nullptr;
  int* d1pi = nullptr;
  int d1_chunks = 0;
  int64_t d1_count = 0;     // nodes it covered ([tree_n, tree_n + d1_count)); 0: none
  hipEvent_t evd1 = nullptr;
  hipEvent_t evs = nullptr; // the samples are on the device
  // nn_delta_early: the appended-node search's caps taken after the walk's main grid, and the event recorded there
  float* wseed = nullptr;
  hipEvent_t evm = nullptr;
};

static int lag_alloc(clrrt_ctx* c) {
  if (c->side2) return CLRRT_OK;
  const int64_t B = c->cap.max_batch;
  HIPC(c, dalloc(&c->d_samples3, B));
  HIPC(c, dalloc(&c->cand3, B * CAND_K));
  HIPC(c, dalloc(&c->ckey3, B * CAND_K));
  HIPC(c, dalloc(&c->ncand3, B));
  HIPC(c, dalloc(&c->ctie3, B));
  HIPC(c, hipHostMalloc((void**)&c->h_samples3, sizeof(clrrt_sample) * B, hipHostMallocDefault));
  for (auto& e : c->ev_lag) HIPC(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : c->ev_lagw) HIPC(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (c->cu_split > 0) {  // the same CUs as the side stream
    const int nw = (c->n_cu + 31) / 32;
    std::vector<uint32_t> ms(nw, 0u);
    for (int i = 0; i < c->n_cu; i++)
      if ((i % 8) >= c->cu_split) ms[i / 32] |= 1u << (i % 32);
    HIPC(c, hipExtStreamCreateWithCUMask(&c->side2, (uint32_t)nw, ms.data()));
  } else {
    HIPC(c, hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking));
  }
  HIPC(c, hipStreamCreateWithFlags(&c->mst, hipStreamNonBlocking));
  HIPC(c, dalloc(&c->nn_seed2, B));
  for (int q = 0; q < 3; q++) {
    HIPC(c, dalloc(&c->d1pk[q], c->partial_cap));
    HIPC(c, dalloc(&c->wseed[q], B));
    if (q == 0) HIPC(c, dalloc(&c->nn_order, B));
    HIPC(c, hipEventCreateWithFlags(&c->ev_wm[q], hipEventDisableTiming));
    HIPC(c, dalloc(&c->d1pi[q], c->partial_cap));
    HIPC(c, hipEventCreateWithFlags(&c->ev_d1[q], hipEventDisableTiming));
    HIPC(c, hipEventCreateWithFlags(&c->ev_s[q], hipEventDisableTiming));
  }
  return CLRRT_OK;
}

// Stream priorities of the lag-2 rounds (option "stream_prio"): main and merge streams highest, the walk
// streams lowest (1), or all equal (0).  CU-masked streams (cu_split) keep theirs.  Scheduling only.
static int apply_stream_prio(clrrt_ctx* c) {
  const int want = (c->stream_prio ? 1 : 2) + 4 * c->walk_cu_reserve;  // 2: equal priorities
  if (c->stream_prio_applied == want || c->cu_split > 0) return CLRRT_OK;
  int lo = 0, hi = 0;
  HIPC(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
  // the priorities follow stream_prio alone (the CU reservation only masks the walk streams)
  const int p_hi = c->stream_prio ? hi : 0, p_lo = c->stream_prio ? lo : 0;
  HIPC(c, hipDeviceSynchronize());
  auto remake = [&](hipStream_t& st, int pr) -> int {
    if (st) HIPC(c, hipStreamDestroy(st));
    HIPC(c, hipStreamCreateWithPriority(&st, hipStreamNonBlocking, pr));
    return CLRRT_OK;
  };
  int rc;
  if (c->walk_cu_reserve > 0) {  // the walk streams on the CUs with (cu % 8) >= k (no priority on CU-masked streams)
    const int nw = (c->n_cu + 31) / 32;
    std::vector<uint32_t> ms(nw, 0u);
    for (int i = 0; i < c->n_cu; i++)
      if ((i % 8) >= c->walk_cu_reserve) ms[i / 32] |= 1u << (i % 32);
    for (hipStream_t* st : {&c->side, &c->side2}) {
      if (*st) HIPC(c, hipStreamDestroy(*st));
      HIPC(c, hipExtStreamCreateWithCUMask(st, (uint32_t)nw, ms.data()));
    }
    if ((rc = remake(c->mst, p_hi)) != CLRRT_OK) return rc;
  } else if ((!c->side_prio_set && (rc = remake(c->side, p_lo)) != CLRRT_OK) ||
             (rc = remake(c->side2, p_lo)) != CLRRT_OK || (rc = remake(c->mst, p_hi)) != CLRRT_OK) {
    return rc;  // (an explicit side_priority keeps the side stream it made)
  }
  if (c->own_stream && (rc = remake(c->stream, p_hi)) != CLRRT_OK) return rc;
  c->stream_prio_applied = want;
  return CLRRT_OK;
}

static int expand_lag2(clrrt_ctx* c, clrrt_rng* rng, int64_t n_iters, double budget_ms, int32_t batch,
                       clrrt_stats* out) {
  int rc = lag_alloc(c);
  if (rc == CLRRT_OK) rc = apply_stream_prio(c);
  if (rc == CLRRT_OK) rc = defer_begin(c, true);
  if (rc != CLRRT_OK) return rc;
  clrrt_stats st{};
  const auto t0 = std::chrono::steady_clock::now();
  clrrt_rng work = *rng, committed = *rng;
  std::deque<clrrt_sample> pending;
  const int cur = batch;  // samples per round, all ranks
  const bool sharded = c->sh.world > 1;
  c->sh.max_ms = 0;
  c->sh.nd_global = 0;
  c->sh.rows_stop = 0;
  shard_expansion_begin(c);
  if (sharded && (rc = shard_goal_reset(c)) != CLRRT_OK) return rc;
  const int64_t nodes_before = c->n_nodes;
  hipStream_t sides[2] = {c->side, c->side2};
  WalkBufs* W[3] = {&c->nnw, &c->nnw_alt, &c->nnw3};
  int64_t built_n[3] = {-1, -1, -1};  // the tree size each walk set's index was built for
  double built_f[3][7] = {};           // ... and its frame (fr.ox, fr.oy, fr.delta, x0, y0, x1, y1)
  // list sets: this round's (c->*), round r+1's (A) and round r+2's (B)
  LagSlot A, B;
  A.d = c->d_samples2; A.h = c->h_samples2; A.cand = c->cand2; A.ckey = c->ckey2; A.ncand = c->ncand2;
  A.ctie = c->ctie2; A.ev = c->ev_lag[0]; A.evw = c->ev_lagw[0];
  B.d = c->d_samples3; B.h = c->h_samples3; B.cand = c->cand3; B.ckey = c->ckey3; B.ncand = c->ncand3;
  B.ctie = c->ctie3; B.ev = c->ev_lag[1]; B.evw = c->ev_lagw[1];
  A.d1pk = c->d1pk[0]; A.d1pi = c->d1pi[0]; A.evd1 = c->ev_d1[0]; A.evs = c->ev_s[0];
  B.d1pk = c->d1pk[1]; B.d1pi = c->d1pi[1]; B.evd1 = c->ev_d1[1]; B.evs = c->ev_s[1];
  A.wseed = c->wseed[0]; A.evm = c->ev_wm[0];
  B.wseed = c->wseed[1]; B.evm = c->ev_wm[1];
  float* cur_wseed = c->wseed[2];
  hipEvent_t cur_evm = c->ev_wm[2];
  const bool early = c->nn_delta_early != 0;
  hipEvent_t cur_ev = c->ev_lag[2];  // the event of the set this round's lists are in
  hipEvent_t cur_evw = c->ev_lagw[2];
  float* cur_d1pk = c->d1pk[2];       // ... and that set's split-delta buffers and events
  int* cur_d1pi = c->d1pi[2];
  hipEvent_t cur_evd1 = c->ev_d1[2], cur_evs = c->ev_s[2];
  const bool split_delta = c->nn_split_delta != 0;
  // The three list sets rotate every round; whichever way the function is left (an error return of HIPC
  // included), the buffers the context's other paths use get their roles back: (d_samples, cand, ...) and
  // the *2 set are whichever two of the three sets, *3 the third, each freed once by free_all.
  struct RoleGuard {
    std::function<void()> f;
    ~RoleGuard() { f(); }
  } role_guard{[&]() {
    c->d_samples2 = A.d; c->h_samples2 = A.h; c->cand2 = A.cand; c->ckey2 = A.ckey; c->ncand2 = A.ncand; c->ctie2 = A.ctie;
    c->d_samples3 = B.d; c->h_samples3 = B.h; c->cand3 = B.cand; c->ckey3 = B.ckey; c->ncand3 = B.ncand; c->ctie3 = B.ctie;
    c->ev_lag[0] = A.ev; c->ev_lag[1] = B.ev; c->ev_lag[2] = cur_ev;
    c->ev_lagw[0] = A.evw; c->ev_lagw[1] = B.evw; c->ev_lagw[2] = cur_evw;
    c->nnw_built.n = -1;
    c->nnw.sorted_n = -1;
    c->nnw_alt.sorted_n = -1;
    c->nnw3.sorted_n = -1;
  }};
  bool have_cur = false;             // this round's lists come from slot A of the previous round
  int cur_stream = 0;
  double last_round_ms = 0;
  auto frame_of = [](const NnSetup& su, double* f) {
    f[0] = su.fr.ox; f[1] = su.fr.oy; f[2] = su.fr.delta; f[3] = su.x0; f[4] = su.y0; f[5] = su.x1; f[6] = su.y1;
  };
  // the index of the tree as it is now into walk set k (incremental from the set built before, if any)
  auto build = [&](int k, const NnSetup& su) -> int {
    double f[7];
    frame_of(su, f);
    if (built_n[k] == c->n_nodes && std::equal(f, f + 7, built_f[k])) return CLRRT_OK;
    int r2 = ensure_walk_set(c, *W[k]);
    if (r2 != CLRRT_OK) return r2;
    const WalkBufs* prev = nullptr;
    for (int q = 1; q <= 2 && !prev; q++) {
      const WalkBufs* w = W[(k + 3 - q) % 3];
      if (w->P && w->sorted_n > 0) prev = w;
    }
    KTimer kt(c, 0, c->stream);
    HIPC(c, launch_nn_walk_build(c->stream, c->nn, (int)c->n_nodes, su.fr, su.x0, su.y0, su.x1, su.y1, *W[k], prev));
    built_n[k] = c->n_nodes;
    std::copy(f, f + 7, built_f[k]);
    return CLRRT_OK;
  };
  // slot sl: the walk search of its n samples (host copy sl.h) over the current tree (walk set k)
  auto walk = [&](LagSlot& sl, int n, int k, const NnSetup& su, int si) -> int {
    hipStream_t s = sides[si];
    int r2 = ensure_walk_set(c, *W[k]);  // the configuration (budgets) for this tree size
    if (r2 != CLRRT_OK) return r2;
    c->nn_bf_keys += (int64_t)n * c->n_nodes;
    c->nn_samples += n;
    HIPC(c, hipStreamWaitEvent(s, c->ev_tree, 0));
    HIPC(c, hipMemcpyAsync(sl.d, sl.h, sizeof(clrrt_sample) * n, hipMemcpyHostToDevice, s));
    HIPC(c, hipEventRecord(sl.evs, s));  // (the split delta's first search reads them on mst)
    sl.d1_count = 0;
    sl.d1_chunks = 0;
    c->nn_super_bounds += (int64_t)n * walk_super_count(c->n_nodes);
    {
      KTimer kt(c, 0, s), kt3(c, 3, s);
      W[k]->seed_out = early ? sl.wseed : nullptr;
      W[k]->ev_main = early ? sl.evm : nullptr;
      const hipError_t ew = launch_nn_walk_search(s, sl.d, n, c->nn, (int)c->n_nodes, c->dp, su.fr, su.x0, su.y0, su.x1,
                                                  su.y1, *W[k], sl.cand, sl.ckey, sl.ncand, sl.ctie, c->work_ctr + 18,
                                                  c->nnw_stateless);
      W[k]->seed_out = nullptr;
      W[k]->ev_main = nullptr;
      HIPC(c, ew);
    }
    HIPC(c, hipEventRecord(sl.evw, s));
    sl.n = n;
    sl.tree_n = c->n_nodes;
    sl.stream = si;
    return CLRRT_OK;
  };
  auto draw_to = [&](int64_t want) {
    while ((int64_t)pending.size() < want) {
      clrrt_sample smp;
      clrrt_draw_samples(&c->params, &work, 1, &smp);
      pending.push_back(smp);
    }
  };
  for (int64_t k = 0; rc == CLRRT_OK; k++) {
    const auto tr0 = std::chrono::steady_clock::now();
    if (n_iters > 0 && st.iterations >= n_iters) break;
    const double ms0 = std::chrono::duration<double, std::milli>(tr0 - t0).count();
    // sharded: every rank decides on the largest elapsed time over the ranks (the same rounds everywhere)
    if (n_iters == 0 && !((sharded ? c->sh.max_ms : ms0) < budget_ms)) break;
    const int64_t left = n_iters > 0 ? n_iters - st.iterations : INT64_MAX;
    // gb samples this round over all ranks; this rank's slice [f0, f0 + nb)
    const int64_t gb = std::min<int64_t>(cur, left);
    int64_t f0 = 0;
    int nb = (int)gb;
    if (sharded) shard_slice(c, gb, &f0, &nb);
    c->sh.last_nb = nb;
    // (a commit also takes the deferred samples that resolve; sharded, the stop decision must be the same
    // on every rank: node counts only, the deferred samples bounded by the ring's rounds)
    const int64_t nc = gb + (sharded ? c->sh.nd_global : (int64_t)c->def.nd);
    if (c->n_nodes + 2 * nc > c->cap.max_nodes ||
        (sharded ? c->sh.rows_stop > 0 : c->n_rows + 2 * nc * (c->dp.n_steps_max + 1) > c->cap.max_rows)) {
      if (n_iters > 0) { rc = fail(c, CLRRT_ECAPACITY, "tree capacity exhausted"); break; }
      st.capacity_stop = 1;
      break;
    }
    const int wk = (int)(k % 3);
    const NnSetup su = nn_setup(c);
    const bool serve = c->n_nodes >= c->nnw_min_nodes && su.region_ok;
    // samples of rounds r+1 (slot A, unless already searched) and r+2 (slot B) to search this round (gA, gB
    // over all ranks; nA, nB this rank's slices)
    int64_t gA = 0, gB = 0, fA = 0, fB = 0;
    int nA = 0, nB = 0;
    if (serve) {
      const bool more = n_iters > 0 || ms0 + 2.0 * last_round_ms < budget_ms;
      if (A.n == 0 && (n_iters > 0 || ms0 + last_round_ms < budget_ms)) gA = std::max<int64_t>(0, std::min<int64_t>(cur, left - gb));
      const int64_t gA_eff = A.n > 0 ? A.g : gA;
      if (more && gA_eff > 0) gB = std::max<int64_t>(0, std::min<int64_t>(cur, left - gb - gA_eff));
      nA = (int)gA;
      nB = (int)gB;
      if (sharded) {
        shard_slice(c, gA, &fA, &nA);
        shard_slice(c, gB, &fB, &nB);
      }
    }
    const int64_t gA_all = A.n > 0 ? A.g : gA;
    draw_to(gb + gA_all + gB);
    // this round's lists
    if (have_cur) {
      KTimer kt(c, 4);  // the lists' wait (time the main stream stalls on the side streams)
      HIPC(c, hipStreamWaitEvent(c->stream, cur_ev, 0));
    } else {
      for (int j = 0; j < nb; j++) c->h_samples[j] = pending[f0 + j];
      HIPC(c, hipMemcpyAsync(c->d_samples, c->h_samples, sizeof(clrrt_sample) * nb, hipMemcpyHostToDevice, c->stream));
      if (serve) {
        // the side streams' work is done (a first pipelined round searches nothing ahead yet)
        HIPC(c, hipStreamSynchronize(c->side));
        HIPC(c, hipStreamSynchronize(c->side2));
        HIPC(c, hipStreamSynchronize(c->mst));
        if ((rc = build(wk, su)) != CLRRT_OK) break;
        c->nn_bf_keys += (int64_t)nb * c->n_nodes;
        c->nn_samples += nb;
        c->nn_super_bounds += (int64_t)nb * walk_super_count(c->n_nodes);
        KTimer kt(c, 0), kt3(c, 3);
        HIPC(c, launch_nn_walk_search(c->stream, c->d_samples, nb, c->nn, (int)c->n_nodes, c->dp, su.fr, su.x0, su.y0,
                                      su.x1, su.y1, *W[wk], c->cand, c->ckey, c->ncand, c->ctie, c->work_ctr + 18,
                                      c->nnw_stateless));
      } else if ((rc = run_nn(c, nb, nullptr)) != CLRRT_OK) {
        break;
      }
    }
    if (serve && (nA > 0 || nB > 0) && (rc = build(wk, su)) != CLRRT_OK) break;
    // searches ahead, beside this round's rollouts: slot A's (bootstrap) then slot B's; B on the other
    // side stream than A, except when both search this round's index (the walk set's sample scratch
    // is shared: one stream)
    auto ahead = [&]() -> int {
      if (nA > 0) {
        for (int j = 0; j < nA; j++) A.h[j] = pending[gb + fA + j];
        const int r2 = walk(A, nA, wk, su, cur_stream);
        if (r2 != CLRRT_OK) return r2;
        A.g = gA;
      }
      if (nB > 0) {
        for (int j = 0; j < nB; j++) B.h[j] = pending[gb + gA_all + fB + j];
        const int r2 = walk(B, nB, wk, su, nA > 0 ? A.stream : 1 - A.stream);
        if (r2 != CLRRT_OK) return r2;
        B.g = gB;
      }
      return CLRRT_OK;
    };
    int L = nb, nn = 0, n_app = 0;
    if ((rc = eval_samples(c, nb, false, &L, true, (nA > 0 || nB > 0) ? std::function<int()>(ahead) : nullptr,
                           nullptr)) != CLRRT_OK)
      break;
    if ((rc = compact_and_copy(c, L, &nn, true)) != CLRRT_OK) break;
    const double ms_commit = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((rc = commit_round(c, nn, ms_commit, &n_app)) != CLRRT_OK) break;
    // slot A: merge the nodes appended since its walk's tree
    if ((A.n > 0 || (split_delta && B.n > 0)))
      HIPC(c, hipEventRecord(c->ev_commit, c->stream));
    if (A.n > 0 && split_delta) {
      // the nodes its first partial search did not cover (this commit's), their key caps seeded from its walk list;
      // then the walk list, the first partial lists and these are merged
      hipStream_t s = c->mst;
      HIPC(c, hipStreamWaitEvent(s, c->ev_commit, 0));
      HIPC(c, hipStreamWaitEvent(s, early ? A.evm : A.evw, 0));
      const int64_t first2 = A.tree_n + A.d1_count, cnt2 = c->n_nodes - first2;
      int nch2 = 0;
      if (cnt2 > 0) {
        KTimer kt(c, 0, s);
        c->nn_bf_keys += (int64_t)A.n * cnt2;
        const NnSetup su2 = nn_setup(c);
        const int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)A.n * NN_K));
        HIPC(c, launch_nn_delta_partial(s, A.d, A.n, c->nn, (int)first2, (int)cnt2, c->dp, su2.fr, c->pk, c->pi,
                                        max_chunks, A.ckey, A.ncand, early ? A.wseed : c->nn_seed, early,
                                        c->nn_lane_order ? c->nn_order : nullptr, &nch2));
      }
      if (early) HIPC(c, hipStreamWaitEvent(s, A.evw, 0));
      if (A.d1_count > 0) HIPC(c, hipStreamWaitEvent(s, A.evd1, 0));
      {
        KTimer kt(c, 0, s);
        if (A.d1_count > 0)
          HIPC(c, launch_nn_delta_merge(s, A.n, A.d1_chunks, c->dp, A.d1pk, A.d1pi, (int)A.tree_n, A.cand, A.ckey,
                                        A.ncand, A.ctie));
        HIPC(c, launch_nn_delta_merge(s, A.n, nch2, c->dp, c->pk, c->pi, (int)first2, A.cand, A.ckey, A.ncand, A.ctie));
      }
      HIPC(c, hipEventRecord(A.ev, s));
    } else if (A.n > 0 && early) {
      // behind the commit and slot A's main walk grid (caps from its k_walk_seed), beside the walk's overflow split;
      // the merge behind the whole walk
      hipStream_t s = c->mst;
      HIPC(c, hipStreamWaitEvent(s, c->ev_commit, 0));
      HIPC(c, hipStreamWaitEvent(s, A.evm, 0));
      const int64_t first = A.tree_n, cnt = c->n_nodes - A.tree_n;
      int nch = 0;
      if (cnt > 0) {
        KTimer kt(c, 0, s);
        c->nn_bf_keys += (int64_t)A.n * cnt;
        const NnSetup su2 = nn_setup(c);
        const int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)A.n * NN_K));
        HIPC(c, launch_nn_delta_partial(s, A.d, A.n, c->nn, (int)first, (int)cnt, c->dp, su2.fr, c->pk, c->pi,
                                        max_chunks, nullptr, nullptr, A.wseed, true,
                                        c->nn_lane_order ? c->nn_order : nullptr, &nch));
      }
      HIPC(c, hipStreamWaitEvent(s, A.evw, 0));
      {
        KTimer kt(c, 0, s);
        HIPC(c, launch_nn_delta_merge(s, A.n, nch, c->dp, c->pk, c->pi, (int)first, A.cand, A.ckey, A.ncand, A.ctie));
      }
      HIPC(c, hipEventRecord(A.ev, s));
    } else if (A.n > 0) {
      hipStream_t s = c->mst;  // behind the commit and slot A's walk
      HIPC(c, hipStreamWaitEvent(s, c->ev_commit, 0));
      HIPC(c, hipStreamWaitEvent(s, A.evw, 0));
      const int64_t first = A.tree_n, cnt = c->n_nodes - A.tree_n;
      if (cnt > 0) {
        KTimer kt(c, 0, s);
        c->nn_bf_keys += (int64_t)A.n * cnt;
        const NnSetup su2 = nn_setup(c);
        const int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)A.n * NN_K));
        HIPC(c, launch_nn_delta(s, A.d, A.n, c->nn, (int)first, (int)cnt, c->dp, su2.fr, c->pk, c->pi, max_chunks,
                                A.cand, A.ckey, A.ncand, A.ctie, c->nn_seed));
      }
      HIPC(c, hipEventRecord(A.ev, s));
    }
    // slot B (split delta): this commit's nodes, searched for the round-after-next's samples beside the next
    // round's rollouts (merged into B's list after the next commit, when B is slot A); behind slot A's merges
    if (split_delta && B.n > 0) {
      hipStream_t s2 = c->mst;
      HIPC(c, hipStreamWaitEvent(s2, c->ev_commit, 0));
      HIPC(c, hipStreamWaitEvent(s2, B.evs, 0));
      HIPC(c, hipStreamWaitEvent(s2, early ? B.evm : B.evw, 0));  // (its walk list seeds the key caps)
      const int64_t cnt1 = c->n_nodes - B.tree_n;
      B.d1_count = cnt1;
      B.d1_chunks = 0;
      if (cnt1 > 0) {
        KTimer kt(c, 0, s2);
        c->nn_bf_keys += (int64_t)B.n * cnt1;
        const NnSetup su1 = nn_setup(c);
        const int max_chunks = (int)std::max<int64_t>(1, c->partial_cap / ((int64_t)B.n * NN_K));
        HIPC(c, launch_nn_delta_partial(s2, B.d, B.n, c->nn, (int)B.tree_n, (int)cnt1, c->dp, su1.fr, B.d1pk, B.d1pi,
                                        max_chunks, B.ckey, B.ncand, early ? B.wseed : c->nn_seed2, early,
                                        c->nn_lane_order ? c->nn_order : nullptr, &B.d1_chunks));
      }
      HIPC(c, hipEventRecord(B.evd1, s2));
    }
    // the next round's index (the walk of round r+3's samples searches it)
    {
      const NnSetup sn = nn_setup(c);
      if (B.n > 0 && c->n_nodes >= c->nnw_min_nodes && sn.region_ok && (rc = build((int)((k + 1) % 3), sn)) != CLRRT_OK)
        break;
    }
    for (int64_t j = 0; j < gb; j++) {
      pending.pop_front();
      for (int q = 0; q < 3; q++) clrrt_rng_next(&committed);
    }
    st.iterations += gb;
    st.goal_nodes_added += c->last_goal_nodes;
    st.speculated += gb;
    st.rounds++;
    // rotate: A becomes this round's set, B slot A, this round's set slot B
    {
      LagSlot old;
      old.d = c->d_samples; old.h = c->h_samples; old.cand = c->cand; old.ckey = c->ckey; old.ncand = c->ncand;
      old.ctie = c->ctie; old.ev = cur_ev; old.evw = cur_evw; old.stream = cur_stream;
      old.d1pk = cur_d1pk; old.d1pi = cur_d1pi; old.evd1 = cur_evd1; old.evs = cur_evs;
      old.wseed = cur_wseed; old.evm = cur_evm;
      have_cur = A.n > 0;
      c->d_samples = A.d; c->h_samples = A.h; c->cand = A.cand; c->ckey = A.ckey; c->ncand = A.ncand; c->ctie = A.ctie;
      cur_ev = A.ev;
      cur_evw = A.evw;
      cur_stream = A.stream;
      cur_d1pk = A.d1pk; cur_d1pi = A.d1pi; cur_evd1 = A.evd1; cur_evs = A.evs;
      cur_wseed = A.wseed; cur_evm = A.evm;
      A = B;
      B = old;
      B.n = 0;
      B.stream = 1 - A.stream;
    }
    last_round_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count();
  }
  // the deferred samples still pending and the last round's accepted rows (part of the query's output
  // tree, so inside its time)
  if (rc == CLRRT_OK) rc = defer_drain(c, &st.goal_nodes_added);
  st.deferred = c->def.deferred_total;
  if (rc == CLRRT_OK) rc = flush_replays(c);
  if (rc == CLRRT_OK && sharded) rc = shard_goal_count(c, &st.goal_nodes_added);
  rc = shard_expansion_end(c, rc);  // the closing exchange (sharded): every rank learns of any rank's failure
  c->def.active = false;
  for (hipStream_t s : {c->side, c->side2, c->mst, c->stream}) {  // every stream drained, the first error kept
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess && rc == CLRRT_OK) rc = fail(c, CLRRT_EHIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  }
  st.nodes_added = c->n_nodes - nodes_before;
  st.elapsed_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *rng = committed;
  if (out) *out = st;
  return rc;
}

int clrrt_expand(clrrt_ctx* c, clrrt_rng* rng, int64_t n_iters, double budget_ms, int32_t mode, int32_t batch,
                 clrrt_stats* out) {
  if (!c || !rng || n_iters < 0 || (mode != CLRRT_MODE_EXACT && mode != CLRRT_MODE_BATCH)) return CLRRT_EINVAL;
  pf_reset(c);
  if (n_iters == 0 && !(budget_ms > 0)) return CLRRT_EINVAL;
  if (c->n_nodes <= 0) return fail(c, CLRRT_ESTATE, "tree not initialised");
  c->round_sizes.clear();
  const bool sharded = c->sh.world > 1;
  if (sharded && mode != CLRRT_MODE_BATCH) return fail(c, CLRRT_EINVAL, "sharded expansion runs BATCH rounds only");
  HIPC(c, hipSetDevice(c->device));
  // samples per round (all ranks when sharded: each rank's slice must fit max_batch)
  const int64_t bmax = (int64_t)c->cap.max_batch * c->sh.world;
  batch = (int32_t)std::max<int64_t>(1, std::min<int64_t>(batch > 0 ? batch : bmax, bmax));
  if (sharded && batch < c->sh.world) return fail(c, CLRRT_EINVAL, "fewer samples per round than ranks");
  const int lag = c->nn_lag ? c->nn_lag
                  : (n_iters == 0 ? budget_ms >= 1000.0 : n_iters >= 64 * (int64_t)batch) ? 2 : 1;
  if (mode == CLRRT_MODE_BATCH && c->nn_pipeline && lag == 2) return expand_lag2(c, rng, n_iters, budget_ms, batch, out);
  clrrt_stats st{};
  auto t0 = std::chrono::steady_clock::now();
  clrrt_rng work = *rng;       // draws ahead (speculative samples)
  clrrt_rng committed = *rng;  // state after exactly `iterations` iterations
  std::deque<clrrt_sample> pending;
  const bool exact = mode == CLRRT_MODE_EXACT;
  int cur = exact ? std::min(batch, std::max(16, c->exact_min_width)) : batch;
  int64_t nodes_before = c->n_nodes;
  int rc = defer_begin(c, !exact);
  c->sh.max_ms = 0;
  c->sh.nd_global = 0;
  c->sh.rows_stop = 0;
  shard_expansion_begin(c);
  if (rc == CLRRT_OK && sharded) rc = shard_goal_reset(c);
  bool have_next = false;  // this round's samples and lists were prepared by the previous round
  double last_round_ms = 0;
  auto draw_to = [&](int64_t want) {
    while ((int64_t)pending.size() < want) {
      clrrt_sample smp;
      clrrt_draw_samples(&c->params, &work, 1, &smp);
      pending.push_back(smp);
    }
  };
  for (; rc == CLRRT_OK;) {
    const auto tr0 = std::chrono::steady_clock::now();
    if (n_iters > 0 && st.iterations >= n_iters) break;
    if (n_iters == 0) {
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      // sharded: every rank decides on the largest elapsed time over the ranks (the same rounds everywhere)
      if (!((sharded ? c->sh.max_ms : ms) < budget_ms)) break;
    }
    // gb samples this round over all ranks; this rank's slice [f0, f0 + nb)
    int64_t gb = cur;
    if (n_iters > 0) gb = std::min<int64_t>(gb, n_iters - st.iterations);
    int64_t f0 = 0;
    int nb = (int)gb;
    if (sharded) shard_slice(c, gb, &f0, &nb);
    c->sh.last_nb = nb;
    // a round appends at most 2 nodes and 2 full-horizon trajectories per sample (+ the deferred samples;
    // sharded, the same decision on every rank: node counts only, deferred samples bounded by the ring)
    const int64_t nc = gb + (sharded ? c->sh.nd_global : (int64_t)c->def.nd);
    if (c->n_nodes + 2 * nc > c->cap.max_nodes ||
        (sharded ? c->sh.rows_stop > 0 : c->n_rows + 2 * nc * (c->dp.n_steps_max + 1) > c->cap.max_rows)) {
      if (n_iters > 0) { rc = fail(c, CLRRT_ECAPACITY, "tree capacity exhausted"); break; }
      st.capacity_stop = 1;
      break;
    }
    draw_to(gb);
    if (!have_next) {
      for (int j = 0; j < nb; j++) c->h_samples[j] = pending[f0 + j];
      HIPC(c, hipMemcpyAsync(c->d_samples, c->h_samples, sizeof(clrrt_sample) * nb, hipMemcpyHostToDevice, c->stream));
    }
    // Pipelined BATCH rounds: the next round's samples are known now (BATCH rounds commit every
    // sample), so their walk search over this round's tree runs on the side stream while this round's
    // rollouts run (the rollout kernel's last waves leave most CUs idle); after the commit, the nodes
    // this round appended are searched and merged in (launch_nn_delta).  The lists equal a search over
    // the committed tree, so the rounds' results are unchanged.
    int64_t gb2 = 0, f2 = 0;
    int nb2 = 0;
    NnSetup su{};
    if (!exact && c->nn_pipeline) {
      gb2 = cur;
      if (n_iters > 0) gb2 = std::max<int64_t>(0, std::min<int64_t>(gb2, n_iters - st.iterations - gb));
      if (n_iters == 0) {
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (!(ms + last_round_ms < budget_ms)) gb2 = 0;  // this is probably the last round
      }
      nb2 = (int)gb2;
      if (sharded) shard_slice(c, gb2, &f2, &nb2);
      if (nb2 > 0) {
        su = nn_setup(c);
        if (!walk_serves(c, su)) nb2 = 0;
      }
    }
    auto prefetch = [&]() -> int {
      draw_to(gb + gb2);
      for (int j = 0; j < nb2; j++) c->h_samples2[j] = pending[gb + f2 + j];
      return launch_side_walk(c, nb2, su);
    };
    int L = nb, nn = 0, n_app = 0;
    auto build = [&]() -> int { return pre_roll_build(c, su); };
    if ((rc = eval_samples(c, nb, exact, &L, have_next, nb2 > 0 ? std::function<int()>(prefetch) : nullptr,
                           nb2 > 0 ? std::function<int()>(build) : nullptr)) != CLRRT_OK)
      break;
    if (!exact) {
      // BATCH rounds commit every sample, so the next round's samples are known now: draw them
      // while the GPU evaluates this round (the draw is ~0.05 us per sample on the host)
      int64_t want = gb + (int64_t)cur;
      if (n_iters > 0) want = std::min<int64_t>(want, n_iters - st.iterations);
      draw_to(want);
    }
    if ((rc = compact_and_copy(c, L, &nn, true)) != CLRRT_OK) break;
    const int64_t first_new = c->n_nodes;
    const double ms_commit = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((rc = commit_round(c, nn, ms_commit, &n_app)) != CLRRT_OK) break;
    have_next = false;
    if (nb2 > 0) {
      if ((rc = side_delta_launch(c, nb2, first_new, n_app)) != CLRRT_OK) break;
      if (c->nnw_double && (rc = next_round_build(c)) != CLRRT_OK) break;
      if ((rc = side_lists_join(c)) != CLRRT_OK) break;
      have_next = true;
    }
    // iterations consumed: the committed prefix (EXACT) or the whole round (BATCH, every rank's samples)
    const int64_t used = exact ? L : gb;
    for (int64_t j = 0; j < used; j++) {
      pending.pop_front();
      for (int k = 0; k < 3; k++) clrrt_rng_next(&committed);
    }
    st.iterations += used;
    st.goal_nodes_added += c->last_goal_nodes;
    st.speculated += exact ? nb : gb;
    st.rounds++;
    if (exact) cur = std::max(c->exact_min_width, std::min(batch, L == nb ? 2 * nb : 2 * L));
    last_round_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count();
  }
  // the deferred samples still pending and the last round's accepted rows (part of the query's output
  // tree, so inside its time)
  if (rc == CLRRT_OK) rc = defer_drain(c, &st.goal_nodes_added);
  st.deferred = c->def.deferred_total;
  if (rc == CLRRT_OK) rc = flush_replays(c);
  if (rc == CLRRT_OK && sharded) rc = shard_goal_count(c, &st.goal_nodes_added);
  rc = shard_expansion_end(c, rc);  // the closing exchange (sharded): every rank learns of any rank's failure
  c->def.active = false;
  HIPC(c, hipStreamSynchronize(c->side));
  HIPC(c, hipStreamSynchronize(c->stream));
  st.nodes_added = c->n_nodes - nodes_before;
  st.elapsed_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *rng = committed;
  if (out) *out = st;
  return rc;
}

int clrrt_set_shards(clrrt_ctx* c, int32_t rank, int32_t world, void* dev_local, int32_t cap_local,
                     clrrt_exchange_fn exchange, void* user) {
  if (!c || world < 1 || rank < 0 || rank >= world) return CLRRT_EINVAL;
  if (world > 1 && (!dev_local || cap_local <= 0 || !exchange)) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  auto& h = c->sh;
  h.rank = rank;
  h.world = world;
  h.dev_local = world > 1 ? dev_local : nullptr;
  h.cap_local = world > 1 ? cap_local : 0;
  h.fn = world > 1 ? exchange : nullptr;
  h.user = world > 1 ? user : nullptr;
  c->rank = rank;  // owner of this rank's records
  if (world > 1 && !h.d_goal) HIPC(c, dalloc(&h.d_goal, 1));
  return CLRRT_OK;
}

int clrrt_rollout_batch(clrrt_ctx* c, const clrrt_rollout_job* jobs, int32_t n, clrrt_rollout_result* out,
                        double* rows_out, int32_t rows_cap) {
  if (!c || n < 0 || (n > 0 && (!jobs || !out))) return CLRRT_EINVAL;
  pf_reset(c);
  if (rows_out && rows_cap < c->dp.n_steps_max + 1) return fail(c, CLRRT_EINVAL, "rows_cap < max steps + 1");
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  for (int j = 0; j < n; j++)
    if (jobs[j].parent < 0 || jobs[j].parent >= c->n_nodes) return fail(c, CLRRT_EINVAL, "job parent out of range");
  std::vector<Job> hj(n);
  for (int j = 0; j < n; j++) {
    hj[j].parent = jobs[j].parent; hj[j].from_reg = 0; hj[j].gb = jobs[j].gb; hj[j].pad = 0;
    hj[j].sx = jobs[j].sample[0]; hj[j].sy = jobs[j].sample[1];
    hj[j].row_off = rows_out ? (int64_t)j * rows_cap : -1;
  }
  Job* dj = nullptr;
  RollRes* dr = nullptr;
  double* drows = nullptr;
  hipError_t e = hipMalloc((void**)&dj, sizeof(Job) * n);
  if (e == hipSuccess) e = hipMalloc((void**)&dr, sizeof(RollRes) * n);
  if (e == hipSuccess && rows_out) e = hipMalloc((void**)&drows, sizeof(double) * 10 * (size_t)rows_cap * n);
  if (e == hipSuccess) e = hipMemcpyAsync(dj, hj.data(), sizeof(Job) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    RollArgs a = roll_args(c, n);
    a.jobs = dj;
    a.arena = drows;
    a.res = dr;
    KTimer kt(c, 1);
    e = launch_rollout(c->stream, SRC_LIST, a);
  }
  std::vector<RollRes> hr(n);
  if (e == hipSuccess) e = hipMemcpyAsync(hr.data(), dr, sizeof(RollRes) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && rows_out)
    e = hipMemcpyAsync(rows_out, drows, sizeof(double) * 10 * (size_t)rows_cap * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(dj);
  hipFree(dr);
  if (drows) hipFree(drows);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("rollout_batch: ") + hipGetErrorString(e));
  for (int j = 0; j < n; j++) {
    clrrt_rollout_result& o = out[j];
    memset(&o, 0, sizeof(o));
    o.outcome = hr[j].outcome;
    o.nrows = hr[j].nrows;
    o.costE = hr[j].costE;
    o.costS = hr[j].costS;
    for (int k = 0; k < 10; k++) o.final_state[k] = hr[j].st[k];
    o.ref_back[0] = hr[j].bx; o.ref_back[1] = hr[j].by;
    o.ref_vback = hr[j].vback;
    o.ref_n = hr[j].refN;
  }
  return CLRRT_OK;
}

int clrrt_simulate(clrrt_ctx* c, const clrrt_sim_case* cases, int32_t n, clrrt_rollout_result* out, double* rows_out,
                   int32_t rows_cap, double* ref_out, int32_t ref_cap) {
  if (!c || n < 0 || (n > 0 && (!cases || !out)) || (ref_out && ref_cap <= 0)) return CLRRT_EINVAL;
  pf_reset(c);
  if (rows_out && rows_cap < c->dp.n_steps_max + 1) return fail(c, CLRRT_EINVAL, "rows_cap < max steps + 1");
  for (int j = 0; j < n; j++)
    if (!cases[j].goal_biased && cases[j].ref_n < 1) return fail(c, CLRRT_EINVAL, "ref_n < 1");
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  std::vector<SimJob> hj(n);
  for (int j = 0; j < n; j++) {
    const clrrt_sim_case& q = cases[j];
    SimJob& s = hj[j];
    for (int k = 0; k < 10; k++) s.st[k] = q.state[k];
    s.ax = q.ax; s.ay = q.ay; s.hx = q.hx; s.hy = q.hy; s.vstart = q.vstart;
    s.n = q.ref_n; s.gb = q.goal_biased ? 1 : 0;
    s.row_off = rows_out ? (int64_t)j * rows_cap : -1;
    s.ref_off = ref_out ? (int64_t)j * 3 * ref_cap : -1;
  }
  SimJob* dj = nullptr;
  RollRes* dr = nullptr;
  double *drows = nullptr, *dref = nullptr;
  hipError_t e = hipMalloc((void**)&dj, sizeof(SimJob) * n);
  if (e == hipSuccess) e = hipMalloc((void**)&dr, sizeof(RollRes) * n);
  if (e == hipSuccess && rows_out) e = hipMalloc((void**)&drows, sizeof(double) * 10 * (size_t)rows_cap * n);
  if (e == hipSuccess && ref_out) e = hipMalloc((void**)&dref, sizeof(double) * 3 * (size_t)ref_cap * n);
  if (e == hipSuccess) e = hipMemcpyAsync(dj, hj.data(), sizeof(SimJob) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    RollArgs a = roll_args(c, n);
    a.sims = dj;
    a.arena = drows;
    a.refv = dref;
    a.ref_cap = ref_cap;
    a.res = dr;
    KTimer kt(c, 1);
    e = launch_rollout(c->stream, SRC_EXPL, a);
  }
  std::vector<RollRes> hr(n);
  if (e == hipSuccess) e = hipMemcpyAsync(hr.data(), dr, sizeof(RollRes) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && rows_out)
    e = hipMemcpyAsync(rows_out, drows, sizeof(double) * 10 * (size_t)rows_cap * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && ref_out)
    e = hipMemcpyAsync(ref_out, dref, sizeof(double) * 3 * (size_t)ref_cap * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(dj);
  hipFree(dr);
  if (drows) hipFree(drows);
  if (dref) hipFree(dref);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("simulate: ") + hipGetErrorString(e));
  for (int j = 0; j < n; j++) {
    clrrt_rollout_result& o = out[j];
    memset(&o, 0, sizeof(o));
    o.outcome = hr[j].outcome;
    o.nrows = hr[j].nrows;
    o.costE = hr[j].costE;
    o.costS = hr[j].costS;
    for (int k = 0; k < 10; k++) o.final_state[k] = hr[j].st[k];
    o.ref_back[0] = hr[j].bx; o.ref_back[1] = hr[j].by;
    o.ref_vback = hr[j].vback;
    o.ref_n = hr[j].refN;
  }
  return CLRRT_OK;
}

int clrrt_selftest_math(clrrt_ctx* c, int32_t fn, const double* a, const double* b, int32_t n, double* out) {
  if (!c || n < 0 || (n > 0 && (!a || !b || !out)) || fn < 0 || fn > 28) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  double *da = nullptr, *db = nullptr, *dout = nullptr;
  hipError_t e = hipMalloc((void**)&da, sizeof(double) * n);
  if (e == hipSuccess) e = hipMalloc((void**)&db, sizeof(double) * n);
  if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(double) * n);
  if (e == hipSuccess) e = hipMemcpyAsync(da, a, sizeof(double) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(db, b, sizeof(double) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = launch_selftest_math(c->stream, fn, da, db, n, dout);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(da);
  hipFree(db);
  hipFree(dout);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("selftest_math: ") + hipGetErrorString(e));
  return CLRRT_OK;
}

int clrrt_obstacle_distance(clrrt_ctx* c, const double* states, int32_t n, double* out) {
  if (!c || n < 0 || (n > 0 && (!states || !out))) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  double *din = nullptr, *dout = nullptr;
  hipError_t e = hipMalloc((void**)&din, sizeof(double) * 10 * (size_t)n);
  if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(double) * (size_t)n);
  if (e == hipSuccess) e = hipMemcpyAsync(din, states, sizeof(double) * 10 * (size_t)n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = launch_obs_distance(c->stream, c->dp, c->obs, din, n, dout);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(din);
  hipFree(dout);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("obstacle_distance: ") + hipGetErrorString(e));
  return CLRRT_OK;
}

int clrrt_selftest_units(clrrt_ctx* c, int32_t unit, const double* in, int32_t n, double* out) {
  const int K = CLRRT_UNIT_CTRL_K;
  static const int kin[10] = {11, 9, 9, 12, 2, 6, 7, 8, 8, 12 + 6 * K};
  static const int kout[10] = {1, 8, 1, 1 + 3 * CLRRT_UNIT_PROFILE_NMAX, 2, 2, 3, 1, 1 + 3 * CLRRT_UNIT_PROFILE_NMAX,
                               4 + 8 * K};
  if (!c || n < 0 || (n > 0 && (!in || !out)) || unit < 0 || unit > CLRRT_UNIT_CTRL) return CLRRT_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  const size_t nin = (size_t)kin[unit] * n, nout = (size_t)kout[unit] * n;
  std::vector<BakedObs> baked;
  if (unit == CLRRT_UNIT_OBB) {
    baked.resize(n);
    for (int i = 0; i < n; i++) {
      const double* a = in + 11 * (size_t)i;
      clrrt_obstacle o = {a[4], a[5], a[6], a[7], a[8], a[9], a[10]};
      bake_obstacle(o, baked[i]);
    }
  }
  // per-case parameters: the context's, with the case's goal / vmax / ref_res, derived as
  // clrrt_set_params derives them
  std::vector<DevParams> cps;
  if (unit >= CLRRT_UNIT_FEASIBLE) {
    cps.resize(n);
    for (int i = 0; i < n; i++) {
      const double* a = in + (size_t)kin[unit] * i;
      clrrt_params q = c->params;
      if (unit == CLRRT_UNIT_FEASIBLE) q.ref_res = a[6];
      if (unit == CLRRT_UNIT_GOALBIAS) for (int k = 0; k < 4; k++) q.goal[k] = a[k];
      if (unit == CLRRT_UNIT_GOALREF) { for (int k = 0; k < 4; k++) q.goal[k] = a[k]; q.ref_res = a[7]; }
      if (unit == CLRRT_UNIT_CTRL) { for (int k = 0; k < 4; k++) q.goal[k] = a[5 + k]; q.vmax = a[10]; q.ref_res = a[11]; }
      derive(q, cps[i], c->n_obs);
    }
  }
  double *din = nullptr, *dout = nullptr;
  BakedObs* dobs = nullptr;
  DevParams* dcp = nullptr;
  hipError_t e = hipMalloc((void**)&din, sizeof(double) * nin);
  if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(double) * nout);
  if (e == hipSuccess && !baked.empty()) e = hipMalloc((void**)&dobs, sizeof(BakedObs) * baked.size());
  if (e == hipSuccess && !cps.empty()) e = hipMalloc((void**)&dcp, sizeof(DevParams) * cps.size());
  if (e == hipSuccess) e = hipMemcpyAsync(din, in, sizeof(double) * nin, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && dobs)
    e = hipMemcpyAsync(dobs, baked.data(), sizeof(BakedObs) * baked.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && dcp)
    e = hipMemcpyAsync(dcp, cps.data(), sizeof(DevParams) * cps.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(dout, 0, sizeof(double) * nout, c->stream);
  if (e == hipSuccess) e = launch_selftest_units(c->stream, unit, din, dobs, n, c->dp, dcp, dout);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double) * nout, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(din);
  hipFree(dout);
  if (dobs) hipFree(dobs);
  if (dcp) hipFree(dcp);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("selftest_units: ") + hipGetErrorString(e));
  return CLRRT_OK;
}

int clrrt_nn_batch(clrrt_ctx* c, const clrrt_sample* samples, int32_t n, int32_t mode, int32_t* out_ids,
                   float* out_keys) {
  if (!c || n < 0 || (n > 0 && (!samples || !out_ids))) return CLRRT_EINVAL;
  pf_reset(c);
  if (mode != CLRRT_MODE_EXACT && mode != CLRRT_MODE_BATCH) return CLRRT_EINVAL;
  if (n > c->cap.max_batch) return fail(c, CLRRT_ECAPACITY, "batch larger than max_batch");
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  memcpy(c->h_samples, samples, sizeof(clrrt_sample) * n);
  HIPC(c, hipMemcpyAsync(c->d_samples, c->h_samples, sizeof(clrrt_sample) * n, hipMemcpyHostToDevice, c->stream));
  int rc = CLRRT_OK;
  if (mode == CLRRT_MODE_EXACT && (rc = ensure_sort_scratch(c, (int64_t)n * c->n_nodes)) != CLRRT_OK) return rc;
  if ((rc = run_nn(c, n, mode == CLRRT_MODE_EXACT ? c->sort_scratch : nullptr)) != CLRRT_OK) return rc;
  HIPC(c, hipMemcpyAsync(out_ids, c->cand, sizeof(int) * CAND_K * n, hipMemcpyDeviceToHost, c->stream));
  if (out_keys)
    HIPC(c, hipMemcpyAsync(out_keys, c->ckey, sizeof(float) * CAND_K * n, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return CLRRT_OK;
}

int clrrt_round_sizes(clrrt_ctx* c, int64_t* out, int64_t cap, int64_t* n) {
  if (!c || cap < 0 || (cap > 0 && !out)) return CLRRT_EINVAL;
  const int64_t m = (int64_t)c->round_sizes.size();
  for (int64_t i = 0; i < std::min(m, cap); i++) out[i] = c->round_sizes[(size_t)i];
  if (n) *n = m;
  return CLRRT_OK;
}

int clrrt_walk_audit(clrrt_ctx* c, const clrrt_sample* samples, int32_t n, int32_t* out) {
  if (!c || n < 0 || (n > 0 && (!samples || !out))) return CLRRT_EINVAL;
  pf_reset(c);
  if (n > c->cap.max_batch) return fail(c, CLRRT_ECAPACITY, "batch larger than max_batch");
  HIPC(c, hipSetDevice(c->device));
  if (n == 0) return CLRRT_OK;
  const NnSetup su = nn_setup(c);
  if (!walk_serves(c, su)) return fail(c, CLRRT_ESTATE, "the walk does not serve this tree (too small or no region)");
  int rc = ensure_walk(c);
  if (rc != CLRRT_OK) return rc;
  memcpy(c->h_samples, samples, sizeof(clrrt_sample) * n);
  HIPC(c, hipMemcpyAsync(c->d_samples, c->h_samples, sizeof(clrrt_sample) * n, hipMemcpyHostToDevice, c->stream));
  c->nnw_built.n = -1;
  HIPC(c, launch_nn_walk_build(c->stream, c->nn, (int)c->n_nodes, su.fr, su.x0, su.y0, su.x1, su.y1, c->nnw));
  int* d_out = nullptr;
  HIPC(c, hipMalloc(&d_out, sizeof(int32_t) * 20 * (size_t)n));
  hipError_t e = launch_walk_audit(c->stream, c->d_samples, n, c->nn, (int)c->n_nodes, c->dp, su.fr, c->nnw, d_out);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, sizeof(int32_t) * 20 * (size_t)n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(d_out);
  if (e != hipSuccess) return fail(c, CLRRT_EHIP, std::string("clrrt_walk_audit: ") + hipGetErrorString(e));
  return CLRRT_OK;
}

}  // extern "C"
