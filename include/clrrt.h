/*
 * clrrt.h — C-ABI of libclrrt, the MI355X (gfx950) closed-loop RRT tree-expansion engine.
 *
 * This is the drop-in boundary for the reference's `expandTree` hot path (vdBerg93/cl-rrt).
 * Every entry point is extern "C", takes plain pointers and sizes, and returns an int
 * status (0 = ok, <0 = error; the message is available from clrrt_last_error()).
 *
 * Reference interfaces each entry point replaces (paths relative to the reference root):
 *   clrrt_params_default   <- updateParameters() rrt/src/rrt_node.cpp:28-38, parameters.launch:3-20,
 *                             Vehicle::setPrius rrt/include/rrt/vehicle.h:39-60,
 *                             MyRRT::MyRRT Wcost rrt/src/rrtplanner.cpp:12-19,
 *                             updateReferenceResolution rrt/src/controller.cpp:18-21
 *   clrrt_rng_*            <- glibc rand()/srand() as consumed by rrt/src/rrtplanner.cpp:142,193-194
 *   clrrt_draw_samples     <- sampleAroundVehicle rrt/src/rrtplanner.cpp:187-201 + heuristic draw :142-143
 *   clrrt_set_obstacles    <- MotionPlanner::updateObstacles rrt/src/motionplanner.cpp:81-86 (det) feeding
 *                             checkObsDistance rrt/src/collisioncheck.cpp:6-8 (stub) or the OBB SAT of
 *                             rrt/src/old_collisioncheck.cpp:6-148
 *   clrrt_tree_init        <- initializeTree (empty branch) rrt/src/rrtplanner.cpp:39-48 + addInitialNode :21-37
 *   clrrt_tree_load        <- RRT.tree assignment (std::vector<Node>) rrt/include/rrt/rrtplanner.h:75
 *   clrrt_expand           <- the budget loop `for(; timer.Get(); ) expandTree(...)`
 *                             rrt/src/motionplanner.cpp:39-43 around expandTree rrt/src/rrtplanner.cpp:123-174
 *   clrrt_round_eval /     <- one batch of expandTree iterations split in its evaluate half (sampling, sort,
 *   clrrt_round_commit        Simulation) and its append half (RRT.addNode, rrtplanner.h:111-113), so the host
 *                             can all-gather accepted nodes across GPUs between the two halves
 *   clrrt_rollout_batch    <- Simulation::Simulation + propagate rrt/src/simulation.cpp:36-47,55-143
 *   clrrt_simulate         <- Simulation::Simulation (rrt/include/rrt/simulation.h:18-19) for an explicit
 *                             state and reference (the C++ Simulation adapter)
 *   clrrt_nn_batch         <- sortNodesExplore / sortNodesOptimize rrt/src/rrtplanner.cpp:227-268
 *   clrrt_get_counters     <- sim_count / fail_* globals rrt/src/rrt_node.cpp:21-24
 *
 * Threading: one context per host thread; a context is not thread-safe (the reference is not
 * reentrant either: rrt_node.cpp globals).  Device buffers are owned by the context.
 */
#ifndef CLRRT_H
#define CLRRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLRRT_ABI_VERSION 11

/* ---- status codes ---- */
#define CLRRT_OK 0
#define CLRRT_EINVAL (-1)
#define CLRRT_EHIP (-2)
#define CLRRT_ECAPACITY (-3)
#define CLRRT_ESTATE (-4)

/* ---- expansion modes ---- */
/* EXACT: the reference's sequential semantics (every iteration sees every node appended before it),
 *        realised by speculative rounds + in-order prefix commit.  Trees equal the reference's.
 * BATCH: frozen tree per round, every sample of the round is committed (throughput mode). */
#define CLRRT_MODE_EXACT 0
#define CLRRT_MODE_BATCH 1

/* parent id of a goal-biased record in a round's node batch: "the record just before me" */
#define CLRRT_PARENT_PREV (-2)

/* ---- collision modes ---- */
#define CLRRT_COLLISION_STUB 0 /* checkObsDistance returns 100 (rrt/src/collisioncheck.cpp:6-8) */
#define CLRRT_COLLISION_OBB 1  /* OBB separating-axis test (rrt/src/old_collisioncheck.cpp:6-148) */

/* ---- rollout outcomes (Simulation flags + the fail_* counter it bumped) ---- */
#define CLRRT_ROLL_ITERLIMIT 0 /* horizon exhausted: fail_iterlimit (simulation.cpp:142) */
#define CLRRT_ROLL_END 1       /* endReached (simulation.cpp:115-121) */
#define CLRRT_ROLL_GOAL 2      /* goalReached (simulation.cpp:125-132) */
#define CLRRT_ROLL_COLLISION 3 /* fail_collision (simulation.cpp:84-86) */
#define CLRRT_ROLL_ACCLIMIT 4  /* fail_acclimit (simulation.cpp:100-104) */

/* ---- initializeTree outcomes (rrtplanner.cpp:39-95) ---- */
#define CLRRT_REINIT_EMPTY 0      /* no committed nodes: addInitialNode(carState) (:43-48) */
#define CLRRT_REINIT_ALL_ERASED 1 /* every node behind the car; the reference reads nodes.front() of an
                                     empty vector (:90, undefined): taken as an empty tree */
#define CLRRT_REINIT_COLLISION 2  /* a committed row collides: empty tree (goto makeEmptyTree, :72-81) */
#define CLRRT_REINIT_KEPT 3       /* surviving nodes chained (parent i-1), goal flags and costS redone */

/* transformNodes* directions (transformations.cpp:289-315) */
#define CLRRT_WORLD_TO_CAR 0
#define CLRRT_CAR_TO_WORLD 1

/* Vehicle parameters (class Vehicle, rrt/include/rrt/vehicle.h:4-60).  Only the fields the
 * hot path reads are carried. */
typedef struct clrrt_vehicle {
  double dmax;  /* max steering angle */
  double ddmax; /* max steering rate */
  double Td;    /* steer damping */
  double Ta;    /* acceleration damping */
  double amin;  /* min acceleration */
  double amax;  /* max acceleration */
  double L;     /* wheel base */
  double Vch;   /* characteristic velocity */
  double Kus;   /* understeer gradient */
} clrrt_vehicle;

/* Everything the reference reads from mutable globals, the ROS parameter server and MyRRT
 * (rrt_node.cpp:13-18, parameters.launch:3-20, rrtplanner.cpp:12-19). */
typedef struct clrrt_params {
  clrrt_vehicle veh;
  double sim_dt;       /* ctrl/sampleTime */
  double ctrl_tla;     /* ctrl/tla */
  double ctrl_mindla;  /* ctrl/mindla */
  double ctrl_dlavmin; /* ctrl/dlavmin */
  double ctrl_Kp;      /* ctrl/Kp */
  double ctrl_Ki;      /* ctrl/Ki */
  double ref_int;      /* ctrl/refint */
  double ref_mindist;  /* ctrl/refmindist */
  double ref_res;      /* reference resolution of the query (updateReferenceResolution) */
  double vmax;         /* MotionRequest.vmax */
  double ay_road_max;  /* never set in the reference: 0 */
  double goal[4];      /* MotionRequest.goal: x, y, heading, velocity (car frame) */
  double Wcost[5];     /* motionplanner/weight_* */
  double lane_shift0;  /* MotionRequest.laneShifts[0] (only read when bend) */
  double Cxy[3];       /* MotionRequest.Cxy (only read when bend) */
  int32_t bend;        /* MotionRequest.bend */
  int32_t obs_use_pred;   /* obstacle constant-velocity prediction at x[6] (rrt_node.cpp:11) */
  int32_t sort_limit;     /* MyRRT::sortLimit = 10 */
  int32_t collision_mode; /* CLRRT_COLLISION_* */
} clrrt_params;

/* car_msgs/Obstacle2D: bbox centre (x, y, theta), size (x, y), twist linear (x, y). */
typedef struct clrrt_obstacle {
  double cx, cy, theta, size_x, size_y, vx, vy;
} clrrt_obstacle;

/* Tree node header (the hot-path part of struct Node, rrt/include/rrt/rrtplanner.h:35-48).
 * The trajectory (Node::tra) lives in a row arena: rows [row_offset, row_offset+nrows) of
 * 10 doubles each (x, y, theta, delta, v, a, t, IDwp, vref, delta_cmd).  ref_* are the
 * reference endpoints Node::ref.x/y.front()/back() and Node::ref.v.back(). */
typedef struct clrrt_node {
  double state[10];
  double ref_front[2];
  double ref_back[2];
  double ref_vback;
  double ang_par; /* atan2(ref_back - ref_front): feasibleNode's angPar (rrtplanner.cpp:273) */
  int32_t parent;
  float costE;
  float costS;
  int32_t goal;
  int32_t nrows;
  int32_t owner; /* rank whose arena holds the rows */
  int64_t row_offset;
} clrrt_node; /* 160 bytes */

/* glibc TYPE_3 additive-feedback generator state (random_r, srand(seed) semantics). */
typedef struct clrrt_rng {
  int32_t r[34];
  int32_t pos;
} clrrt_rng;

/* One expansion sample (a drawn iteration): point + heuristic (1 = explore, Dubins; 0 = optimize). */
typedef struct clrrt_sample {
  double x, y;
  int32_t explore;
  int32_t pad;
} clrrt_sample;

typedef struct clrrt_counters {
  int64_t sim_count;      /* simulated steps */
  int64_t fail_collision;
  int64_t fail_acclimit;
  int64_t fail_iterlimit;
  int64_t rollouts;
} clrrt_counters;

typedef struct clrrt_stats {
  int64_t iterations;   /* expandTree iterations consumed (3 rand() draws each) */
  int64_t nodes_added;  /* regular + goal-biased */
  int64_t goal_nodes_added;
  int64_t rounds;
  int64_t speculated;   /* samples evaluated (>= iterations in EXACT mode) */
  double elapsed_ms;
  int64_t capacity_stop; /* 1 when the loop ended because the next round could overflow capacity */
  int64_t deferred;      /* BATCH with option "defer_steps": samples committed at least one round late */
} clrrt_stats;

typedef struct clrrt_capacity {
  int64_t max_nodes; /* tree header capacity */
  int64_t max_rows;  /* trajectory arena capacity (rows of 10 doubles) */
  int32_t max_batch; /* samples per round */
  int32_t max_obstacles;
} clrrt_capacity;

/* Kernel-level rollout job: a Simulation from tree node `parent` towards `sample`
 * (gb = 0: getReference + regular profile; gb = 1: getGoalReference + GoalBiased profile). */
typedef struct clrrt_rollout_job {
  int32_t parent;
  int32_t gb;
  double sample[2];
} clrrt_rollout_job;

typedef struct clrrt_rollout_result {
  int32_t outcome; /* CLRRT_ROLL_* */
  int32_t nrows;   /* rows in stateArray (steps + 1) */
  double costE;    /* Simulation::costE (double, before the Node's float narrowing) */
  double costS;
  double final_state[10];
  double ref_back[2];
  double ref_vback;
  int32_t ref_n;
  int32_t pad;
} clrrt_rollout_result;

/* ---- parameters / RNG (host only, no device needed) ---- */
int clrrt_abi_version(void);
int clrrt_params_default(clrrt_params* p, double v0, const double goal[4], double vmax);
void clrrt_rng_seed(clrrt_rng* rng, uint32_t seed);
int32_t clrrt_rng_next(clrrt_rng* rng);
int clrrt_draw_samples(const clrrt_params* p, clrrt_rng* rng, int32_t n, clrrt_sample* out);

/* ---- context ---- */
typedef struct clrrt_ctx clrrt_ctx;
int clrrt_create(const clrrt_params* p, const clrrt_capacity* cap, int device, clrrt_ctx** out);
void clrrt_destroy(clrrt_ctx* ctx);
const char* clrrt_last_error(const clrrt_ctx* ctx);
int clrrt_set_stream(clrrt_ctx* ctx, void* hip_stream);
int clrrt_set_params(clrrt_ctx* ctx, const clrrt_params* p);
int clrrt_set_obstacles(clrrt_ctx* ctx, const clrrt_obstacle* obs, int32_t m);
int clrrt_set_rank(clrrt_ctx* ctx, int32_t rank);

/* ---- tree ---- */
int clrrt_tree_init(clrrt_ctx* ctx, const double root_state[10]);
int clrrt_tree_load(clrrt_ctx* ctx, const clrrt_node* nodes, int64_t n);
int clrrt_tree_size(clrrt_ctx* ctx, int64_t* n_nodes, int64_t* n_rows);
int clrrt_tree_download(clrrt_ctx* ctx, int64_t first, int64_t count, clrrt_node* out);
int clrrt_tree_rows(clrrt_ctx* ctx, int64_t row_offset, int64_t nrows, double* out);
/* Engine extension (no reference counterpart): drop the nodes [n, size) appended last (and their rows), e.g. the
 * iterations a caller speculated but did not take (clrrt_adapter's dropin::expandTree cache). 1 <= n <= size. */
int clrrt_tree_truncate(clrrt_ctx* ctx, int64_t n);

/* Per-iteration record of the expandTree iterations an expansion commits, in iteration order (clrrt_iteration_log
 * on; EXACT rounds and BATCH rounds without deferred samples): the nodes the iteration appended (0, 1 regular, 2
 * regular + goal-biased, rrtplanner.cpp:150-173) and its share of the reference's counters (rrt_node.cpp:21-24:
 * sim_count, fail_collision, fail_acclimit, fail_iterlimit) and rollouts. */
typedef struct clrrt_iteration {
  int32_t nodes;
  int32_t sim_count, fail_collision, fail_acclimit, fail_iterlimit, rollouts;
} clrrt_iteration;
/* EXACT rounds since the context was made: out[0] rounds with a conflict check, out[1] conflicts resolved by
 * fix-up rollouts (option "exact_fixup"), out[2] fix-up rollouts run, out[3] rounds whose prefix ended at a
 * conflict; why those conflicts were not resolved: out[4] a fix-up rollout succeeded, out[5] a key tie in the
 * sample's list, out[6] a new key equal to the sample's threshold, out[7] more new nodes than fix-up slots,
 * out[8] the accepted candidate pushed out of the sortLimit window; out[9] reserved (0: a window without a result
 * is always resolved by ranking the new nodes into it). */
int clrrt_exact_stats(clrrt_ctx* ctx, int64_t out[10]);
/* on != 0: start (or restart) logging, clearing the records; 0: stop and clear. */
int clrrt_iteration_log(clrrt_ctx* ctx, int32_t on);
/* Records logged so far (*n_total), and records [first, first + count) into out. */
int clrrt_iteration_records(clrrt_ctx* ctx, int64_t first, int64_t count, clrrt_iteration* out, int64_t* n_total);

/* extractBestPath (rrtplanner.cpp:318-368; declared rrtplanner.h:92): among the nodes with
 * goalReached set, in tree order, the front after the reference's std::sort by costS (ascending,
 * same unstable introsort) and its ancestors.  Writes the node ids root -> goal into path[0 .. cap)
 * and the full length into *n_path (0 when no node reached the goal -- the reference logs
 * "No feasible path found" and returns an empty vector).  Optional outputs: *best_cost (costS of
 * the chosen node, +inf when none) and *n_goal (goal nodes in the tree). */
int clrrt_extract_best_path(clrrt_ctx* ctx, int32_t* path, int32_t cap, int32_t* n_path, float* best_cost,
                            int64_t* n_goal);

/* ---- committed path (MotionPlanner::bestNodes, motionplanner.h:23) and tree re-initialisation ----
 * The path is held on the device: node headers (row_offset local to the path's own row buffer) and
 * their trajectories.  A planMotion query with commit_path = 1 (motionplanner.cpp:22-32, 50-54) is
 *   clrrt_path_transform(ctx, CLRRT_WORLD_TO_CAR, worldState)      transformNodesWorldToCar (:22)
 *   clrrt_set_params / clrrt_set_obstacles for the query
 *   clrrt_tree_init_from_path(ctx, carPose, &outcome)               initializeTree (:32)
 *   clrrt_expand(...)                                                the Timer(200) loop (:39-43)
 *   clrrt_extract_best_path + clrrt_path_commit                     bestNodes = extractBestPath (:51)
 *   clrrt_path_transform(ctx, CLRRT_CAR_TO_WORLD, worldState)      transformNodesCarToworld (:54)  */
/* bestNodes = the tree nodes ids[0 .. n) (headers and trajectories copied; rows of nodes owned by
 * another rank are zero-filled and counted in *n_remote -- fetch them from the owner and
 * clrrt_path_load the result). */
int clrrt_path_commit(clrrt_ctx* ctx, const int32_t* ids, int32_t n, int32_t* n_remote);
/* Replace the committed path with host data: n headers whose row_offset/nrows index `rows`
 * (n_rows rows of 10 doubles); every node needs nrows >= 1. */
int clrrt_path_load(clrrt_ctx* ctx, const clrrt_node* nodes, int32_t n, const double* rows, int64_t n_rows);
int clrrt_path_size(clrrt_ctx* ctx, int32_t* n, int64_t* n_rows);
int clrrt_path_download(clrrt_ctx* ctx, clrrt_node* nodes, double* rows);
/* transformNodesWorldToCar (dir CLRRT_WORLD_TO_CAR) / transformNodesCarToworld (CLRRT_CAR_TO_WORLD)
 * (transformations.cpp:289-315) of the committed path; pose = carState[0..2] (x, y, heading). */
int clrrt_path_transform(clrrt_ctx* ctx, int32_t dir, const double pose[3]);
/* initializeTree(RRT, veh, bestNodes, carState) (rrtplanner.cpp:39-95; getNodeCost :104-119) with
 * carState = 6 doubles (x, y, heading, delta, v, a; four zeros are appended as in :41): replaces the
 * tree with the re-initialised one and reports CLRRT_REINIT_* in *outcome.  Collision checks and
 * the obstacle cost term evaluate each trajectory row (the commented-out call at :74/:108) under
 * the context's collision mode and obstacles. */
int clrrt_tree_init_from_path(clrrt_ctx* ctx, const double car_state[6], int32_t* outcome);
/* The MPC trajectory message of the committed path (convertNodesToPath motionplanner.cpp:264-275 +
 * generateMPCmessage :103-128; with `filtered`, filterMPCmessage :130-151, waypoints >= 5 m apart).
 * One point = 8 doubles (x, y, theta, delta, v, a, a_cmd = row[8], d_cmd = row[9]); rows 1.. of
 * every node.  The filtered message carries no delta (the reference does not copy it): NaN there.
 * Writes min(*n_points, cap) points.  An empty message stays empty (the reference's loops over
 * size()-1 / from index 1 are undefined for it). */
int clrrt_path_mpc_message(clrrt_ctx* ctx, int32_t filtered, double* out, int32_t cap, int32_t* n_points);

/* ---- expansion ---- */
/* Runs expandTree iterations drawn from `rng` until `n_iters` iterations are consumed
 * (n_iters > 0) or, with n_iters == 0, until `budget_ms` of wall time has elapsed (checked
 * between rounds).  EXACT mode reproduces the reference's sequential tree; BATCH mode evaluates
 * `batch` samples per round against a frozen tree and commits all of them in sample order. */
int clrrt_expand(clrrt_ctx* ctx, clrrt_rng* rng, int64_t n_iters, double budget_ms, int32_t mode,
                 int32_t batch, clrrt_stats* out);

/* ---- multi-GPU expansion (engine extension, no reference counterpart) ----
 * With world > 1, clrrt_expand in BATCH mode runs sharded rounds: `batch` is the GLOBAL number of samples
 * per round (all drawn from the one glibc stream, as the reference's loop draws them); this rank evaluates
 * the contiguous slice [batch*rank/world, batch*(rank+1)/world) against the replicated tree, writes its
 * accepted-node records (clrrt_node, owner = rank, rows in this rank's arena) to dev_local, and calls
 * `exchange` once per round, which must return in io->dev_all the records of every rank concatenated in
 * rank order (device memory, valid until the next call; a collective such as one all-gather over RCCL) and
 * in io->n_all their count, in io->max_elapsed_ms the largest `elapsed_ms` over the ranks -- the budget is
 * checked against it, so every rank runs the same rounds --, in io->aux_sum the sum of `aux_local` over the
 * ranks (the engine's capacity bookkeeping: pending deferred samples, ranks whose arena is full; bit 48 and up:
 * ranks that failed) and in io->bbox_all the union of the ranks' `bbox_local` (the walk index's frame).  Every
 * rank then appends the same records in the same order (deferred samples: the oldest round first), so the trees
 * stay identical.  The caller chooses weak scaling (batch = world x per-GPU samples) or strong scaling (batch
 * fixed).  world = 1 turns sharding off.  dev_local holds cap_local records (>= 2 x the slice, + the deferred
 * samples).
 * No host synchronisation (ABI 11): the engine writes dev_local on io->stream and calls the hook without waiting
 * for it, so the hook's collective must be ordered after io->stream's work (a stream wait on an event, or the
 * same stream); the engine reads io->dev_all on io->stream after the hook returns, so the hook must order
 * io->stream after its own writes of it the same way.  Every sharded expansion ends with one closing exchange
 * (io->flags bit 0, n_local = 0), which carries a failure of any rank after its last round to the others. */
typedef struct clrrt_exchange_io {
  /* in */
  int32_t n_local;      /* records this rank wrote to dev_local */
  int32_t flags;        /* bit 0: the expansion's closing exchange */
  double elapsed_ms;    /* this rank's elapsed query time */
  int64_t aux_local;
  double bbox_local[4]; /* x0, y0, x1, y1 of the finite positions among this rank's records (+inf, +inf, -inf, -inf: none) */
  void* stream;         /* the engine's HIP stream */
  /* out */
  void* dev_all;
  int32_t n_all;
  int32_t pad;
  double max_elapsed_ms;
  int64_t aux_sum;
  double bbox_all[4];
} clrrt_exchange_io;
typedef int32_t (*clrrt_exchange_fn)(void* user, clrrt_exchange_io* io);
int clrrt_set_shards(clrrt_ctx* ctx, int32_t rank, int32_t world, void* dev_local, int32_t cap_local,
                     clrrt_exchange_fn exchange, void* user);

/* Evaluate `n` samples (host array) against the current tree; accepted nodes (regular and
 * goal-biased, in sample order) are written compacted to `dev_out` (device pointer, capacity
 * 2*n records) with row_offset local to this context's arena and owner = this rank.
 * *n_out receives the count. */
int clrrt_round_eval(clrrt_ctx* ctx, const clrrt_sample* samples, int32_t n, void* dev_out,
                     int32_t* n_out);
/* Append `n` node records (device pointer) to the tree in their order.  `local_first`/`local_count`
 * name the slice of them that this context produced in its last clrrt_round_eval (informational:
 * clrrt_round_eval reserved those records' rows in this context's arena, at the row_offset the
 * records carry, and the rows are written by the next rollout launch or clrrt_rows_flush); records
 * outside the slice are remote nodes whose rows stay on their owner (`owner`; clrrt_path_commit + a
 * gather of the path's rows complete a committed path). */
int clrrt_round_commit(clrrt_ctx* ctx, const void* dev_nodes, int32_t n, int32_t local_first,
                       int32_t local_count);
/* Engine extension (no reference counterpart): declares the samples of the NEXT clrrt_round_eval.
 * The coming clrrt_round_eval then runs their nearest-node search over the current tree beside its
 * rollouts, and clrrt_round_commit merges the committed nodes into those lists, so the next
 * clrrt_round_eval called with exactly these samples skips its search.  Results are identical to
 * calls without it; any other tree change discards the prefetch. */
int clrrt_round_prefetch(clrrt_ctx* ctx, const clrrt_sample* next_samples, int32_t n);
/* Engine extension (no reference counterpart): trajectory rows are deferred -- the rollouts a commit
 * accepts are replayed into the arena by the next rollout launch (option "rows_deferred").  This
 * writes the pending ones now (stream-ordered).  clrrt_expand does it before returning, and every call
 * that reads rows (clrrt_tree_rows, clrrt_path_commit) or changes what they depend on
 * (clrrt_set_obstacles, clrrt_set_params) does it first; a round-API caller ends a query with it. */
int clrrt_rows_flush(clrrt_ctx* ctx);

/* checkObsDistance(const vector<double>& x) (rrt/include/rrt/collision.h:41, the documented collision
 * hook README.md:40-47): out[i] = the distance the context's collision mode gives for states[i] (10
 * doubles: x, y, theta, ..., t in column 6) — 100 under CLRRT_COLLISION_STUB
 * (collisioncheck.cpp:6-8), the OBB form of old_collisioncheck.cpp:24-51 (0 on overlap, else the
 * smallest first-separating-axis gap, 10000 without obstacles) under CLRRT_COLLISION_OBB.  Evaluated on
 * the device by the rollout kernels' own collision code. */
int clrrt_obstacle_distance(clrrt_ctx* ctx, const double* states, int32_t n, double* out);

/* ---- kernel-level parity entries ---- */
int clrrt_rollout_batch(clrrt_ctx* ctx, const clrrt_rollout_job* jobs, int32_t n,
                        clrrt_rollout_result* out, double* rows_out, int32_t rows_cap);
/* Simulation::Simulation(RRT, state, ref, veh, GoalBiased, genProfile = true, Vstart) (simulation.h:18-19,
 * simulation.cpp:36-143) for n explicit cases, evaluated by the rollout kernels' own code (the C++
 * Simulation adapter, include/clrrt_adapter.hpp).  Per case: state (10 doubles), the reference as its
 * generator -- goal_biased = 0: the ref_n points a + i h accumulated (getReference's LinearSpacedVector,
 * functions.h:11-21); goal_biased = 1: getGoalReference (reference.cpp:25-70) from a with the context's goal
 * (h, ref_n ignored) -- and Vstart.  Writes results[i], rows (min(nrows, rows_cap) of stateArray per case,
 * rows_cap >= max steps + 1 or rows = NULL) and, with ref_out, the reference the Simulation used with the
 * velocity profile it generated: x, y, v (3 x ref_cap doubles per case, first min(N, ref_cap) points). */
typedef struct clrrt_sim_case {
  double state[10];
  double ax, ay, hx, hy;
  double vstart;
  int32_t ref_n;
  int32_t goal_biased;
} clrrt_sim_case;
int clrrt_simulate(clrrt_ctx* ctx, const clrrt_sim_case* cases, int32_t n, clrrt_rollout_result* results,
                   double* rows, int32_t rows_cap, double* ref_out, int32_t ref_cap);
/* Candidate lists (<= sortLimit node ids per sample, ascending key).  mode CLRRT_MODE_EXACT orders
 * equal keys as the reference's std::sort does (replayed per tied sample, O(n * tree) scratch);
 * CLRRT_MODE_BATCH orders them by node index. */
int clrrt_nn_batch(clrrt_ctx* ctx, const clrrt_sample* samples, int32_t n, int32_t mode, int32_t* out_ids,
                   float* out_keys);

/* Test hook: evaluates, on the device, the elementary functions exactly as the kernels call them,
 * out[i] = f(a[i], b[i]) for fn = 0 sin, 1 cos, 2 tan (glibc restatements), 3 sqrt, 4 fmod, 5 atan2,
 * 6 exp, 7 a/b, 8 cosf, 9 sinf (glibc sincosf restatement), 10 atan2f, 11 acosf, 12 asinf (glibc
 * restatements), 13 sqrtf, 14 float a/b, 15 round,
 * 16 sin and 17 cos of glibc's generic sincos, 20/21 the same through the rollout step's case-selected
 * form, 22 sin and 23 cos through the case-selected pair of FMA-build calls, 24..28 the rollout step's
 * branch-free trig block with x2 = a, x3 = b: sincos sin / cos, FMA-build sin / cos of a, tan of b
 * (float functions take (float)a, (float)b and return the float widened to double). */
int clrrt_selftest_math(clrrt_ctx* ctx, int32_t fn, const double* a, const double* b, int32_t n, double* out);
/* Test hook: the hot-path units exactly as the kernels evaluate them, n cases (tests/test_ref_units.py
 * bit-compares them with the reference's own code).  Per case, in -> out (doubles):
 *   CLRRT_UNIT_OBB      x, y, theta, t, obstacle cx, cy, theta, size_x, size_y, vx, vy -> getOBBdist of the
 *                       vehicle box (old_collisioncheck.cpp:34-36) and the obstacle box at t  [11 -> 1]
 *   CLRRT_UNIT_ODE      x0..x6, dc, ac -> x0..x6 after VehicleODE + IntegrateEuler, dx[2]  [9 -> 8]
 *                       (simulation.cpp:11-34, vehicle and sim_dt of the context's params)
 *   CLRRT_UNIT_LATERAL  xval[3], yval[3], (Px, Py, heading) -> interpolate(transformToVehicle(..))
 *                       (controller.cpp:115-148)  [9 -> 1]
 *   CLRRT_UNIT_PROFILE  ax, ay, sx, sy, ref_res, v0, vmax, goal[4], GB -> N, v[NMAX], x[NMAX], y[NMAX] of
 *                       getReference's line (reference.cpp:13-18) and generateVelocityProfile
 *                       (reference.cpp:73-170)  [12 -> 1 + 3 * CLRRT_UNIT_PROFILE_NMAX]
 *   CLRRT_UNIT_ANGLE    a, b -> angleDiff(a, b), wrapToPi(a) (functions.h:43-57)  [2 -> 2]
 * The units below take the goal / vmax / ref_res of each case (the rest of the context's params):
 *   CLRRT_UNIT_DUBINS   sx, sy, node x, y, heading, costE -> the explore key dubinsDistance (float) and
 *                       the optimize key costE + dubinsDistance (rrtplanner.cpp:231,254,371-406) as the
 *                       nearest-node kernels evaluate them  [6 -> 2]
 *   CLRRT_UNIT_FEASIBLE sx, sy, node ref front x, y, ref back x, y, ref_res -> feasibleNode
 *                       (rrtplanner.cpp:271-289) evaluated exactly (new nodes, conflicts), as the nearest-node
 *                       searches decide it (float with an exact fallback), and 1 when the brute-force
 *                       prefilter lets the node through  [7 -> 3]
 *   CLRRT_UNIT_GOALBIAS goal[4], node x, y, ref back x, y -> feasibleGoalBias (rrtplanner.cpp:292-315)
 *                       [8 -> 1]
 *   CLRRT_UNIT_GOALREF  goal[4], parent ref back x, y, v0, ref_res -> N, v, x, y of getGoalReference
 *                       (reference.cpp:25-70) + generateVelocityProfile(GB) (:72-170)
 *                       [8 -> 1 + 3 * CLRRT_UNIT_PROFILE_NMAX]
 *   CLRRT_UNIT_CTRL     kind (0: getReference from (a0, a1) to (a2, a3); 1: getGoalReference from ref back
 *                       (a0, a1)), a0..a3, goal[4], Vstart, vmax, ref_res, then CLRRT_UNIT_CTRL_K states
 *                       (x, y, heading, delta, v, a) -> the Controller of a Simulation (simulation.cpp:39-43,
 *                       controller.cpp:23-113): IDwp, endreached, Ppreview x, y after the constructor, then per
 *                       state getControls' IDwp, endreached, Ppreview x, y, ym, dc, ac, iE
 *                       [12 + 6 K -> 4 + 8 K] */
#define CLRRT_UNIT_OBB 0
#define CLRRT_UNIT_ODE 1
#define CLRRT_UNIT_LATERAL 2
#define CLRRT_UNIT_PROFILE 3
#define CLRRT_UNIT_ANGLE 4
#define CLRRT_UNIT_DUBINS 5
#define CLRRT_UNIT_FEASIBLE 6
#define CLRRT_UNIT_GOALBIAS 7
#define CLRRT_UNIT_GOALREF 8
#define CLRRT_UNIT_CTRL 9
#define CLRRT_UNIT_PROFILE_NMAX 1024
#define CLRRT_UNIT_CTRL_K 24
int clrrt_selftest_units(clrrt_ctx* ctx, int32_t unit, const double* in, int32_t n, double* out);

int clrrt_get_counters(clrrt_ctx* ctx, clrrt_counters* out);
int clrrt_reset_counters(clrrt_ctx* ctx);
/* Algorithmic work done by rollout kernels since the last reset (SURVEY §8(d) roofline basis):
 * out[0] = simulated steps (incl. speculative candidates), out[1] = reference
 * points scanned by findClosestPoint, out[2] = OBB box tests (first overlap ends a step's scan). */
int clrrt_work_counters(clrrt_ctx* ctx, int64_t out[3]);

/* Launch-time profile of the last clrrt_expand / round call: device milliseconds per kernel
 * family measured with HIP events on the stream each launch runs on.  which: 0 = nn (index builds,
 * walk searches, merges), 1 = rollout, 2 = commit, 3 = the walk searches alone (part of 0), 4 = the main
 * stream's waits for the side streams' lists (the search's share of the round's critical path), 5 = sharded
 * exchanges (the stream span from the records' copy to the gathered records); returns the summed ms and the
 * launch (or wait) count. */
int clrrt_kernel_time(clrrt_ctx* ctx, int32_t which, double* ms, int64_t* launches);
int clrrt_enable_timing(clrrt_ctx* ctx, int32_t on);

/* Execution knobs (results never depend on them): "roll_persistent" (1: candidate rollouts run on
 * persistent waves with a job queue, default; 0: one lane per candidate), "roll_blocks" (persistent
 * blocks of 256 lanes; 0: by tree size), "nn_walk_min" (trees of at least this many nodes use the
 * walk search, default 8192; below it the brute force), "nn_walk_stateless", "nn_walk_budget_tiles",
 * "nn_walk_budget_keys", "nn_walk_chunks", "nn_walk_max_over", "nn_walk_half_max", "nn_walk_waves", "nn_walk_lds_floor", "nn_walk_double", "nn_pipeline",
 * "nn_lag" (0: by query length, 1, 2), "nn_exact_fused", "nn_debug" (diagnostics; changes results),
 * "roll_priority", "roll_coop", "roll_spread", "roll_lanes", "rows_deferred", "exact_min_width",
 * "cu_split", "walk_cu_reserve", "stream_prio", "side_priority" (see clrrt_capi.hip). */
int clrrt_set_option(clrrt_ctx* ctx, const char* key, int64_t value);
/* Nearest-node search diagnostics since the last clrrt_reset_counters.  out[0..6] unused (0).  Brute
 * force: out[7] (sample, node) pairs passing the float prefilter, out[8] exact Dubins keys evaluated.  Walk search: out[10] super-tiles visited, out[11]
 * tiles visited, out[12] nodes passing the prefilter, out[13] exact Dubins keys evaluated, out[14..18]
 * shader clocks per phase when the "nn_debug" option is 2 (diagnostics). */
int clrrt_nn_stats(clrrt_ctx* ctx, int64_t out[19]);
/* Nearest-node search work since the last clrrt_reset_counters (SURVEY §8(d) roofline basis of
 * sortNodesExplore/Optimize, rrtplanner.cpp:227-268): out[0] = brute-force-equivalent Dubins keys
 * (samples x tree nodes of every search, plus the appended nodes merged into prefetched lists),
 * out[1] = samples searched, out[2] = walk-search tiles visited, out[3] = exact keys evaluated. */
int clrrt_search_work(clrrt_ctx* ctx, int64_t out[4]);
/* The same plus the walk's bound work (the hardware roofline basis of the walk search): out[0..3] as
 * clrrt_search_work, out[4] = phase-1 super-tile bounds (samples x super-tiles of each walk search), out[5] =
 * super-tile visits (each evaluates its 32 tile bounds), out[6] = records past the prefilter, out[7] = 0. */
int clrrt_search_work_ex(clrrt_ctx* ctx, int64_t out[8]);
/* Diagnostics (engine extension): for samples[0 .. n) over the current tree's walk index, what any search over the
 * index's tile bounds must touch, from the sample's true 11th key kth (brute force).  out[20 i + q]: q = 0 tiles whose
 * bound is <= kth, 1 of them holding a list member, 2 feasible records with key <= kth (ties included), 3 records of
 * those tiles whose stage-1 key bound is <= kth, 4 super-tiles whose bound is <= kth, 5 explore flag, 6 kth (float
 * bits), 7 records of the tiles of q = 0, of which 8 infeasible, 9 feasible but farther than kth, 10 feasible, within
 * kth, key > kth; 11 tiles of q = 0 holding a feasible record with key <= kth; 12 tiles of q = 0 whose ref.back() disc
 * holds the sample, 13 / 14 their position / ref.back() disc radii summed (mm), 15 those with an unbounded arc, 16
 * those inside one run of equal key inputs, 17 records of the tiles of q = 0 in such a run; 18, 19 reserved.  out
 * holds 20 values per sample. */
int clrrt_walk_audit(clrrt_ctx* ctx, const clrrt_sample* samples, int32_t n, int32_t* out);
/* Engine extension: the tree size after each commit of the last clrrt_expand -- its rounds in order, then the commit
 * of the deferred samples still pending at its end (defer_steps), when there were any -- into out[0 .. min(n, cap));
 * *n = the count.  With deferred samples, round r's samples are evaluated against the tree of out[r - 1] nodes (the
 * tree before the expansion for r = 0) and appended by the commit that is due for them. */
int clrrt_round_sizes(clrrt_ctx* ctx, int64_t* out, int64_t cap, int64_t* n);
/* Diagnostics: the context's 64 raw work counters (0..2 rollout work, 8..39 search statistics,
 * 40..63 rollout profile counters of a -DCLRRT_ROLL_PROFILE build: 40..47 per-phase clocks, 48..51 wave
 * lifetimes (sum, max), busiest lane's steps, waves, 52..55 queue-drain times and tail steps). */
int clrrt_debug_counters(clrrt_ctx* ctx, int64_t out[64]);

#ifdef __cplusplus
}
#endif

#endif /* CLRRT_H */
