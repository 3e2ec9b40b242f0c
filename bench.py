#!/usr/bin/env python3
"""Benchmark of the MI355X closed-loop RRT expansion engine (BASELINE.json metric:
nodes expanded/sec + feasible-paths/sec, 200-obstacle scene, 1/2/4/8 GPU).

A step is one planning query (MotionPlanner::planMotion, rrt/src/motionplanner.cpp:8-77 of the
reference): a fresh tree from the root, then expansion rounds of `batch` samples per GPU (BATCH mode:
every round evaluates its samples against the tree as it was at the round's start and appends all
accepted nodes) until the query's wall-clock horizon is spent.  Default workload: config 3 of
BASELINE.json — 200 static obstacles, 16384 samples per batch per GPU, 2 s horizon.

N > 1: one process per GPU (torch.distributed, RCCL); each round every rank evaluates its own
`batch` samples (weak scaling), the accepted-node records are all-gathered and every rank appends
the union in global sample order, so the trees stay identical.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))

CONFIGS = {
    # name: static obstacles, moving obstacles, samples per batch (per GPU), horizon ms
    "cfg2": dict(obstacles=50, moving=0, batch=4096, horizon_ms=200.0, defer_steps=64,
                 desc="cfg2: 50-obstacle static urban scene, 4096 samples/batch, 0.2 s horizon"),
    "cfg3": dict(obstacles=200, moving=0, batch=16384, horizon_ms=2000.0,
                 desc="cfg3: 200-obstacle static urban scene, 16384 samples/batch per GPU, 2 s horizon"),
    "cfg5": dict(obstacles=200, moving=20, batch=16384, horizon_ms=200.0, replan=True,
                 desc="cfg5: 200 static + 20 moving obstacles, 5 Hz replanning (0.2 s per query) with the tree "
                      "re-initialised from the previous best path, 16384 samples/batch per GPU"),
}

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_FP32_VALU_TF = 157.3
PEAK_FP64_VALU_TF = 78.6
PEAK_HBM_GBS = 8000.0
# Algorithmic FLOP per unit: FP64 per simulated step = 160 + 6 per reference
# point scanned by findClosestPoint; FP32 per OBB box test = 36.
FLOP_STEP, FLOP_SCAN, FLOP_BOX = 160, 6, 36
FLOP_KEY = 40  # FP32 FLOP per nearest-node (Dubins) key
# the walk search's own work (hardware roofline of k_walk_search): per tile / super-tile lower bound (walk_lb: two
# approximate acos, a square root, a reciprocal, the dot products: ~40 FP32 FLOP) and per record of a visited tile
# through the prefilter (distance + turning-bound + feasibility-cone tests: ~12 FLOP)
FLOP_TILE_BOUND, FLOP_PREFILTER = 40, 12
# BATCH option defer_steps of the headline run (a config may set its own)
DEFER_STEPS = 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="samples per round per GPU (default: config)")
    ap.add_argument("--horizon-ms", type=float, default=0.0, help="per-query budget (default: config)")
    ap.add_argument("--max-nodes", type=int, default=0,
                    help="tree capacity per rank (0: max(6 Mi, 2 Mi x N) -- the replicated tree grows N x faster)")
    ap.add_argument("--rows-per-node", type=int, default=64)
    ap.add_argument("--cpu-queries", type=int, default=5, help="oracle queries timed for cpu_baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-exact", action="store_true", help="skip the secondary EXACT-mode figure")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--defer-steps", type=int, default=-1,
                    help="BATCH deferred samples: rollout chains run at most this many steps per round's launch, "
                         "longer ones resume in the next and their sample commits in a later round (0: off; "
                         "default: the config's, else DEFER_STEPS)")
    ap.add_argument("--no-sync", action="store_true", help="skip the secondary figure without deferred samples")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = batch samples per GPU per round (N x batch per round), strong = batch "
                         "samples per round split over the GPUs")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the multi-rank path (e.g. several ranks sharing one GPU)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="clrrt_set_option before the run (A/B of scheduling options; results do not change)")
    return ap.parse_args()


def source_fingerprint():
    """sha256 (16 hex) of the engine's sources (cl-rrt_amd/csrc, include/clrrt.h): the build a committed PMC pass
    was collected on records it as "_src" (tools/summarize_pmc.py), so the bench line can name a pass of THIS
    build (the GPU box has no git history to compare commits against)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "cl-rrt_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "cl-rrt_amd", "csrc", "*.hpp")) + [os.path.join(ROOT, "include", "clrrt.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _tag_key(path):
    """Profile tags sort by round, then by suffix length, then alphabetically: r04q < r04z < r04aa < r04ah."""
    import re
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def pick_profile(paths, need=None):
    """The committed pass of the current sources if there is one (its "_src" field), else the newest by tag.
    Returns (path, json, same_build) or (None, None, False).  need(path) filters candidates."""
    fp = source_fingerprint()
    cands = sorted((p for p in paths if need is None or need(p)), key=_tag_key)
    loaded = []
    for p in cands:
        try:
            loaded.append((p, json.load(open(p))))
        except (OSError, ValueError):
            pass
    for p, d in reversed(loaded):
        if d.get("_src") == fp:
            return p, d, True
    if loaded:
        return loaded[-1][0], loaded[-1][1], False
    return None, None, False


def walk_wave_state(config):
    """Hardware view of the walk search (verdict item 2): how the main k_walk_search grid's wave time splits
    into issuing instructions, parked on s_waitcnt (memory / LDS) and issue stalls, from the newest committed SQ
    pass of this config (profiles/r*_<config>_walk_sq.json, tools/pmc_walk_bench.sh; the counters cannot be
    collected inside bench.py).  Returns a dict or None."""
    import glob
    path, d, same = pick_profile(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_walk_sq.json")))
    if not path:
        return None
    try:
        tot = {}
        for k, v in d.items():
            # the main grid: k_walk_search<FMT, SPLIT = false, ...>
            if k.startswith("void clrrt::k_walk_search<") and k.split(",")[1].strip() == "false":
                for c, x in v["total"].items():
                    tot[c] = tot.get(c, 0.0) + x
        wc = tot.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            return None
        return {"kernel": "k_walk_search (main grid)", "bound": "latency: wave time parked on memory / LDS waits",
                "frac": tot["SQ_ACTIVE_INST_ANY"] / wc, "unit": "fraction of wave time issuing",
                "parked_frac": tot["SQ_WAIT_ANY"] / wc, "issue_stall_frac": tot["SQ_WAIT_INST_ANY"] / wc,
                "valu_insts_per_wave": tot["SQ_INSTS_VALU"] / max(1.0, tot["SQ_WAVES"]),
                "source": f"{os.path.basename(path)} ({d.get('_build', 'unrecorded build')})",
                "same_build": same}
    except (KeyError, OSError, ValueError, IndexError):
        return None


def measured_traffic(config):
    """HBM bytes per rollout launch from the committed rocprofv3 PMC passes of THIS config
    (profiles/r*_<config>_pmc_{fetch,write}.json: FETCH_SIZE and WRITE_SIZE collected in separate runs,
    MI355X_MICROARCH.md HBM section); bench.py cannot collect counters itself.  The newest pass that has
    both files is used and named in the note.  Returns (bytes or None, note)."""
    import glob
    prof = os.path.join(ROOT, "profiles")
    write = {os.path.basename(w).split("_")[0]: w for w in glob.glob(os.path.join(prof, f"r*_{config}_pmc_write.json"))}
    fpath, f, same = pick_profile(glob.glob(os.path.join(prof, f"r*_{config}_pmc_fetch.json")),
                                  need=lambda p: os.path.basename(p).split("_")[0] in write)
    if not fpath:
        return None, f"no PMC profile committed for {config}"
    tag = os.path.basename(fpath).split("_")[0]
    try:
        w = json.load(open(write[tag]))

        def per_dispatch(summary, prefix, counter):
            # every template instantiation of the kernel (e.g. k_roll_run<false, false>), weighted
            # by its dispatch count
            rows = [v for k, v in summary.items() if k.startswith(prefix + "<")]
            n = sum(v["dispatches"] for v in rows)
            if not n:
                raise KeyError(prefix)
            return sum(v["total"][counter] for v in rows) / n

        kb = 0.0
        # the rollout launch: k_roll_run (+ k_roll_prep in builds before the Simulation ctor moved into
        # k_roll_run; absent from newer profiles)
        for name in ("void clrrt::k_roll_prep", "void clrrt::k_roll_run"):
            try:
                kb += 2.0 * per_dispatch(f, name, "FETCH_SIZE") + per_dispatch(w, name, "WRITE_SIZE")
            except KeyError:
                if name.endswith("k_roll_run"):
                    raise
        build = f.get("_build", "unrecorded build")
        which = "this build's sources" if same else "an EARLIER build (no pass of these sources is committed)"
        return kb * 1024.0, (f"{os.path.basename(fpath)} + {os.path.basename(write[tag])} ({build}; {which}): "
                             "(2 x FETCH_SIZE [gfx950 half-count correction] + WRITE_SIZE) KiB per launch")
    except (KeyError, OSError, ValueError) as e:
        return None, f"PMC profile unreadable: {e}"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cpu_queries(cfg, horizon_ms, n_queries, seed):
    """The reference-faithful CPU restatement (oracle/, kind 'port'), 1 thread: n_queries planning
    queries of the same scene and horizon (fresh trees; config 5: the replanning sequence with the tree
    re-initialised from the committed path).  Returns (nodes appended, goal nodes, wall seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    from clrrt import abi, replan, scenes
    from oracle_binding import Oracle

    obs = scenes.urban_scene(cfg["obstacles"], cfg["moving"])
    nodes = goals = 0
    t_total = 0.0
    pose = np.zeros(6)
    o = None
    for q in range(n_queries):
        if cfg.get("replan"):
            o = o or Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), None)
            Oracle.srand(seed + q)
            t0 = time.perf_counter()
            o.set_params(abi.default_params(v0=pose[4], goal=replan.goal_in_car_frame((40.0, 0.0, 0.0, 0.0), pose),
                                            collision_mode=abi.CLRRT_COLLISION_OBB))
            o.set_obstacles(replan.obstacles_in_car_frame(obs, q * replan.QUERY_PERIOD, pose))
            o.path_transform(False, pose)
            n0 = 1 if o.initialize_tree([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]]) != abi.REINIT_KEPT else o.size()
            o.expand_budget(horizon_ms, wall=True)
            ids = o.extract_best_path()
            o.path_commit(ids)
            o.path_transform(True, pose)
            t_total += time.perf_counter() - t0
            n = o.nodes()
            nodes += len(n["goal"]) - n0
            goals += int(n["goal"][n0:].sum())
            rows = [o.path_rows(i) for i in range(len(ids))]
            pose = replan.advance_pose(pose, np.concatenate(rows) if rows else None)
            continue
        o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
        Oracle.srand(seed + q)
        o.init_tree()
        t0 = time.perf_counter()
        o.expand_budget(horizon_ms, wall=True)
        t_total += time.perf_counter() - t0
        n = o.nodes()
        nodes += len(n["goal"]) - 1
        goals += int(n["goal"].sum())
    return nodes, goals, t_total


def _replica(cfg_name, horizon_ms, n_queries, seed, barrier, out):
    _cpu_queries(CONFIGS[cfg_name], 1.0, 1, seed)  # imports and library loads before the start line
    barrier.wait()
    t0 = time.perf_counter()
    nodes, goals, _ = _cpu_queries(CONFIGS[cfg_name], horizon_ms, n_queries, seed)
    out.put((nodes, goals, time.perf_counter() - t0))


def _gpu_exact_replica(cfg_name, horizon_ms, n_queries, seed, barrier, out, opts=None):
    """One GPU EXACT-mode planner process (its own HIP context and streams): a warm-up query, then n_queries
    queries of horizon_ms (fresh tree each, seeds seed, seed + 1, ...) after the common start line."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "cl-rrt_amd"))
    import clrrt
    from clrrt import abi, scenes
    cfg = CONFIGS[cfg_name]
    obs = scenes.urban_scene(cfg["obstacles"], cfg["moving"])
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 18,
                       max_rows=1 << 24, max_batch=1024, max_obstacles=max(1, len(obs)))
    pl.set_obstacles(obs)
    for k, v in (opts or {}).items():
        pl.set_option(k, v)
    pl.tree_init()
    pl.expand(clrrt.Rng(seed + 999), n_iters=0, budget_ms=200.0, mode=clrrt.CLRRT_MODE_EXACT, batch=1024)
    barrier.wait()
    t0 = time.perf_counter()
    nodes = goals = 0
    for q in range(n_queries):
        pl.tree_init()
        st = pl.expand(clrrt.Rng(seed + q), n_iters=0, budget_ms=horizon_ms, mode=clrrt.CLRRT_MODE_EXACT, batch=1024)
        nodes += st["nodes_added"]
        goals += st["goal_nodes_added"]
    out.put((nodes, goals, time.perf_counter() - t0))
    pl.close()


def gpu_exact_replicas(cfg_name, horizon_ms, R, seed, n_queries=2, opts=None):
    """EXACT mode as the CPU baseline's replicas run the reference: R independent planner processes sharing the GPU
    (each query's tree is the reference's sequential one), started together; aggregate nodes/s over the slowest
    replica's wall time.  Runs before the bench process touches the GPU (the replicas are separate processes)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    barrier, out = ctx.Barrier(R), ctx.Queue()
    procs = [ctx.Process(target=_gpu_exact_replica, args=(cfg_name, horizon_ms, n_queries, seed + 100 * k, barrier, out,
                                                          opts)) for k in range(R)]
    for p in procs:
        p.start()
    res = [out.get() for _ in range(R)]
    for p in procs:
        p.join()
    wall = max(r[2] for r in res)
    return {"value": sum(r[0] for r in res) / wall, "unit": "nodes/s", "replicas": R,
            "feasible_paths_per_s": sum(r[1] for r in res) / wall,
            "sample": f"{R} independent EXACT-mode planner processes on the one GPU x {n_queries} queries x "
                      f"{horizon_ms:.0f} ms, seeds {seed}+100k, started together, aggregate nodes over the slowest "
                      f"replica's {wall:.2f} s (each tree the reference's sequential one for its seed)"}


def cpu_share():
    """Host cores this job may use: the affinity set, capped by OMP_NUM_THREADS where the GPU box sets
    the job's CPU share (16 per GPU) — os.cpu_count() there is the whole machine's."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(cfg_name, horizon_ms, n_queries, seed, replica_queries=2):
    """(1) one planner on 1 thread (the reference's execution model); (2) `cpu_share()` independent
    planner replicas in separate processes, seeds seed..seed+R-1, aggregate nodes/s over the slowest
    replica's wall time (SURVEY.md §8(d) CPU baseline)."""
    import multiprocessing as mp
    cfg = CONFIGS[cfg_name]
    nodes, goals, t_total = _cpu_queries(cfg, horizon_ms, n_queries, seed)
    R = cpu_share()
    ctx = mp.get_context("spawn")
    barrier, out = ctx.Barrier(R), ctx.Queue()
    procs = [ctx.Process(target=_replica, args=(cfg_name, horizon_ms, replica_queries, seed + 100 * k, barrier, out))
             for k in range(R)]
    for p in procs:
        p.start()
    res = [out.get() for _ in range(R)]
    for p in procs:
        p.join()
    wall = max(r[2] for r in res)
    return {
        "value": nodes / t_total, "unit": "nodes/s", "cores": 1, "kind": "port",
        "feasible_paths_per_s": goals / t_total,
        "sample": f"{n_queries} planMotion queries x {horizon_ms:.0f} ms wall budget, {cfg['obstacles']}+"
                  f"{cfg['moving']} obstacles, srand({seed}..{seed + n_queries - 1}), 1 thread, {cpu_model()}",
        "replicas": {
            "value": sum(r[0] for r in res) / wall, "unit": "nodes/s", "cores": R,
            "feasible_paths_per_s": sum(r[1] for r in res) / wall,
            "sample": f"{R} independent planner processes x {replica_queries} queries x {horizon_ms:.0f} ms, "
                      f"seeds {seed}+100k, started together, aggregate nodes over the slowest replica's {wall:.2f} s, "
                      f"{cpu_model()}",
        },
    }


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    B = args.batch or cfg["batch"]
    horizon = args.horizon_ms or cfg["horizon_ms"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # the CPU baseline runs first, before this process touches the GPU (its replicas are separate
    # processes; nothing else competes for the host cores while it runs)
    cpu_line = None
    if world == 1 and not args.no_cpu:
        cpu_line = cpu_baseline(args.config, horizon, args.cpu_queries, args.seed)
    # EXACT mode the way the CPU baseline's replicas run the reference: as many independent planner processes as
    # the CPU replicas (at most 16 share the GPU), also before this process touches the GPU
    exact_rep = None
    if world == 1 and not args.no_exact and not cfg.get("replan"):
        exact_rep = gpu_exact_replicas(args.config, horizon, min(16, cpu_share()), args.seed)

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % max(1, ndev))
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    import clrrt
    from clrrt import abi, scenes

    obs = scenes.urban_scene(cfg["obstacles"], cfg["moving"])
    params = clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB)
    GOAL_WORLD = (40.0, 0.0, 0.0, 0.0)
    # the tree is replicated and grows N x faster with N ranks: size it so a 2 s query runs its whole
    # horizon instead of stopping at capacity (rows: 80 B x rows_per_node per node, 82 GB at 16 Mi nodes)
    max_nodes = args.max_nodes if args.max_nodes > 0 else max(6 << 20, (2 << 20) * world)
    max_rows = max_nodes * args.rows_per_node
    # samples per round over all ranks (weak: B per GPU; strong: B split over the GPUs) and per rank
    G = B * world if args.scaling == "weak" else B
    B_rank = -(-G // world)
    pl = clrrt.Planner(params, device=local % max(1, ndev), max_nodes=max_nodes, max_rows=max_rows, max_batch=B_rank,
                       max_obstacles=max(1, len(obs)))
    defer = args.defer_steps if args.defer_steps >= 0 else cfg.get("defer_steps", DEFER_STEPS)
    pl.set_option("defer_steps", defer)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        pl.set_option(k, int(v))
    pl.set_obstacles(obs)
    pl.set_rank(rank)
    stream = torch.cuda.current_stream()
    pl.set_stream(stream.cuda_stream)

    if world > 1:
        # one code path for 1 and N GPUs: clrrt_expand runs the sharded rounds itself (this rank's slice of
        # every round, lag-2 pipeline, deferred samples) and calls back once per round for the all-gather
        from clrrt import dist as cdist
        ex = cdist.ShardExchange(pl, cdist.exchange_capacity(B_rank, defer), "cuda", slice_size=B_rank)

    replanning = bool(cfg.get("replan"))
    if replanning:
        from clrrt import replan
        make_params = replan.default_make_params(abi.CLRRT_COLLISION_OBB)
        backend = replan.PlannerBackend(pl, make_params)
        rp = {"pose": [0.0, 0.0, 0.0, 0.0, 0.0, 0.0], "q": 0, "outcomes": [], "reinit_ms": 0.0, "path_len": []}

    deferred = [0]
    rounds = [0]

    def expand_query(rng):
        st = pl.expand(rng, n_iters=0, budget_ms=horizon, mode=clrrt.CLRRT_MODE_BATCH, batch=G)
        deferred[0] += st["deferred"]
        rounds[0] += st["rounds"]
        return st["nodes_added"], st["goal_nodes_added"], st["capacity_stop"]

    def query(seed):
        """One planning query; returns (nodes appended, goal nodes appended, capacity_stop)."""
        rng = clrrt.Rng(seed)
        if not replanning:
            pl.tree_init()
            return expand_query(rng)
        # config 5: MotionPlanner::planMotion with commit_path = 1 (replan.py)
        import numpy as np
        pose = np.asarray(rp["pose"])
        t_w = rp["q"] * replan.QUERY_PERIOD
        t0 = time.perf_counter()
        oc = backend.begin_query(pose, replan.goal_in_car_frame(GOAL_WORLD, pose),
                                 replan.obstacles_in_car_frame(obs, t_w, pose))
        rp["reinit_ms"] += (time.perf_counter() - t0) * 1e3
        rp["outcomes"].append(oc)
        res = expand_query(rng)
        ids, _, n_goal = pl.extract_best_path()
        rp.setdefault("goal_nodes", []).append(n_goal)
        pl.path_commit(ids)
        if world > 1:
            cdist.fetch_path_rows(pl, rank)
        pl.path_transform(True, pose)
        _, rows = pl.path_download()
        rp["path_len"].append(len(ids))
        rp["pose"] = replan.advance_pose(pose, rows)
        rp["q"] += 1
        return res

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for w in range(args.warmup):
        query(args.seed + 1000 + w)
    pl.enable_timing(True)
    pl.reset_counters()
    rounds[0] = 0
    barrier_sync()
    t0 = time.perf_counter()
    tot_nodes = tot_goals = cap_stops = 0
    for k in range(args.steps):
        n, g, c = query(args.seed + k)
        tot_nodes += n
        tot_goals += g
        cap_stops += c
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    trees_identical = None
    if world > 1:
        # every rank appended the same records in the same order: compare the trees of the last query
        import numpy as np
        raw = np.frombuffer(bytes(pl.nodes_raw()), dtype=np.uint8).reshape(-1, 160)
        hdr = np.ascontiguousarray(raw[:, :148])  # headers without the owner / row-offset fields
        sig = torch.tensor([float(hdr.shape[0]), float(hdr.view(np.int32).astype(np.int64).sum() % (1 << 40))],
                           dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        sigs = [torch.empty_like(sig) for _ in range(world)]
        dist.all_gather(sigs, sig)
        trees_identical = all(bool(torch.equal(x, sigs[0])) for x in sigs)

    roll_ms, roll_n = pl.kernel_time(1)
    nn_ms, nn_n = pl.kernel_time(0)
    walk_ms, walk_n = pl.kernel_time(3)
    other_ms, other_n = pl.kernel_time(2)
    wait_ms, wait_n = pl.kernel_time(4)
    xch_ms, xch_n = pl.kernel_time(5)
    # where a round's time goes on this rank (per round of the timed queries): wall time, the rollout launch, the
    # walk searches' summed event time (overlapping launches: not a critical-path figure), the main stream's wait
    # for the side streams' lists (the search's share of the critical path) and the exchange's stream span
    nr = max(1, rounds[0])
    split = [float(rounds[0]), elapsed * 1e3 / nr, roll_ms / nr, walk_ms / nr, wait_ms / nr,
             xch_ms / nr, float(pl.size()[0])]
    per_rank = [split]
    if world > 1:
        t = torch.tensor(split, dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        per_rank = [p.cpu().tolist() for p in parts]
    round_split = [dict(zip(("rounds", "round_ms", "rollout_ms", "walk_event_ms", "list_wait_ms", "exchange_ms",
                             "tree_nodes_last"), v)) for v in per_rank]
    work = pl.work_counters()
    cnt = pl.counters()
    sw = pl.search_work_ex()

    sync_line = None
    if world == 1 and not replanning and not args.no_sync and defer > 0:
        # secondary figure: plain BATCH rounds (every sample commits in its own round), one query from a
        # fresh tree, same scene, horizon and seed
        pl.set_option("defer_steps", 0)
        pl.tree_init()
        st = pl.expand(clrrt.Rng(args.seed), n_iters=0, budget_ms=horizon, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        sync_line = {"value": st["nodes_added"] / (st["elapsed_ms"] * 1e-3), "unit": "nodes/s",
                     "feasible_paths_per_s": st["goal_nodes_added"] / (st["elapsed_ms"] * 1e-3),
                     "rounds": st["rounds"], "horizon_ms": horizon,
                     "note": "BATCH rounds without deferred samples (defer_steps 0); 1 query, wall clock"}
        pl.set_option("defer_steps", defer)

    exact_line = None
    if world == 1 and not replanning and not args.no_exact:
        # secondary figure: EXACT mode (the reference's sequential expandTree tree, bit for bit) on the
        # same scene and horizon, one query from a fresh tree
        pl.tree_init()
        x0 = pl.exact_stats()
        pl.enable_timing(True)
        st = pl.expand(clrrt.Rng(args.seed), n_iters=0, budget_ms=horizon, mode=clrrt.CLRRT_MODE_EXACT, batch=B)
        x1 = pl.exact_stats()
        ex_ms = {name: pl.kernel_time(w)[0] / max(1, st["rounds"]) for name, w in (("nn", 0), ("rollout", 1), ("commit", 2))}
        exact_line = {"value": st["nodes_added"] / (st["elapsed_ms"] * 1e-3), "unit": "nodes/s",
                      "ms_per_round": st["elapsed_ms"] / max(1, st["rounds"]),
                      "device_ms_per_round": ex_ms,
                      "fixups": {k: x1[k] - x0[k] for k in x1},
                      "feasible_paths_per_s": st["goal_nodes_added"] / (st["elapsed_ms"] * 1e-3),
                      "iterations": st["iterations"], "rounds": st["rounds"], "speculated": st["speculated"],
                      "horizon_ms": horizon,
                      "note": "EXACT mode: trees identical to the reference's sequential expandTree (same seed); "
                              "1 query, wall clock"}
        if exact_rep is not None:
            exact_line["replicas"] = exact_rep

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    traffic, traffic_note = measured_traffic(args.config)
    # Algorithmic work credited to the rollout kernel: the reference's own steps (sim_count: the
    # candidates expandTree simulates, up to the first success), not the speculative candidates the
    # kernel also started; scan points and box tests are counted on executed steps and scaled by the
    # same ratio (they are per-step quantities).
    spec = work["steps"] / cnt["sim_count"] if cnt["sim_count"] else 1.0
    fp64 = FLOP_STEP * cnt["sim_count"] + FLOP_SCAN * work["scan_points"] / spec
    fp32 = FLOP_BOX * work["box_tests"] / spec
    achieved_tf = (fp64 + fp32) / (roll_ms * 1e-3) / 1e12 if roll_ms > 0 else 0.0
    t_mix = fp64 / PEAK_FP64_VALU_TF + fp32 / PEAK_FP32_VALU_TF
    peak_tf = (fp64 + fp32) / t_mix if t_mix > 0 else PEAK_FP32_VALU_TF
    avg_launch_ms = roll_ms / roll_n if roll_n else 0.0
    hbm_gbs = traffic / (avg_launch_ms * 1e-3) / 1e9 if traffic and avg_launch_ms > 0 else None
    # walk search: the FLOP of the work it does (exact keys, tile / super-tile bounds, prefiltered records) over
    # its own launches' time, against the FP32 VALU peak; the brute-force keys it avoids are a separate ratio
    walk_flop = (FLOP_KEY * sw["exact_keys"] + FLOP_TILE_BOUND * (sw["super_bounds"] + 32 * sw["super_visits"])
                 + FLOP_PREFILTER * 32 * sw["tiles"])
    walk_tf = walk_flop / (walk_ms * 1e-3) / 1e12 if walk_ms > 0 else 0.0
    done_keys = sw["exact_keys"] + 32 * sw["tiles"]
    value = tot_nodes / elapsed
    line = {
        "metric": "nodes expanded/sec (200-obstacle scene)",
        "value": value,
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "feasible_paths_per_s": tot_goals / elapsed,
        "config": {
            "workload": cfg["desc"],
            "samples_per_batch": B,
            "samples_per_round": G,
            "obstacles": cfg["obstacles"] + cfg["moving"],
            "horizon_ms": horizon,
            "mode": "BATCH",
            "parallelism": f"dp{world}",
            "capacity_stops": cap_stops,
            "defer_steps": defer,
            "samples_deferred": deferred[0],
            "trees_identical_across_ranks": trees_identical,
        },
        "roofline": {
            "bound": "valu",
            "kernel": "k_roll_run (candidate and goal-biased rollouts, replays of the accepted ones)",
            "achieved": achieved_tf,
            "peak": peak_tf,
            "unit": "TFLOP/s",
            "frac": achieved_tf / peak_tf if peak_tf else 0.0,
            "traffic": traffic,
            "traffic_note": traffic_note,
            "launches": roll_n,
            "avg_launch_ms": avg_launch_ms,
            "flop_per_launch": (fp64 + fp32) / roll_n if roll_n else 0.0,
            "fp64_flop": fp64,
            "fp32_flop": fp32,
            "work_basis": "reference-semantic steps (sim_count); executed steps incl. speculative candidates "
                          "= speculative_overhead x sim_count",
            "speculative_overhead": spec,
            "hbm_gbs": hbm_gbs,
            "hbm_frac": hbm_gbs / PEAK_HBM_GBS if hbm_gbs else None,
            "hbm_note": "traffic (PMC bytes per launch) / avg_launch_ms vs 8 TB/s HBM3E peak",
            "peak_note": "mix-weighted VALU peak: FP64 78.6 TF/s, FP32 157.3 TF/s (MI355X_MICROARCH.md)",
        },
        "roofline_nn": {
            "bound": "valu",
            "kernel": "k_walk_search (the walk searches: sample order, main grid, overflow split + merge)",
            "achieved": walk_tf,
            "peak": PEAK_FP32_VALU_TF,
            "unit": "TFLOP/s",
            "frac": walk_tf / PEAK_FP32_VALU_TF,
            "work_basis": f"work the walk does: {FLOP_KEY} FLOP per exact Dubins key, {FLOP_TILE_BOUND} per tile or "
                          f"super-tile bound, {FLOP_PREFILTER} per record of a visited tile (prefilter), over the "
                          "walk launches' HIP-event time",
            "walk_ms": walk_ms,
            "walk_launches": walk_n,
            "walk_flop": walk_flop,
            "work_avoided": sw["bf_keys"] / done_keys if done_keys else None,
            "work_avoided_note": "brute-force-equivalent keys (samples x tree nodes) per key-or-record the walk "
                                 "touched (exact keys + records of visited tiles)",
            "super_bounds_per_sample": sw["super_bounds"] / sw["samples"] if sw["samples"] else 0.0,
            "bf_keys": sw["bf_keys"],
            "samples": sw["samples"],
            "tiles_per_sample": sw["tiles"] / sw["samples"] if sw["samples"] else 0.0,
            "exact_keys_per_sample": sw["exact_keys"] / sw["samples"] if sw["samples"] else 0.0,
            "nn_launches": nn_n,
            "nn_kernel_ms": nn_ms,
        },
        "kernel_ms": {"rollout": roll_ms, "nn": nn_ms, "select_commit": other_ms,
                      "launches": {"rollout": roll_n, "nn": nn_n, "other": other_n}},
        "round_split": round_split if world > 1 else round_split[0],
        "round_split_note": "per round of the timed queries (per rank with N > 1): wall ms, rollout launch ms, walk "
                            "searches' summed event ms (overlapping launches), the main stream's wait for the lists "
                            "(the search's share of the critical path), the exchange's stream span",
        "work": {**work, **cnt},
    }
    if replanning:
        nq = max(1, len(rp["outcomes"]))
        line["config"]["replanning"] = {
            "queries": len(rp["outcomes"]), "reinit_outcomes": rp["outcomes"][-args.steps:],
            "path_lengths": rp["path_len"][-args.steps:], "goal_nodes": rp["goal_nodes"][-args.steps:],
            "tree_nodes_last": pl.size()[0], "reinit_ms_avg": rp["reinit_ms"] / nq,
            "note": "outcome 0 empty, 1 all erased, 2 committed path collides, 3 re-initialised from the path"}
    if sync_line:
        line["batch_sync"] = sync_line
    ww = walk_wave_state(args.config)
    if ww:
        line["roofline_walk"] = ww
    if exact_line:
        line["exact_mode"] = exact_line
    if cpu_line:
        line["cpu_baseline"] = cpu_line
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


C_SAMPLE = 24

if __name__ == "__main__":
    main()
