"""clrrt — Python binding of libclrrt (the MI355X closed-loop RRT tree-expansion engine).

The product is the C-ABI shared library `cl-rrt_amd/libclrrt.so` (HIP kernels for gfx950 + host
orchestration).  This module only marshals arguments through ctypes; it never computes any part of
the hot path itself, and it raises if the library (or a GPU, for device entry points) is missing.

The class names mirror the reference's planner objects (vdBerg93/cl-rrt):
  Planner.expand_tree(...)  <- expandTree           rrt/src/rrtplanner.cpp:123-174
  Planner.plan(budget_ms)   <- MotionPlanner::planMotion's Timer loop  rrt/src/motionplanner.cpp:39-43
  Planner.simulate(...)     <- Simulation            rrt/src/simulation.cpp:36-143
  Planner.sort_nodes(...)   <- sortNodesExplore/Optimize  rrt/src/rrtplanner.cpp:227-268
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .abi import (CLRRT_COLLISION_OBB, CLRRT_COLLISION_STUB, CLRRT_MODE_BATCH,  # noqa: F401
                  CLRRT_MODE_EXACT, ROLL_NAMES)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("CLRRT_LIB") or os.path.join(PKG_DIR, "libclrrt.so")  # CLRRT_LIB: diagnostics builds
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "clrrt.h")

_lib = None
P = C.POINTER
# clrrt_exchange_fn (include/clrrt.h): (user, clrrt_exchange_io*) -> status
EXCHANGE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, P(abi.ExchangeIO))

_SIGS = {
    "clrrt_abi_version": (C.c_int, []),
    "clrrt_params_default": (C.c_int, [P(abi.Params), C.c_double, P(C.c_double), C.c_double]),
    "clrrt_rng_seed": (None, [P(abi.Rng), C.c_uint32]),
    "clrrt_rng_next": (C.c_int32, [P(abi.Rng)]),
    "clrrt_draw_samples": (C.c_int, [P(abi.Params), P(abi.Rng), C.c_int32, P(abi.Sample)]),
    "clrrt_create": (C.c_int, [P(abi.Params), P(abi.Capacity), C.c_int, P(C.c_void_p)]),
    "clrrt_destroy": (None, [C.c_void_p]),
    "clrrt_last_error": (C.c_char_p, [C.c_void_p]),
    "clrrt_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "clrrt_set_params": (C.c_int, [C.c_void_p, P(abi.Params)]),
    "clrrt_set_obstacles": (C.c_int, [C.c_void_p, P(abi.Obstacle), C.c_int32]),
    "clrrt_set_rank": (C.c_int, [C.c_void_p, C.c_int32]),
    "clrrt_set_shards": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, EXCHANGE_FN, C.c_void_p]),
    "clrrt_tree_init": (C.c_int, [C.c_void_p, P(C.c_double)]),
    "clrrt_tree_load": (C.c_int, [C.c_void_p, P(abi.Node), C.c_int64]),
    "clrrt_tree_size": (C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64)]),
    "clrrt_tree_download": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, P(abi.Node)]),
    "clrrt_tree_rows": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, P(C.c_double)]),
    "clrrt_extract_best_path": (C.c_int, [C.c_void_p, P(C.c_int32), C.c_int32, P(C.c_int32), P(C.c_float),
                                          P(C.c_int64)]),
    "clrrt_path_commit": (C.c_int, [C.c_void_p, P(C.c_int32), C.c_int32, P(C.c_int32)]),
    "clrrt_path_load": (C.c_int, [C.c_void_p, P(abi.Node), C.c_int32, P(C.c_double), C.c_int64]),
    "clrrt_path_size": (C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int64)]),
    "clrrt_path_download": (C.c_int, [C.c_void_p, P(abi.Node), P(C.c_double)]),
    "clrrt_path_transform": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_double)]),
    "clrrt_tree_init_from_path": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_int32)]),
    "clrrt_path_mpc_message": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_double), C.c_int32, P(C.c_int32)]),
    "clrrt_expand": (C.c_int, [C.c_void_p, P(abi.Rng), C.c_int64, C.c_double, C.c_int32, C.c_int32, P(abi.Stats)]),
    "clrrt_round_eval": (C.c_int, [C.c_void_p, P(abi.Sample), C.c_int32, C.c_void_p, P(C.c_int32)]),
    "clrrt_round_commit": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "clrrt_rows_flush": (C.c_int, [C.c_void_p]),
    "clrrt_round_prefetch": (C.c_int, [C.c_void_p, P(abi.Sample), C.c_int32]),
    "clrrt_simulate": (C.c_int, [C.c_void_p, P(abi.SimCase), C.c_int32, P(abi.RolloutResult), P(C.c_double),
                                 C.c_int32, P(C.c_double), C.c_int32]),
    "clrrt_rollout_batch": (C.c_int, [C.c_void_p, P(abi.RolloutJob), C.c_int32, P(abi.RolloutResult),
                                      P(C.c_double), C.c_int32]),
    "clrrt_nn_batch": (C.c_int, [C.c_void_p, P(abi.Sample), C.c_int32, C.c_int32, P(C.c_int32), P(C.c_float)]),
    "clrrt_selftest_math": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_double), P(C.c_double), C.c_int32,
                                      P(C.c_double)]),
    "clrrt_selftest_units": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_double), C.c_int32, P(C.c_double)]),
    "clrrt_get_counters": (C.c_int, [C.c_void_p, P(abi.Counters)]),
    "clrrt_reset_counters": (C.c_int, [C.c_void_p]),
    "clrrt_work_counters": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_kernel_time": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_double), P(C.c_int64)]),
    "clrrt_enable_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "clrrt_nn_stats": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_search_work": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_search_work_ex": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_walk_audit": (C.c_int, [C.c_void_p, P(abi.Sample), C.c_int32, P(C.c_int32)]),
    "clrrt_round_sizes": (C.c_int, [C.c_void_p, P(C.c_int64), C.c_int64, P(C.c_int64)]),
    "clrrt_tree_truncate": (C.c_int, [C.c_void_p, C.c_int64]),
    "clrrt_iteration_log": (C.c_int, [C.c_void_p, C.c_int32]),
    "clrrt_exact_stats": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_iteration_records": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, P(abi.Iteration), P(C.c_int64)]),
    "clrrt_obstacle_distance": (C.c_int, [C.c_void_p, P(C.c_double), C.c_int32, P(C.c_double)]),
    "clrrt_debug_counters": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "clrrt_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
}


class ClrrtError(RuntimeError):
    pass


def lib():
    """Load libclrrt.so (raises loudly when it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: when PyTorch is present its bundled libamdhip64.so.7 must be
        # the one loaded (same soname), so import it before libclrrt pulls /opt/rocm's copy in.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ClrrtError(f"libclrrt.so not built at {LIB_PATH}: run `make -C cl-rrt_amd/csrc` "
                             "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.clrrt_abi_version() != abi.CLRRT_ABI_VERSION:
            raise ClrrtError(f"{LIB_PATH}: ABI version {L.clrrt_abi_version()} != {abi.CLRRT_ABI_VERSION}; rebuild")
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


# ----------------------------------------------------------------------------- host-only helpers
def default_params(v0=0.0, goal=(40.0, 0.0, 0.0, 0.0), vmax=5.0, collision_mode=CLRRT_COLLISION_STUB):
    p = abi.Params()
    g = (C.c_double * 4)(*goal)
    rc = lib().clrrt_params_default(C.byref(p), v0, g, vmax)
    if rc != 0:
        raise ClrrtError(f"clrrt_params_default -> {rc}")
    p.collision_mode = collision_mode
    return p


class Rng:
    """glibc rand() stream (TYPE_3 additive feedback), srand(seed) semantics."""

    def __init__(self, seed=1):
        self.state = abi.Rng()
        lib().clrrt_rng_seed(C.byref(self.state), seed)

    def next(self):
        return lib().clrrt_rng_next(C.byref(self.state))

    def draw_samples(self, params, n):
        out = (abi.Sample * n)()
        rc = lib().clrrt_draw_samples(C.byref(params), C.byref(self.state), n, out)
        if rc != 0:
            raise ClrrtError(f"clrrt_draw_samples -> {rc}")
        return out


def samples_to_numpy(samples):
    xy = np.array([(s.x, s.y) for s in samples], dtype=np.float64).reshape(-1, 2)
    ex = np.array([s.explore for s in samples], dtype=np.int32)
    return xy, ex


def nodes_to_numpy(nodes):
    n = len(nodes)
    raw = np.frombuffer(bytes(nodes), dtype=np.uint8).reshape(n, C.sizeof(abi.Node))
    f64 = lambda a, b: raw[:, a:b].copy().view(np.float64)  # noqa: E731
    i32 = lambda a, b: raw[:, a:b].copy().view(np.int32).reshape(-1)  # noqa: E731
    f32 = lambda a, b: raw[:, a:b].copy().view(np.float32).reshape(-1)  # noqa: E731
    return {
        "state": f64(0, 80).reshape(-1, 10), "ref_front": f64(80, 96).reshape(-1, 2),
        "ref_back": f64(96, 112).reshape(-1, 2), "ref_vback": f64(112, 120).reshape(-1),
        "ang_par": f64(120, 128).reshape(-1), "parent": i32(128, 132), "costE": f32(132, 136),
        "costS": f32(136, 140), "goal": i32(140, 144), "nrows": i32(144, 148), "owner": i32(148, 152),
        "row_offset": raw[:, 152:160].copy().view(np.int64).reshape(-1),
    }


# ----------------------------------------------------------------------------- device planner
class Planner:
    """One libclrrt context on one GPU: a MyRRT tree plus the query's parameters and obstacles."""

    def __init__(self, params, device=0, max_nodes=1 << 20, max_rows=1 << 24, max_batch=4096,
                 max_obstacles=4096):
        self.L = lib()
        self.params = params
        cap = abi.Capacity(max_nodes, max_rows, max_batch, max_obstacles)
        h = C.c_void_p()
        rc = self.L.clrrt_create(C.byref(params), C.byref(cap), device, C.byref(h))
        if rc != 0:
            raise ClrrtError(f"clrrt_create failed ({rc}): no usable HIP device {device}?")
        self.h = h
        self.max_batch = max_batch
        # engine options for A/B runs: CLRRT_OPTIONS="key=value,key=value" (clrrt_set_option)
        for kv in filter(None, os.environ.get("CLRRT_OPTIONS", "").split(",")):
            k, v = kv.split("=")
            self.set_option(k.strip(), int(v))

    def close(self):
        if getattr(self, "h", None):
            self.L.clrrt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.L.clrrt_last_error(self.h)
            raise ClrrtError(f"{what} -> {rc}: {msg.decode() if msg else ''}")

    def set_stream(self, stream_ptr):
        self._chk(self.L.clrrt_set_stream(self.h, C.c_void_p(stream_ptr)), "set_stream")

    def set_params(self, params):
        self.params = params
        self._chk(self.L.clrrt_set_params(self.h, C.byref(params)), "set_params")

    def set_rank(self, rank):
        self._chk(self.L.clrrt_set_rank(self.h, rank), "set_rank")

    def set_shards(self, rank, world, dev_local=0, cap_local=0, exchange=None):
        """Sharded BATCH expansion (clrrt_set_shards): `exchange` is an EXCHANGE_FN (keep a reference to it
        for as long as the planner uses it; clrrt.dist.ShardExchange does)."""
        self._exchange = exchange
        fn = exchange if exchange is not None else EXCHANGE_FN()
        self._chk(self.L.clrrt_set_shards(self.h, rank, world, C.c_void_p(dev_local), cap_local, fn, None),
                  "set_shards")

    def set_obstacles(self, obs):
        obs = np.ascontiguousarray(obs, dtype=np.float64).reshape(-1, 7)
        arr = (abi.Obstacle * max(1, len(obs)))()
        C.memmove(arr, obs.ctypes.data, obs.nbytes)
        self._chk(self.L.clrrt_set_obstacles(self.h, arr, len(obs)), "set_obstacles")

    def tree_init(self, root=None):
        root = np.zeros(10) if root is None else np.ascontiguousarray(root, dtype=np.float64)
        self._chk(self.L.clrrt_tree_init(self.h, root.ctypes.data_as(P(C.c_double))), "tree_init")

    def tree_load(self, nodes_raw):
        self._chk(self.L.clrrt_tree_load(self.h, nodes_raw, len(nodes_raw)), "tree_load")

    def size(self):
        n, r = C.c_int64(), C.c_int64()
        self._chk(self.L.clrrt_tree_size(self.h, C.byref(n), C.byref(r)), "tree_size")
        return n.value, r.value

    def nodes_raw(self, first=0, count=None):
        n = self.size()[0] - first if count is None else count
        arr = (abi.Node * max(1, n))()
        if n:
            self._chk(self.L.clrrt_tree_download(self.h, first, n, arr), "tree_download")
        return arr if n else (abi.Node * 0)()

    def nodes(self):
        return nodes_to_numpy(self.nodes_raw())

    def rows(self, row_offset, nrows):
        out = np.zeros((nrows, 10))
        self._chk(self.L.clrrt_tree_rows(self.h, row_offset, nrows, out.ctypes.data_as(P(C.c_double))), "tree_rows")
        return out

    def extract_best_path(self, cap=4096):
        """extractBestPath (rrtplanner.cpp:318-368): node ids root -> goal ([] when no node reached
        the goal), the chosen node's costS and the number of goal nodes."""
        ids = np.zeros(max(1, cap), dtype=np.int32)
        n, cost, ng = C.c_int32(), C.c_float(), C.c_int64()
        self._chk(self.L.clrrt_extract_best_path(self.h, ids.ctypes.data_as(P(C.c_int32)), cap, C.byref(n),
                                                 C.byref(cost), C.byref(ng)), "extract_best_path")
        return [int(v) for v in ids[:min(n.value, cap)]], float(cost.value), int(ng.value)

    # committed path (MotionPlanner::bestNodes) and initializeTree -- include/clrrt.h
    def path_commit(self, ids):
        arr = np.ascontiguousarray(ids, dtype=np.int32)
        rem = C.c_int32()
        self._chk(self.L.clrrt_path_commit(self.h, arr.ctypes.data_as(P(C.c_int32)), len(arr), C.byref(rem)),
                  "path_commit")
        return rem.value

    def path_load(self, nodes_raw, rows):
        rows = np.ascontiguousarray(rows, dtype=np.float64).reshape(-1, 10)
        self._chk(self.L.clrrt_path_load(self.h, nodes_raw, len(nodes_raw), rows.ctypes.data_as(P(C.c_double)),
                                         len(rows)), "path_load")

    def path_size(self):
        n, r = C.c_int32(), C.c_int64()
        self._chk(self.L.clrrt_path_size(self.h, C.byref(n), C.byref(r)), "path_size")
        return n.value, r.value

    def path_download(self):
        """(headers as abi.Node array, rows (R, 10)) of the committed path."""
        n, r = self.path_size()
        nodes = (abi.Node * max(1, n))()
        rows = np.zeros((max(1, r), 10))
        self._chk(self.L.clrrt_path_download(self.h, nodes, rows.ctypes.data_as(P(C.c_double))), "path_download")
        return (nodes if n else (abi.Node * 0)()), rows[:r]

    def path_transform(self, to_world, pose):
        pose = np.ascontiguousarray(pose[:3], dtype=np.float64)
        d = abi.CLRRT_CAR_TO_WORLD if to_world else abi.CLRRT_WORLD_TO_CAR
        self._chk(self.L.clrrt_path_transform(self.h, d, pose.ctypes.data_as(P(C.c_double))), "path_transform")

    def tree_init_from_path(self, car_state):
        cs = np.zeros(6)
        cs[:min(6, len(car_state))] = np.asarray(car_state, dtype=np.float64)[:6]
        oc = C.c_int32()
        self._chk(self.L.clrrt_tree_init_from_path(self.h, cs.ctypes.data_as(P(C.c_double)), C.byref(oc)),
                  "tree_init_from_path")
        return oc.value

    def path_mpc_message(self, filtered=True):
        """(P, 8) array x, y, theta, delta, v, a, a_cmd, d_cmd of the committed path's MPC message."""
        n = C.c_int32()
        self._chk(self.L.clrrt_path_mpc_message(self.h, int(filtered), None, 0, C.byref(n)), "path_mpc_message")
        out = np.zeros((max(1, n.value), 8))
        self._chk(self.L.clrrt_path_mpc_message(self.h, int(filtered), out.ctypes.data_as(P(C.c_double)), n.value,
                                                C.byref(n)), "path_mpc_message")
        return out[:n.value]

    def expand(self, rng, n_iters=0, budget_ms=0.0, mode=CLRRT_MODE_EXACT, batch=0):
        st = abi.Stats()
        self._chk(self.L.clrrt_expand(self.h, C.byref(rng.state), n_iters, budget_ms, mode, batch, C.byref(st)),
                  "expand")
        return {k: getattr(st, k) for k, _ in abi.Stats._fields_}

    # reference-named conveniences
    def expand_tree(self, rng, n_iters=1):
        """n_iters sequential expandTree iterations (EXACT semantics)."""
        return self.expand(rng, n_iters=n_iters, mode=CLRRT_MODE_EXACT)

    def plan(self, rng, budget_ms=200.0, mode=CLRRT_MODE_BATCH, batch=0):
        """The planMotion budget loop: expand until budget_ms of wall time has elapsed."""
        return self.expand(rng, n_iters=0, budget_ms=budget_ms, mode=mode, batch=batch)

    def round_eval(self, samples, dev_out_ptr):
        n_out = C.c_int32()
        self._chk(self.L.clrrt_round_eval(self.h, samples, len(samples), C.c_void_p(dev_out_ptr), C.byref(n_out)),
                  "round_eval")
        return n_out.value

    def round_prefetch(self, next_samples):
        """Declare the next round_eval's samples: their search runs beside the coming round's rollouts
        (results unchanged; the next round_eval must pass exactly these samples to use it)."""
        self._chk(self.L.clrrt_round_prefetch(self.h, next_samples, len(next_samples)), "round_prefetch")

    def round_commit(self, dev_nodes_ptr, n, local_first=0, local_count=0):
        self._chk(self.L.clrrt_round_commit(self.h, C.c_void_p(dev_nodes_ptr), n, local_first, local_count),
                  "round_commit")

    def rows_flush(self):
        """Write the deferred trajectory rows of the last commit (clrrt_rows_flush)."""
        self._chk(self.L.clrrt_rows_flush(self.h), "rows_flush")

    def simulate_batch(self, jobs, rows=False):
        """jobs: list of (parent, gb, sx, sy).  Returns a list of result dicts (+ rows)."""
        n = len(jobs)
        arr = (abi.RolloutJob * n)()
        for i, (par, gb, sx, sy) in enumerate(jobs):
            arr[i].parent, arr[i].gb = par, gb
            arr[i].sample[0], arr[i].sample[1] = sx, sy
        out = (abi.RolloutResult * n)()
        cap = 1100 if rows else 1
        buf = np.zeros((n, cap, 10)) if rows else None
        self._chk(self.L.clrrt_rollout_batch(self.h, arr, n, out,
                                             buf.ctypes.data_as(P(C.c_double)) if rows else None, cap),
                  "rollout_batch")
        res = []
        for i in range(n):
            o = out[i]
            d = {"outcome": o.outcome, "nrows": o.nrows, "costE": o.costE, "costS": o.costS,
                 "final": np.array(o.final_state[:]), "ref_back": np.array(o.ref_back[:]),
                 "ref_vback": o.ref_vback, "ref_n": o.ref_n}
            if rows:
                d["rows"] = buf[i, :o.nrows].copy()
            res.append(d)
        return res

    def simulate(self, cases, ref_cap=1024):
        """Simulation::Simulation for explicit cases (clrrt_simulate): cases = list of (state[10], ax, ay,
        hx, hy, ref_n, goal_biased, vstart).  Returns result dicts with rows and the reference (x, y, v)."""
        n = len(cases)
        arr = (abi.SimCase * n)()
        for i, (st, ax, ay, hx, hy, rn, gb, vs) in enumerate(cases):
            for k in range(10):
                arr[i].state[k] = st[k]
            arr[i].ax, arr[i].ay, arr[i].hx, arr[i].hy, arr[i].vstart = ax, ay, hx, hy, vs
            arr[i].ref_n, arr[i].goal_biased = rn, gb
        out = (abi.RolloutResult * n)()
        cap = 1100
        rows = np.zeros((n, cap, 10))
        ref = np.zeros((n, 3, ref_cap))
        self._chk(self.L.clrrt_simulate(self.h, arr, n, out, rows.ctypes.data_as(P(C.c_double)), cap,
                                        ref.ctypes.data_as(P(C.c_double)), ref_cap), "simulate")
        res = []
        for i in range(n):
            o = out[i]
            m = min(o.ref_n, ref_cap)
            res.append({"outcome": o.outcome, "nrows": o.nrows, "costE": o.costE, "costS": o.costS,
                        "final": np.array(o.final_state[:]), "ref_n": o.ref_n, "rows": rows[i, :o.nrows].copy(),
                        "ref_x": ref[i, 0, :m].copy(), "ref_y": ref[i, 1, :m].copy(), "ref_v": ref[i, 2, :m].copy()})
        return res

    def sort_nodes_batch(self, samples, exact=True):
        """Candidate lists (ids, keys) for a list of abi.Sample; exact: std::sort order of equal keys
        (else node-index order)."""
        n = len(samples)
        arr = (abi.Sample * n)(*samples)
        ids = np.zeros((n, 10), dtype=np.int32)
        keys = np.zeros((n, 10), dtype=np.float32)
        mode = CLRRT_MODE_EXACT if exact else CLRRT_MODE_BATCH
        self._chk(self.L.clrrt_nn_batch(self.h, arr, n, mode, ids.ctypes.data_as(P(C.c_int32)),
                                        keys.ctypes.data_as(P(C.c_float))), "nn_batch")
        return ids, keys

    def counters(self):
        c = abi.Counters()
        self._chk(self.L.clrrt_get_counters(self.h, C.byref(c)), "get_counters")
        return {k: getattr(c, k) for k, _ in abi.Counters._fields_}

    def selftest_math(self, fn, a, b=None):
        a = np.ascontiguousarray(a, dtype=np.float64)
        b = np.zeros_like(a) if b is None else np.ascontiguousarray(b, dtype=np.float64)
        out = np.zeros_like(a)
        self._chk(self.L.clrrt_selftest_math(self.h, fn, a.ctypes.data_as(P(C.c_double)),
                                             b.ctypes.data_as(P(C.c_double)), len(a),
                                             out.ctypes.data_as(P(C.c_double))), "selftest_math")
        return out

    # in/out widths per CLRRT_UNIT_* (include/clrrt.h)
    UNIT_IN = {0: 11, 1: 9, 2: 9, 3: 12, 4: 2, 5: 6, 6: 7, 7: 8, 8: 8, 9: 12 + 6 * abi.UNIT_CTRL_K}
    UNIT_OUT = {0: 1, 1: 8, 2: 1, 3: 1 + 3 * abi.UNIT_PROFILE_NMAX, 4: 2, 5: 2, 6: 3, 7: 1,
                8: 1 + 3 * abi.UNIT_PROFILE_NMAX, 9: 4 + 8 * abi.UNIT_CTRL_K}

    def selftest_units(self, unit, cases):
        """Device evaluation of a hot-path unit (clrrt_selftest_units): cases [n, UNIT_IN] -> [n, UNIT_OUT]."""
        cases = np.ascontiguousarray(cases, dtype=np.float64).reshape(-1, self.UNIT_IN[unit])
        out = np.zeros((cases.shape[0], self.UNIT_OUT[unit]))
        self._chk(self.L.clrrt_selftest_units(self.h, unit, cases.ctypes.data_as(P(C.c_double)), cases.shape[0],
                                              out.ctypes.data_as(P(C.c_double))), "selftest_units")
        return out

    def work_counters(self):
        out = (C.c_int64 * 3)()
        self._chk(self.L.clrrt_work_counters(self.h, out), "work_counters")
        return {"steps": out[0], "scan_points": out[1], "box_tests": out[2]}

    def check_obs_distance(self, states):
        """checkObsDistance (collision.h:41) for states [n, 10] -> [n] (clrrt_obstacle_distance)."""
        x = np.ascontiguousarray(states, dtype=np.float64).reshape(-1, 10)
        out = np.zeros(x.shape[0])
        self._chk(self.L.clrrt_obstacle_distance(self.h, x.ctypes.data_as(P(C.c_double)), x.shape[0],
                                                 out.ctypes.data_as(P(C.c_double))), "obstacle_distance")
        return out

    def search_work(self):
        out = (C.c_int64 * 4)()
        self._chk(self.L.clrrt_search_work(self.h, out), "search_work")
        return {"bf_keys": out[0], "samples": out[1], "tiles": out[2], "exact_keys": out[3]}

    def tree_truncate(self, n):
        """Drop the nodes appended after the first n (clrrt_tree_truncate)."""
        self._chk(self.L.clrrt_tree_truncate(self.h, int(n)), "tree_truncate")

    def exact_stats(self):
        out = (C.c_int64 * 10)()
        self._chk(self.L.clrrt_exact_stats(self.h, out), "exact_stats")
        # (out[9] is reserved: a window without a result is always resolved, clrrt.h)
        return dict(zip(("rounds", "resolved", "fixup_rollouts", "conflict_rounds", "end_fixup_succeeded", "end_tie",
                         "end_key_eq_thr", "end_over_slots", "end_pushed_out"), list(out)[:9]))

    def iteration_log(self, on=True):
        self._chk(self.L.clrrt_iteration_log(self.h, 1 if on else 0), "iteration_log")

    def iterations(self):
        """The logged per-iteration records (clrrt_iteration_records) as a dict of numpy arrays."""
        n = C.c_int64()
        self._chk(self.L.clrrt_iteration_records(self.h, 0, 0, None, C.byref(n)), "iteration_records")
        arr = (abi.Iteration * max(1, n.value))()
        self._chk(self.L.clrrt_iteration_records(self.h, 0, n.value, arr, C.byref(n)), "iteration_records")
        return {f: np.array([getattr(arr[i], f) for i in range(n.value)], dtype=np.int64)
                for f, _ in abi.Iteration._fields_}

    def round_sizes(self):
        """clrrt_round_sizes: the tree size after each commit of the last expand (rounds, then the drain)."""
        n = C.c_int64()
        self._chk(self.L.clrrt_round_sizes(self.h, None, 0, C.byref(n)), "round_sizes")
        out = np.zeros(max(1, n.value), dtype=np.int64)
        self._chk(self.L.clrrt_round_sizes(self.h, out.ctypes.data_as(P(C.c_int64)), n.value, C.byref(n)), "round_sizes")
        return out[:n.value]

    def walk_audit(self, samples):
        """clrrt_walk_audit (diagnostics): per sample (n, 12) int32 -- tiles with bound <= the true 11th key kth,
        those holding a list member, feasible records with key <= kth, records past the stage-1 bound at kth,
        super-tiles with bound <= kth, explore flag, kth bits, records of the admissible tiles, of which
        infeasible / farther than kth / within kth but key > kth, admissible tiles holding a record with key <= kth,
        admissible tiles whose ref.back() disc holds the sample, their disc radii summed (mm), unbounded arcs, tiles
        inside one run of equal records, records in such runs."""
        n = len(samples)
        arr = (abi.Sample * n)(*samples)
        out = np.zeros((n, 20), dtype=np.int32)
        self._chk(self.L.clrrt_walk_audit(self.h, arr, n, out.ctypes.data_as(P(C.c_int32))), "walk_audit")
        return out

    def search_work_ex(self):
        """search_work + the walk's bound work: phase-1 super-tile bounds, super-tile visits (32 tile bounds
        each), records past the prefilter."""
        out = (C.c_int64 * 8)()
        self._chk(self.L.clrrt_search_work_ex(self.h, out), "search_work_ex")
        return {"bf_keys": out[0], "samples": out[1], "tiles": out[2], "exact_keys": out[3],
                "super_bounds": out[4], "super_visits": out[5], "queued": out[6]}

    def reset_counters(self):
        self._chk(self.L.clrrt_reset_counters(self.h), "reset_counters")

    def enable_timing(self, on=True):
        self._chk(self.L.clrrt_enable_timing(self.h, 1 if on else 0), "enable_timing")

    def set_option(self, key, value):
        self._chk(self.L.clrrt_set_option(self.h, key.encode(), int(value)), f"set_option({key})")

    def nn_stats(self):
        out = (C.c_int64 * 19)()
        self._chk(self.L.clrrt_nn_stats(self.h, out), "nn_stats")
        return {"waves": out[0], "nodes_read": out[1], "rings": out[2], "truncated_waves": out[3],
                "last_fallback_samples": out[4], "tiles_seen": out[5], "tiles_searched": out[6],
                "pairs_queued": out[7], "exact_keys": out[8], "walk_supers": out[10], "walk_tiles": out[11],
                "walk_queued": out[12], "walk_exact": out[13], "walk_clk_bounds": out[14], "walk_clk_super": out[15],
                "walk_clk_visit": out[16], "walk_clk_drain": out[17], "walk_clk_total": out[18]}

    def debug_counters(self):
        out = (C.c_int64 * 64)()
        self._chk(self.L.clrrt_debug_counters(self.h, out), "debug_counters")
        return list(out)

    def kernel_time(self, which):
        ms, n = C.c_double(), C.c_int64()
        self._chk(self.L.clrrt_kernel_time(self.h, which, C.byref(ms), C.byref(n)), "kernel_time")
        return ms.value, n.value
