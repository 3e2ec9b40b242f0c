"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE (the checker, never the product).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
from clrrt import abi  # noqa: E402

_LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle not built: {_LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(_LIB_PATH)
        vp, d, i, l, f = C.c_void_p, C.c_double, C.c_int, C.c_long, C.c_float
        P = C.POINTER
        sig = {
            "orc_create": (vp, [P(abi.Params)]),
            "orc_destroy": (None, [vp]),
            "orc_srand": (None, [C.c_uint]),
            "orc_rand": (i, []),
            "orc_set_params": (None, [vp, P(abi.Params)]),
            "orc_set_obstacles": (None, [vp, P(d), i]),
            "orc_init_tree": (None, [vp, P(d)]),
            "orc_expand": (None, [vp, l]),
            "orc_expand_budget": (l, [vp, d, i]),
            "orc_expand_batch": (None, [vp, l, i, i]),
            "orc_expand_batch_defer": (None, [vp, l, i, i, i, C.POINTER(C.c_long)]),
            "orc_expand_batch_defer_mt": (None, [vp, l, i, i, i, i, C.POINTER(C.c_long)]),
            "orc_tree_size": (l, [vp]),
            "orc_get_nodes": (None, [vp, l, l, P(abi.Node)]),
            "orc_node_ref_len": (l, [vp, l]),
            "orc_get_ref": (None, [vp, l, P(d), P(d), P(d)]),
            "orc_get_rows": (None, [vp, l, P(d)]),
            "orc_counters": (None, [vp, P(l)]),
            "orc_reset_counters": (None, [vp]),
            "orc_load_tree": (None, [vp, P(abi.Node), l]),
            "orc_simulate": (i, [vp, i, i, d, d, P(i), P(d), P(d), P(d), P(i), P(d), i]),
            "orc_feasible_goal_bias": (i, [vp, l]),
            "orc_sort_nodes": (i, [vp, d, d, i, i, P(i), P(f)]),
            "orc_dubins": (f, [vp, d, d, l]),
            "orc_obb_dist": (d, [d, d, f, f, f, d, d, f, f, f]),
            "orc_check_obs": (d, [vp, P(d)]),
            "orc_draw_samples": (None, [vp, i, P(d), P(i)]),
            "orc_eval_iteration": (i, [vp, d, d, i, i, P(abi.Node)]),
            "orc_eval_iterations": (None, [vp, i, P(C.c_double), P(C.c_double), P(C.c_int), i, i, P(abi.Node),
                                           P(C.c_int)]),
            "orc_eval_iterations_upto": (None, [vp, i, P(C.c_double), P(C.c_double), P(C.c_int), i, i, C.c_long,
                                                P(abi.Node), P(C.c_int), P(C.c_long)]),
            "orc_extract_best_path": (i, [vp, P(i), i]),
            "orc_path_commit": (None, [vp, P(i), i]),
            "orc_path_size": (C.c_long, [vp]),
            "orc_path_transform": (None, [vp, i, P(d)]),
            "orc_path_get_nodes": (None, [vp, P(abi.Node)]),
            "orc_path_get_rows": (None, [vp, C.c_long, P(d)]),
            "orc_initialize_tree": (i, [vp, P(d)]),
            "orc_path_mpc_message": (i, [vp, i, P(d), i]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def nodes_to_numpy(nodes):
    """Array of abi.Node -> structured numpy view (copy)."""
    raw = np.frombuffer(bytes(nodes), dtype=np.uint8).reshape(len(nodes), C.sizeof(abi.Node))
    out = {
        "state": raw[:, 0:80].copy().view(np.float64).reshape(-1, 10),
        "ref_front": raw[:, 80:96].copy().view(np.float64).reshape(-1, 2),
        "ref_back": raw[:, 96:112].copy().view(np.float64).reshape(-1, 2),
        "ref_vback": raw[:, 112:120].copy().view(np.float64).reshape(-1),
        "ang_par": raw[:, 120:128].copy().view(np.float64).reshape(-1),
        "parent": raw[:, 128:132].copy().view(np.int32).reshape(-1),
        "costE": raw[:, 132:136].copy().view(np.float32).reshape(-1),
        "costS": raw[:, 136:140].copy().view(np.float32).reshape(-1),
        "goal": raw[:, 140:144].copy().view(np.int32).reshape(-1),
        "nrows": raw[:, 144:148].copy().view(np.int32).reshape(-1),
    }
    return out


class Oracle:
    """The reference's sequential planner state (one MyRRT + the rrt_node.cpp globals)."""

    def __init__(self, params, obstacles=None):
        self.L = lib()
        self.params = params
        self.h = self.L.orc_create(C.byref(params))
        if obstacles is not None:
            self.set_obstacles(obstacles)

    def __del__(self):
        try:
            self.L.orc_destroy(self.h)
        except Exception:
            pass

    def set_params(self, params):
        self.params = params
        self.L.orc_set_params(self.h, C.byref(params))

    def set_obstacles(self, obs):
        obs = np.ascontiguousarray(obs, dtype=np.float64).reshape(-1, 7)
        self.L.orc_set_obstacles(self.h, _dp(obs), obs.shape[0])

    def init_tree(self, root=None):
        root = np.zeros(10) if root is None else np.ascontiguousarray(root, dtype=np.float64)
        self.L.orc_init_tree(self.h, _dp(root))

    @staticmethod
    def srand(seed):
        lib().orc_srand(seed)

    def expand(self, n):
        self.L.orc_expand(self.h, n)

    def expand_batch(self, n, batch, stable=True, defer_steps=0, threads=0):
        """BATCH rounds (the engine's semantics); defer_steps T > 0: deferred samples (orc_expand_batch_defer).
        threads > 0: each round's samples evaluated on that many host threads (orc_expand_batch_defer_mt, same
        tree).  Returns the number of samples deferred at least one round."""
        if threads > 0:
            nd = C.c_long(0)
            self.L.orc_expand_batch_defer_mt(self.h, n, batch, 1 if stable else 0, max(0, defer_steps), threads,
                                             C.byref(nd))
            return nd.value
        if defer_steps <= 0:
            self.L.orc_expand_batch(self.h, n, batch, 1 if stable else 0)
            return 0
        nd = C.c_long(0)
        self.L.orc_expand_batch_defer(self.h, n, batch, 1 if stable else 0, defer_steps, C.byref(nd))
        return nd.value

    def expand_budget(self, ms, wall=True):
        return self.L.orc_expand_budget(self.h, ms, 1 if wall else 0)

    def size(self):
        return self.L.orc_tree_size(self.h)

    def nodes_raw(self, first=0, count=None):
        n = self.size() if count is None else count
        arr = (abi.Node * n)()
        if n:
            self.L.orc_get_nodes(self.h, first, n, arr)
        return arr

    def nodes(self):
        return nodes_to_numpy(self.nodes_raw())

    def rows(self, i):
        nr = self.nodes_raw(i, 1)[0].nrows
        out = np.zeros((nr, 10))
        self.L.orc_get_rows(self.h, i, _dp(out))
        return out

    def ref(self, i):
        n = self.L.orc_node_ref_len(self.h, i)
        x, y, v = np.zeros(n), np.zeros(n), np.zeros(n)
        self.L.orc_get_ref(self.h, i, _dp(x), _dp(y), _dp(v))
        return x, y, v

    def counters(self):
        out = (C.c_long * 5)()
        self.L.orc_counters(self.h, out)
        return dict(zip(("sim_count", "fail_collision", "fail_acclimit", "fail_iterlimit", "rollouts"), list(out)))

    def reset_counters(self):
        self.L.orc_reset_counters(self.h)

    def load_tree(self, nodes_raw):
        self.L.orc_load_tree(self.h, nodes_raw, len(nodes_raw))

    def simulate(self, parent, gb, sx=0.0, sy=0.0, rows=False, rows_cap=512):
        oc, rn = C.c_int(), C.c_int()
        costs, fin, rb = np.zeros(2), np.zeros(10), np.zeros(3)
        buf = np.zeros((rows_cap, 10)) if rows else None
        nr = self.L.orc_simulate(self.h, parent, gb, sx, sy, C.byref(oc), _dp(costs), _dp(fin), _dp(rb),
                                 C.byref(rn), _dp(buf) if rows else None, rows_cap)
        out = {"outcome": oc.value, "nrows": nr, "costE": costs[0], "costS": costs[1], "final": fin,
               "ref_back": rb[:2].copy(), "ref_vback": rb[2], "ref_n": rn.value}
        if rows:
            out["rows"] = buf[:nr].copy()
        return out

    def sort_nodes(self, sx, sy, explore, stable=False):
        ids = (C.c_int * 64)()
        keys = (C.c_float * 64)()
        n = self.L.orc_sort_nodes(self.h, sx, sy, 1 if explore else 0, 1 if stable else 0, ids, keys)
        return list(ids[:n]), list(keys[:n])

    def dubins(self, sx, sy, node):
        return self.L.orc_dubins(self.h, sx, sy, node)

    def feasible_goal_bias(self, node):
        return bool(self.L.orc_feasible_goal_bias(self.h, node))

    def check_obs(self, x10):
        x = np.ascontiguousarray(x10, dtype=np.float64)
        return self.L.orc_check_obs(self.h, _dp(x))

    def draw_samples(self, n):
        xy = np.zeros(2 * n)
        ex = (C.c_int * n)()
        self.L.orc_draw_samples(self.h, n, _dp(xy), ex)
        return xy.reshape(n, 2), np.array(list(ex), dtype=np.int32)

    def extract_best_path(self, cap=4096):
        ids = (C.c_int * cap)()
        n = self.L.orc_extract_best_path(self.h, ids, cap)
        return list(ids[:min(n, cap)])

    def path_commit(self, ids):
        assert all(0 <= i < self.size() for i in ids), "path_commit: node id outside the tree"
        arr = (C.c_int * max(1, len(ids)))(*ids)
        self.L.orc_path_commit(self.h, arr, len(ids))

    def path_transform(self, to_world, pose):
        self.L.orc_path_transform(self.h, 1 if to_world else 0, _dp(np.ascontiguousarray(pose[:3], dtype=np.float64)))

    def path_nodes(self):
        n = self.L.orc_path_size(self.h)
        arr = (abi.Node * max(1, n))()
        if n:
            self.L.orc_path_get_nodes(self.h, arr)
        return arr if n else (abi.Node * 0)()

    def path_rows(self, i):
        nr = self.path_nodes()[i].nrows
        out = np.zeros((nr, 10))
        self.L.orc_path_get_rows(self.h, i, _dp(out))
        return out

    def path_mpc_message(self, filtered=True):
        n = self.L.orc_path_mpc_message(self.h, int(filtered), None, 0)
        out = np.zeros((max(1, n), 8))
        self.L.orc_path_mpc_message(self.h, int(filtered), _dp(out), n)
        return out[:n]

    def initialize_tree(self, car_state):
        cs = np.zeros(6)
        cs[:min(6, len(car_state))] = np.asarray(car_state, dtype=np.float64)[:6]
        return self.L.orc_initialize_tree(self.h, _dp(cs))

    def eval_iteration(self, sx, sy, explore, stable=False):
        out = (abi.Node * 2)()
        n = self.L.orc_eval_iteration(self.h, sx, sy, 1 if explore else 0, 1 if stable else 0, out)
        return [out[i] for i in range(n)]

    def eval_iterations(self, xs, ys, explore, stable=False, threads=8):
        """eval_iteration for each (x, y, explore) against the same frozen tree, on host threads."""
        n = len(xs)
        x = np.ascontiguousarray(xs, dtype=np.float64)
        y = np.ascontiguousarray(ys, dtype=np.float64)
        e = np.ascontiguousarray(explore, dtype=np.int32)
        out = (abi.Node * (2 * n))()
        cnt = np.zeros(n, dtype=np.int32)
        P = C.POINTER
        self.L.orc_eval_iterations(self.h, n, _dp(x), _dp(y), e.ctypes.data_as(P(C.c_int)), 1 if stable else 0,
                                   threads, out, cnt.ctypes.data_as(P(C.c_int)))
        return [[out[2 * k + i] for i in range(cnt[k])] for k in range(n)]

    def eval_iterations_upto(self, xs, ys, explore, upto, stable=True, threads=16):
        """eval_iterations against the first `upto` nodes of the loaded tree (a frozen round's tree inside a larger
        one); returns (records per sample, the deciding chain in steps per sample)."""
        n = len(xs)
        x = np.ascontiguousarray(xs, dtype=np.float64)
        y = np.ascontiguousarray(ys, dtype=np.float64)
        e = np.ascontiguousarray(explore, dtype=np.int32)
        out = (abi.Node * (2 * n))()
        cnt = np.zeros(n, dtype=np.int32)
        chains = np.zeros(n, dtype=np.int64)
        P = C.POINTER
        self.L.orc_eval_iterations_upto(self.h, n, _dp(x), _dp(y), e.ctypes.data_as(P(C.c_int)), 1 if stable else 0,
                                        threads, int(upto), out, cnt.ctypes.data_as(P(C.c_int)),
                                        chains.ctypes.data_as(P(C.c_long)))
        return [[out[2 * k + i] for i in range(cnt[k])] for k in range(n)], chains


def obb_dist(a, b):
    """getOBBdist KAT hook: a, b = (px, py, w, h, o)."""
    return lib().orc_obb_dist(*a, *b)
