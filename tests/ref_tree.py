"""Tree-level pins to the reference's OWN code — TEST INFRASTRUCTURE.

oracle/_ref/libref_units_O3.so (oracle/Makefile `ref`, oracle/ref_units.cpp) holds, compiled from
verbatim line ranges of /root/reference, the reference's
  sampleAroundVehicle + the heuristic draw   rrtplanner.cpp:187-201, 142            (a2, a3)
  sortNodesExplore / sortNodesOptimize       rrtplanner.cpp:227-268 (+ dubinsDistance, feasibleNode)  (a4)
  Simulation (ctor + propagate)              simulation.cpp:36-143 (+ Controller, references)       (a5-a12)
  expandTree                                 rrtplanner.cpp:123-174                                 (a1)
  initializeTree / getNodeCost               rrtplanner.cpp:39-119                                  (f1)
  transformNodesWorldToCar / CarToworld      transformations.cpp:6-17, 113-120, 289-315             (f1)
  extractBestPath                            rrtplanner.cpp:318-368                                 (f2)
  updateLookahead / updateReferenceResolution controller.cpp:13-21                                  (a14)
This module builds the cases, runs them on the reference build, the oracle and the device, and
reduces trajectories to per-node digests (tests/golden/make_ref_tree.py writes the fixture
tests/golden/ref_tree.npz; tests/test_ref_tree.py compares).
"""
import ctypes as C
import hashlib
import math
import os

import numpy as np

import ref_units as RU

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "ref_tree.npz")
NODE_W = 22  # ref_units.cpp export_node: state[10], parent, costE, costS, goal, nrows, refN, front, back, vback, nv
P = C.POINTER
dp = RU._dp

# ------------------------------------------------------------------------------------------- configs
# (name, collision mode, obstacles (static, moving), seed, iterations, goal)
EXPAND_CASES = [
    ("stub_s1", 0, (0, 0), 1, 200, (40.0, 0.0, 0.0, 0.0)),
    ("obb200_s3", 1, (200, 0), 3, 300, (40.0, 0.0, 0.0, 0.0)),
    ("obb50m10_s7", 1, (50, 10), 7, 300, (40.0, 0.0, 0.0, 0.0)),
    ("stub_goal_s5", 0, (0, 0), 5, 250, (30.0, -6.0, -0.4, 2.0)),
    ("obb200_goal_s9", 1, (200, 0), 9, 250, (45.0, 8.0, 0.5, 1.0)),
]
# round 4: a reference tree of >= 2000 nodes at cfg3's scene (the bench's EXACT query appends ~4.4 k)
EXPAND_CASES.append(("obb200_s11_4k", 1, (200, 0), 11, 4000, (40.0, 0.0, 0.0, 0.0)))
SAMPLE_GOALS = [(40.0, 0.0, 0.0, 0.0), (30.0, -6.0, -0.4, 2.0), (-12.0, 25.0, 2.0, 0.0)]
# Simulation sets: tag -> (collision mode, (static, moving) obstacles, parameter overrides).
#   stub_w2  : the obstacle-gap cost term Wcost[2] exp(-Wcost[3] Dobs) (simulation.cpp:91) on, with the shipped
#              stub (Dobs = 100): exp(-1) per step, glibc's exp restated on the device (clrrt_glibc.hpp)
#   obb_bend : the lane-deviation cost Wcost[4] getDistToLane (simulation.cpp:92-95, :49-53) with a sloped
#              lane (Cxy[1] = 0.05, Cxy[2] = -1, laneShifts[0] = 0.5), 200 obstacles
# (The gap term with the OBB check is not pinned to the reference: its gap reads the OBB normal
# normsY[3] that setNorms leaves unset, old_collisioncheck.cpp:74-75; tests/test_gpu_parity.py pins the
# device to the oracle's canonical normal there.)
SIM_CASES = {"stub": (0, (0, 0), {}), "obb": (1, (200, 0), {}), "moving": (1, (200, 20), {}),
             "stub_w2": (0, (0, 0), {"Wcost2": 1.0, "Wcost3": 0.01}),
             "obb_bend": (1, (200, 0), {"bend": 1, "lane_shift0": 0.5, "Cxy": (0.0, 0.05, -1.0)})}


def sim_params(tag):
    coll, _, ov = SIM_CASES[tag]
    p = params(coll)
    if "Wcost2" in ov:
        p.Wcost[2] = ov["Wcost2"]
    if "Wcost3" in ov:
        p.Wcost[3] = ov["Wcost3"]
    if "bend" in ov:
        p.bend = ov["bend"]
        p.lane_shift0 = ov["lane_shift0"]
        for i in range(3):
            p.Cxy[i] = ov["Cxy"][i]
    return p
SAMPLE_SEEDS = [1, 3, 12345]


def scene(n_static, n_moving):
    from clrrt import scenes
    if n_static == 0 and n_moving == 0:
        return np.zeros((0, 7))
    return scenes.urban_scene(n_static, n_moving)


def params(coll, goal=(40.0, 0.0, 0.0, 0.0), v0=0.0, vmax=5.0):
    import clrrt
    return clrrt.default_params(v0=v0, goal=goal, vmax=vmax, collision_mode=coll)


# ------------------------------------------------------------------------------------------- reference
_L = None


def ref_lib():
    """The reference build with the tree-level entry points typed, or None (no /root/reference)."""
    global _L
    if _L is not None:
        return _L
    L = RU.reference_lib("O3")
    if L is None:
        return None
    sig = {
        "ref_set_obstacles": [P(C.c_double), C.c_int], "ref_srand": [C.c_uint], "ref_rand": [],
        "ref_counters": [P(C.c_long)], "ref_reset_counters": [],
        "ref_lookahead_res": [C.c_int, P(C.c_double), P(C.c_double)],
        "ref_sample": [C.c_int, P(C.c_double), P(C.c_double)],
        "ref_sort_nodes": [C.c_int, P(C.c_double), C.c_int, P(C.c_double), P(C.c_int), P(C.c_int)],
        "ref_simulate": [C.c_int, P(C.c_double), C.c_int, P(C.c_double), C.c_int, P(C.c_double), P(C.c_double)],
        "ref_tree_init": [P(C.c_double)], "ref_tree_load": [C.c_int, P(C.c_double)],
        "ref_tree_expand": [C.c_long], "ref_tree_size": [], "ref_tree_nodes": [C.c_long, C.c_long, P(C.c_double)],
        "ref_tree_rows": [C.c_long, P(C.c_double)], "ref_best_path": [], "ref_best_size": [],
        "ref_best_nodes": [P(C.c_double)], "ref_best_rows": [C.c_long, P(C.c_double)],
        "ref_best_transform": [C.c_int, P(C.c_double)], "ref_initialize_tree": [P(C.c_double)],
        "ref_best_clear": [],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = C.c_long if name in ("ref_tree_size", "ref_best_path", "ref_best_size") else (
            C.c_int if name == "ref_rand" else None)
    _L = L
    return L


def ref_configure(L, p, obs):
    L.ref_config(dp(RU.config_vector(p)))
    obs = np.ascontiguousarray(obs, dtype=np.float64).reshape(-1, 7)
    L.ref_set_obstacles(dp(obs), obs.shape[0])


def ref_tree(L):
    """(headers (n, NODE_W), [rows (nrows, 10)]) of the reference driver's tree."""
    n = L.ref_tree_size()
    H = np.zeros((n, NODE_W))
    if n:
        L.ref_tree_nodes(0, n, dp(H))
    rows = []
    for i in range(n):
        r = np.zeros((int(H[i, 14]), 10))
        L.ref_tree_rows(i, dp(r))
        rows.append(r)
    return H, rows


def ref_best(L):
    n = L.ref_best_size()
    H = np.zeros((n, NODE_W))
    if n:
        L.ref_best_nodes(dp(H))
    rows = []
    for i in range(n):
        r = np.zeros((int(H[i, 14]), 10))
        L.ref_best_rows(i, dp(r))
        rows.append(r)
    return H, rows


# ------------------------------------------------------------------------------------------- digests
def digest(a):
    """20-byte SHA-1 of a float64 array's bits, NaN canonicalised (payloads are unspecified)."""
    a = np.ascontiguousarray(a, dtype=np.float64).copy()
    a[np.isnan(a)] = np.nan
    return np.frombuffer(hashlib.sha1(a.tobytes()).digest(), dtype=np.uint8)


def digests(rows_list):
    return np.stack([digest(r) for r in rows_list]) if rows_list else np.zeros((0, 20), np.uint8)


# ------------------------------------------------------------------------------------------- headers
def headers_from_numpy(nd, ref_n=None):
    """NODE_W headers from a nodes_to_numpy dict (oracle or device): the fields both sides carry
    (ref N / v.size() columns are zero: the C-ABI header does not hold them)."""
    n = len(nd["parent"])
    H = np.zeros((n, NODE_W))
    H[:, :10] = nd["state"]
    H[:, 10] = nd["parent"]
    H[:, 11] = nd["costE"]
    H[:, 12] = nd["costS"]
    H[:, 13] = nd["goal"]
    H[:, 14] = nd["nrows"]
    H[:, 16:18] = nd["ref_front"]
    H[:, 18:20] = nd["ref_back"]
    H[:, 20] = nd["ref_vback"]
    return H


HDR_COLS = list(range(15)) + [16, 17, 18, 19, 20]  # compared columns (not ref N, not v.size())


def node_array(H):
    """abi.Node records from NODE_W headers (ang_par as the reference's feasibleNode forms it,
    glibc atan2 through math.atan2)."""
    from clrrt import abi
    arr = (abi.Node * max(1, len(H)))()
    for i, h in enumerate(H):
        d = arr[i]
        for k in range(10):
            d.state[k] = h[k]
        d.ref_front[0], d.ref_front[1] = h[16], h[17]
        d.ref_back[0], d.ref_back[1] = h[18], h[19]
        d.ref_vback = h[20]
        d.ang_par = math.atan2(h[19] - h[17], h[18] - h[16])
        d.parent = int(h[10])
        d.costE = float(np.float32(h[11]))
        d.costS = float(np.float32(h[12]))
        d.goal = int(h[13])
        d.nrows = 1
        d.owner = 0
        d.row_offset = 0
    return arr if len(H) else (abi.Node * 0)()


# ------------------------------------------------------------------------------------------- cases
def sort_tree(rng, n, n_root_copies):
    """A synthetic tree of NODE_W headers for the candidate-list pin: nodes scattered over the sample
    region with headings and 2-point references, costE with exact repeats, and `n_root_copies` exact
    copies of the root (zero-length children: equal keys for every sample, the std::sort tie case),
    plus clusters of copies of a few other nodes."""
    H = np.zeros((n, NODE_W))
    x = rng.uniform(-5, 60, n); y = rng.uniform(-22, 22, n)
    th = rng.uniform(-math.pi, math.pi, n)
    L = np.where(rng.random(n) < 0.05, 0.0, rng.uniform(0.5, 25, n))
    a = th + rng.normal(0, 0.3, n)
    H[:, 0], H[:, 1], H[:, 2] = x, y, th
    H[:, 4] = rng.uniform(0, 6, n)
    H[:, 6] = rng.uniform(0, 30, n)
    H[:, 10] = -1
    ce = rng.uniform(0, 60, n)
    rep = rng.random(n) < 0.3
    ce[rep] = np.round(ce[rep])
    H[:, 11] = ce.astype(np.float32)
    H[:, 12] = H[:, 11]
    H[:, 18], H[:, 19] = x + rng.normal(0, 0.5, n), y + rng.normal(0, 0.5, n)
    H[:, 16], H[:, 17] = H[:, 18] - L * np.cos(a), H[:, 19] - L * np.sin(a)
    H[:, 20] = H[:, 4]
    # the root and its zero-length children
    H[0, :] = 0.0
    H[0, 10] = -1
    H[0, 18] = 0.9  # addInitialNode: linspace(0, 1, 10) ends at 0.9 (accumulated)
    H[0, 16] = 0.0
    k = min(n_root_copies, n - 1)
    H[1:1 + k] = H[0]
    # clusters of equal records elsewhere
    for c in range(5):
        src = int(rng.integers(1 + k, n))
        m = int(rng.integers(5, 60))
        dst = rng.integers(1 + k, n, m)
        H[dst] = H[src]
    return H


def sort_samples(rng, H, n):
    """Samples: half uniform over the sample region, half placed relative to tree nodes (just outside
    and inside turning circles, at feasibility limits), explore/optimize mixed."""
    S = np.zeros((n, 3))
    S[:, 0] = rng.uniform(-5, 60, n); S[:, 1] = rng.uniform(-20, 20, n)
    near = rng.random(n) < 0.5
    idx = rng.integers(0, len(H), n)
    d = rng.choice([0.05, 0.42, 2.0, 5.0, 9.6, 15.0], n)
    ang = rng.uniform(-math.pi, math.pi, n)
    S[near, 0] = H[idx[near], 18] + d[near] * np.cos(ang[near])
    S[near, 1] = H[idx[near], 19] + d[near] * np.sin(ang[near])
    S[:, 2] = (rng.random(n) < 0.7).astype(np.float64)
    return S


def ref_sort(L, H, S):
    n = len(S)
    ids = np.zeros((n, 10), np.int32); cnt = np.zeros(n, np.int32)
    L.ref_sort_nodes(len(H), dp(np.ascontiguousarray(H)), n, dp(np.ascontiguousarray(S)),
                     ids.ctypes.data_as(P(C.c_int)), cnt.ctypes.data_as(P(C.c_int)))
    return ids, cnt


def sim_parents(rng, n):
    """Parent nodes for rollout jobs: states around the scene with speeds 0-8 m/s, steering and
    acceleration states, 2-point references ending near the state."""
    H = np.zeros((n, NODE_W))
    H[:, 0] = rng.uniform(-2, 50, n); H[:, 1] = rng.uniform(-15, 15, n)
    H[:, 2] = rng.normal(0, 0.6, n)
    H[:, 3] = rng.uniform(-0.3, 0.3, n)
    H[:, 4] = np.where(rng.random(n) < 0.15, 0.0, rng.uniform(0, 8, n))
    H[:, 5] = rng.uniform(-1, 1, n)
    H[:, 6] = rng.uniform(0, 15, n)
    H[:, 7] = rng.integers(0, 50, n)
    H[:, 10] = -1
    H[:, 11] = rng.uniform(0, 40, n).astype(np.float32)
    H[:, 12] = rng.uniform(0, 400, n).astype(np.float32)
    H[:, 18] = H[:, 0] + 3.2 * np.cos(H[:, 2]) + rng.normal(0, 0.3, n)
    H[:, 19] = H[:, 1] + 3.2 * np.sin(H[:, 2]) + rng.normal(0, 0.3, n)
    H[:, 16] = H[:, 18] - 5 * np.cos(H[:, 2]); H[:, 17] = H[:, 19] - 5 * np.sin(H[:, 2])
    H[:, 20] = np.where(rng.random(n) < 0.3, 0.0, H[:, 4] + rng.normal(0, 0.5, n))
    H[0, :] = 0.0
    H[0, 10] = -1
    H[0, 18] = 0.9
    return H


def sim_jobs(rng, H, n):
    """Rollout jobs (parent, gb, sx, sy): samples 1-40 m ahead and around (incl. the orbiting 30-90
    degree band, very short references), ~15% goal-biased."""
    J = np.zeros((n, 4))
    J[:, 0] = rng.integers(0, len(H), n)
    J[:, 1] = (rng.random(n) < 0.15).astype(np.float64)
    p = J[:, 0].astype(int)
    d = np.where(rng.random(n) < 0.1, rng.uniform(0.3, 1.5, n), rng.uniform(1, 40, n))
    a = H[p, 2] + np.where(rng.random(n) < 0.3, rng.uniform(0.5, 1.6, n) * np.sign(rng.normal(size=n)),
                           rng.normal(0, 0.5, n))
    J[:, 2] = H[p, 18] + d * np.cos(a)
    J[:, 3] = H[p, 19] + d * np.sin(a)
    return J


def ref_simulate(L, H, J, rows_cap=520):
    n = len(J)
    meta = np.zeros((n, 10))
    rows = np.zeros((n, rows_cap, 10))
    L.ref_simulate(len(H), dp(np.ascontiguousarray(H)), n, dp(np.ascontiguousarray(J)), rows_cap, dp(meta), dp(rows))
    return meta, [rows[k, :int(meta[k, 1])] for k in range(n)]


def oracle_simulate(o, J):
    from oracle_binding import lib as olib
    L = olib()
    n = len(J)
    meta = np.zeros((n, 10))
    rows = []
    oc = C.c_int(); costs = (C.c_double * 2)(); fin = (C.c_double * 10)(); rb = (C.c_double * 3)(); rn = C.c_int()
    buf = np.zeros((520, 10))
    for k in range(n):
        nr = L.orc_simulate(o.h, int(J[k, 0]), int(J[k, 1]), J[k, 2], J[k, 3], C.byref(oc), costs, fin, rb,
                            C.byref(rn), dp(buf), 520)
        meta[k, :8] = [oc.value, nr, costs[0], costs[1], rn.value, rb[2], rb[0], rb[1]]
        rows.append(buf[:nr].copy())
    return meta, rows


def device_simulate(pl, J):
    res = pl.simulate_batch([(int(j[0]), int(j[1]), float(j[2]), float(j[3])) for j in J], rows=True)
    meta = np.zeros((len(J), 10))
    for k, r in enumerate(res):
        meta[k, :8] = [r["outcome"], r["nrows"], r["costE"], r["costS"], r["ref_n"], r["ref_vback"],
                       r["ref_back"][0], r["ref_back"][1]]
    return meta, [r["rows"] for r in res]


SIM_META_COLS = list(range(8))  # outcome, rows, costE, costS, ref N, ref.v.back(), ref back x, y


def ref_expand(L, case):
    name, coll, (ns, nm), seed, iters, goal = case
    ref_configure(L, params(coll, goal), scene(ns, nm))
    L.ref_srand(seed)
    L.ref_tree_init(dp(np.zeros(10)))
    L.ref_reset_counters()
    L.ref_tree_expand(iters)
    c = (C.c_long * 4)()
    L.ref_counters(c)
    H, rows = ref_tree(L)
    return H, rows, np.array(c[:], dtype=np.int64)


def ref_samples(L, goal, seed, n):
    out = np.zeros((n, 3))
    L.ref_srand(seed)
    L.ref_sample(n, dp(np.array(goal, dtype=np.float64)), dp(out))
    return out


# ------------------------------------------------------------------------------------------- replanning
class ReferenceBackend:
    """planMotion's five steps (motionplanner.cpp:14-54) on the reference build (stub collision: the
    unity build's checkObsDistance, which initializeTree calls on RRT.carState)."""

    def __init__(self, L, make_params):
        self.L, self.make_params = L, make_params

    def begin_query(self, pose, goal_car, obs_car):
        ref_configure(self.L, self.make_params(pose[4], goal_car), obs_car)
        self.L.ref_best_transform(0, dp(np.ascontiguousarray(pose[:3], dtype=np.float64)))
        self.L.ref_initialize_tree(dp(np.array([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])))
        return None  # initializeTree reports no outcome

    def end_query(self, pose):
        self.L.ref_best_path()
        self.L.ref_best_transform(1, dp(np.ascontiguousarray(pose[:3], dtype=np.float64)))
        H, rows = ref_best(self.L)
        return H, (np.concatenate(rows) if rows else np.zeros((0, 10)))


REPLAN_GOAL = (40.0, 0.0, 0.0, 0.0)
REPLAN_QUERIES = 4
REPLAN_ITERS = 220
REPLAN_SEED = 11
