"""Tree re-initialisation from the committed path (BASELINE configs[4]):
initializeTree / getNodeCost (rrtplanner.cpp:39-119), transformNodesWorldToCar / CarToworld
(transformations.cpp:289-315) and the commit logic of planMotion (motionplanner.cpp:22-54).

CPU tests pin the oracle's restatement (independent numpy recomputation of the goal flags and the
float cost recurrence, the four outcomes, transform round trips).  GPU tests run the same query
sequence on the oracle and through the C-ABI and require identical trees after every query: node
states, trajectories and float costs bit-for-bit, parent ids, goal flags and outcomes exactly.
"""
import math

import numpy as np
import pytest

import clrrt
from clrrt import abi, replan, scenes
from oracle_binding import Oracle, nodes_to_numpy

GOAL_W = (40.0, 0.0, 0.0, 0.0)


def _moving_scene(drop_208=True):
    """200 static + 20 moving obstacles (the config-5 generator).  drop_208: without moving obstacle 8,
    which crosses the lane in front of the car and can leave the goal unreachable in short runs (the
    full scene runs as kind "moving20")."""
    s = scenes.urban_scene(200, 20)
    return np.delete(s, 208, axis=0) if drop_208 else s


def _make(mode):
    return replan.default_make_params(mode)


class OracleBackend:
    def __init__(self, o, make_params):
        self.o, self.make_params = o, make_params

    def begin_query(self, pose, goal_car, obs_car):
        self.o.set_params(self.make_params(pose[4], goal_car))
        self.o.set_obstacles(obs_car)
        self.o.path_transform(False, pose)
        return self.o.initialize_tree([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])

    def end_query(self, pose):
        ids = self.o.extract_best_path()
        self.o.path_commit(ids)
        self.o.path_transform(True, pose)
        nodes = self.o.path_nodes()
        rows = [self.o.path_rows(i) for i in range(len(nodes))]
        return ids, (np.concatenate(rows) if rows else np.zeros((0, 10)))


def _grown_oracle(mode=abi.CLRRT_COLLISION_STUB, obs=None, seed=3, iters=300):
    o = Oracle(abi.default_params(collision_mode=mode), obs)
    Oracle.srand(seed)
    o.init_tree()
    o.expand(iters)
    return o


def _node_cost_ref(p, parent_cost, rows):
    """getNodeCost rrtplanner.cpp:104-119 in numpy-free Python (STUB collision: Dobs = 100)."""
    cost = float(parent_cost)
    for r in rows:
        kappa = math.tan(r[3]) / p.veh.L
        cost += p.Wcost[0] * r[4] * p.sim_dt + p.Wcost[1] * abs(kappa) + p.Wcost[2] * math.exp(-p.Wcost[3] * 100.0)
    return cost


# ------------------------------------------------------------------------------------ CPU (oracle)
def test_oracle_no_committed_path_gives_root():
    o = _grown_oracle()
    o.path_commit([])
    assert o.initialize_tree([0, 0, 0, 0.1, 2.0, 0.3]) == abi.REINIT_EMPTY
    n = o.nodes()
    assert len(n["parent"]) == 1 and n["parent"][0] == -1
    assert np.array_equal(n["state"][0], [0, 0, 0, 0.1, 2.0, 0.3, 0, 0, 0, 0])


def test_oracle_transform_round_trip():
    o = _grown_oracle()
    ids = o.extract_best_path()
    assert len(ids) >= 2
    o.path_commit(ids)
    before = nodes_to_numpy(o.path_nodes())
    rows_before = [o.path_rows(i) for i in range(len(ids))]
    pose = (3.5, -1.25, 0.4)
    o.path_transform(True, pose)
    o.path_transform(False, pose)
    after = nodes_to_numpy(o.path_nodes())
    assert np.allclose(after["state"], before["state"], atol=1e-12)
    for i in range(len(ids)):
        r = o.path_rows(i)
        assert np.allclose(r[:, :2], rows_before[i][:, :2], atol=1e-12)
        assert np.array_equal(r[:, 2:], rows_before[i][:, 2:])  # only x, y of rows are transformed


def test_oracle_reinit_kept_chain_costs_and_goal_flags():
    o = _grown_oracle()
    ids = o.extract_best_path()
    o.path_commit(ids)
    path_rows = [o.path_rows(i) for i in range(len(ids))]
    hdr = nodes_to_numpy(o.path_nodes())
    # shift the car 1 m forward: the frame moves, nodes whose last row is behind are erased
    pose = (1.0, 0.0, 0.0)
    o.path_transform(False, pose)
    rows_car = [o.path_rows(i) for i in range(len(ids))]
    oc = o.initialize_tree([0, 0, 0, 0, 1.0, 0])
    assert oc == abi.REINIT_KEPT
    keep = [i for i in range(len(ids)) if not (rows_car[i][-1, 0] < 0)]
    t = o.nodes()
    assert len(t["parent"]) == len(keep)
    assert list(t["parent"]) == list(range(-1, len(keep) - 1))
    p = o.params
    parent = 0.0
    for k, i in enumerate(keep):
        c = np.float32(_node_cost_ref(p, parent, rows_car[i]))
        assert t["costS"][k] == c, (k, t["costS"][k], c)
        parent = float(c)
        r = rows_car[i]
        dg = np.sqrt((r[:, 0] - p.goal[0]) ** 2 + r[:, 1] ** 2)
        g = np.any((dg <= 1) & (np.abs(r[:, 2] - p.goal[2]) <= 0.05) & (np.abs(r[:, 4] - p.goal[3]) <= 0.1))
        assert bool(t["goal"][k]) == bool(g)
        assert np.array_equal(o.rows(k), r)
        assert t["costE"][k] == hdr["costE"][i]


def test_oracle_reinit_all_erased():
    o = _grown_oracle()
    o.path_commit(o.extract_best_path())
    o.path_transform(False, (1000.0, 0.0, 0.0))
    assert o.initialize_tree([0, 0, 0, 0, 0, 0]) == abi.REINIT_ALL_ERASED
    assert o.size() == 1


def test_oracle_reinit_collision_gives_root():
    o = _grown_oracle(abi.CLRRT_COLLISION_OBB, scenes.urban_scene(50))
    ids = o.extract_best_path()
    o.path_commit(ids)
    r = o.path_rows(len(ids) - 1)[-1]
    o.set_obstacles(np.array([[r[0], r[1], 0.0, 2.0, 2.0, 0.0, 0.0]]))
    assert o.initialize_tree([0, 0, 0, 0, 0, 0]) == abi.REINIT_COLLISION
    assert o.size() == 1


def test_oracle_replanning_loop_runs():
    obs = _moving_scene()
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), None)
    Oracle.srand(5)
    log = replan.run_queries(OracleBackend(o, _make(abi.CLRRT_COLLISION_OBB)), lambda q: o.expand(120), 4, obs,
                             GOAL_W, v0=1.0)
    assert [e[1] for e in log][0] == abi.REINIT_EMPTY
    assert any(e[1] == abi.REINIT_KEPT for e in log[1:]), [e[1] for e in log]


def _mpc_ref(seg_rows, filtered):
    """generateMPCmessage / filterMPCmessage (motionplanner.cpp:103-151) in plain Python."""
    msg = [[r[0], r[1], r[2], r[3], r[4], r[5], r[8], r[9]] for rows in seg_rows for r in rows[1:]]
    if not filtered or not msg:
        return np.array(msg).reshape(-1, 8)
    out, d = [], 0.0
    for i in range(1, len(msg)):
        if d == 0:
            out.append(msg[i][:3] + [math.nan] + msg[i][4:])
        d += math.sqrt((msg[i][0] - msg[i - 1][0]) ** 2 + (msg[i][1] - msg[i - 1][1]) ** 2)
        if d >= 5:
            d = 0.0
    return np.array(out).reshape(-1, 8)


def test_oracle_mpc_message():
    o = _grown_oracle(iters=400)
    ids = o.extract_best_path()
    o.path_commit(ids)
    o.path_transform(True, (10.0, 5.0, 0.3))
    seg = [o.path_rows(i) for i in range(len(ids))]
    for filtered in (False, True):
        got, ref = o.path_mpc_message(filtered), _mpc_ref(seg, filtered)
        assert got.shape == ref.shape and got.shape[0] > 3
        assert np.array_equal(got, ref, equal_nan=True)
    o.path_commit([])
    assert o.path_mpc_message(True).shape == (0, 8)


# ------------------------------------------------------------------------------------------- GPU
def _planner(mode, max_batch=256):
    return clrrt.Planner(clrrt.default_params(collision_mode=mode), max_nodes=1 << 16, max_rows=1 << 21,
                         max_batch=max_batch)


def _assert_same_tree(o, pl, label):
    on, gn = o.nodes(), pl.nodes()
    assert len(on["parent"]) == len(gn["parent"]), label
    assert np.array_equal(on["parent"], gn["parent"]), label
    assert np.array_equal(on["goal"], gn["goal"]), label
    assert np.array_equal(gn["state"].view(np.uint64), on["state"].view(np.uint64)), label
    assert np.array_equal(gn["costS"].view(np.uint32), on["costS"].view(np.uint32)), label
    assert np.array_equal(gn["costE"].view(np.uint32), on["costE"].view(np.uint32)), label
    for i in range(len(on["parent"])):
        rows = pl.rows(int(gn["row_offset"][i]), int(gn["nrows"][i]))
        assert np.array_equal(rows.view(np.uint64), np.ascontiguousarray(o.rows(i)).view(np.uint64)), (label, i)


@pytest.mark.gpu
def test_path_transform_parity():
    o = _grown_oracle(abi.CLRRT_COLLISION_OBB, scenes.urban_scene(200))
    pl = _planner(abi.CLRRT_COLLISION_OBB)
    pl.set_obstacles(scenes.urban_scene(200))
    pl.tree_init()
    pl.expand(clrrt.Rng(3), n_iters=300, mode=clrrt.CLRRT_MODE_EXACT, batch=256)
    ids = o.extract_best_path()
    assert pl.extract_best_path()[0] == ids and len(ids) >= 2
    o.path_commit(ids)
    assert pl.path_commit(ids) == 0
    for to_world, pose in ((True, (12.5, -3.0, 0.7)), (False, (14.0, -2.0, 0.9)), (False, (-5.0, 1.0, -2.5))):
        o.path_transform(to_world, pose)
        pl.path_transform(to_world, pose)
        on, (gr, grow) = nodes_to_numpy(o.path_nodes()), pl.path_download()
        gn = nodes_to_numpy(gr)
        assert np.array_equal(gn["state"].view(np.uint64), on["state"].view(np.uint64))
        for f in ("ref_front", "ref_back"):
            assert np.array_equal(gn[f].view(np.uint64), on[f].view(np.uint64)), f
        assert np.array_equal(gn["ang_par"].view(np.uint64), on["ang_par"].view(np.uint64))  # glibc atan2
        orow = np.concatenate([o.path_rows(i) for i in range(len(ids))])
        assert np.array_equal(grow.view(np.uint64), orow.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["stub", "obb", "moving", "moving20"])
def test_replanning_queries_parity(kind):
    """Five 5 Hz queries (EXACT expansion, 150 iterations each): after every re-init and every
    expansion the GPU tree equals the oracle's; poses come from the oracle's committed path."""
    mode = abi.CLRRT_COLLISION_STUB if kind == "stub" else abi.CLRRT_COLLISION_OBB
    obs = {"stub": np.zeros((0, 7)), "obb": scenes.urban_scene(200), "moving": _moving_scene(),
           "moving20": _moving_scene(drop_208=False)}[kind]
    make = _make(mode)
    o = Oracle(abi.default_params(collision_mode=mode), None)
    pl = _planner(mode)
    ob, gb = OracleBackend(o, make), replan.PlannerBackend(pl, make)
    seed = 11
    Oracle.srand(seed)
    rng = clrrt.Rng(seed)
    pose = np.array([0.0, 0.0, 0.0, 0.0, 1.0, 0.0])
    outcomes, path_lens = [], []
    for q in range(5):
        t = q * replan.QUERY_PERIOD
        goal_c = replan.goal_in_car_frame(GOAL_W, pose)
        obs_c = replan.obstacles_in_car_frame(obs, t, pose)
        oc_o = ob.begin_query(pose, goal_c, obs_c)
        oc_g = gb.begin_query(pose, goal_c, obs_c)
        assert oc_o == oc_g, (q, oc_o, oc_g)
        outcomes.append(oc_o)
        _assert_same_tree(o, pl, f"{kind} q{q} re-init")
        o.expand(150)
        pl.expand(rng, n_iters=150, mode=clrrt.CLRRT_MODE_EXACT, batch=256)
        _assert_same_tree(o, pl, f"{kind} q{q} expanded")
        ids_o, rows_o = ob.end_query(pose)
        ids_g, rows_g = gb.end_query(pose)
        assert ids_o == ids_g
        path_lens.append(len(ids_o))
        assert np.array_equal(rows_g.view(np.uint64), rows_o.view(np.uint64))
        for filtered in (False, True):
            mo, mg = o.path_mpc_message(filtered), pl.path_mpc_message(filtered)
            assert mo.shape == mg.shape and np.array_equal(mg.view(np.uint64), mo.view(np.uint64)), (q, filtered)
        pose = replan.advance_pose(pose, rows_o)
    print(kind, "outcomes", outcomes, "committed path lengths", path_lens)
    assert outcomes[0] == abi.REINIT_EMPTY
    # a query without a goal-reaching node commits nothing and the next one restarts from the root
    for q in range(1, 5):
        if path_lens[q - 1] == 0:
            assert outcomes[q] == abi.REINIT_EMPTY, (q, outcomes)


@pytest.mark.gpu
def test_moving20_batch_reinit_from_found_path():
    """Config 5's defining branch on the full 20-mover scene: BATCH queries (B = 256, two rounds each,
    rrtplanner.cpp:123-174 in BATCH tie order) find a goal-reaching path in query 0, and queries 1-3
    re-initialise from it (initializeTree, rrtplanner.cpp:39-95: outcome KEPT = 3).  The goal sits 20 m
    ahead instead of 40 m so the oracle reaches it in seconds; the trees equal the oracle's after every
    re-init and every expansion."""
    mode = abi.CLRRT_COLLISION_OBB
    obs = _moving_scene(drop_208=False)
    make = _make(mode)
    B, R, seed, goal_w = 256, 2, 11, (20.0, 0.0, 0.0, 0.0)
    o = Oracle(abi.default_params(collision_mode=mode), None)
    pl = _planner(mode, max_batch=B)
    ob, gb = OracleBackend(o, make), replan.PlannerBackend(pl, make)
    Oracle.srand(seed)
    rng = clrrt.Rng(seed)
    pose = np.array([0.0, 0.0, 0.0, 0.0, 1.0, 0.0])
    outcomes, path_lens = [], []
    for q in range(4):
        t = q * replan.QUERY_PERIOD
        goal_c = replan.goal_in_car_frame(goal_w, pose)
        obs_c = replan.obstacles_in_car_frame(obs, t, pose)
        oc_o = ob.begin_query(pose, goal_c, obs_c)
        oc_g = gb.begin_query(pose, goal_c, obs_c)
        assert oc_o == oc_g, (q, oc_o, oc_g)
        outcomes.append(oc_o)
        _assert_same_tree(o, pl, f"q{q} re-init")
        o.expand_batch(B * R, B, stable=True)
        st = pl.expand(rng, n_iters=B * R, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        assert st["rounds"] == R
        _assert_same_tree(o, pl, f"q{q} expanded")
        ids_o, rows_o = ob.end_query(pose)
        ids_g, rows_g = gb.end_query(pose)
        assert ids_o == ids_g
        path_lens.append(len(ids_o))
        assert np.array_equal(rows_g.view(np.uint64), rows_o.view(np.uint64))
        pose = replan.advance_pose(pose, rows_o)
    print("moving20 BATCH outcomes", outcomes, "committed path lengths", path_lens)
    assert outcomes[0] == abi.REINIT_EMPTY and path_lens[0] > 0
    assert outcomes.count(abi.REINIT_KEPT) >= 2, outcomes
    pl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["erased", "collision", "kept"])
def test_reinit_outcomes_parity(case):
    """ALL_ERASED, COLLISION and KEPT outcomes through the C-ABI match the oracle."""
    obs = scenes.urban_scene(50)
    o = _grown_oracle(abi.CLRRT_COLLISION_OBB, obs, seed=4, iters=250)
    pl = _planner(abi.CLRRT_COLLISION_OBB)
    pl.set_obstacles(obs)
    pl.tree_init()
    pl.expand(clrrt.Rng(4), n_iters=250, mode=clrrt.CLRRT_MODE_EXACT, batch=256)
    ids = o.extract_best_path()
    assert ids and pl.extract_best_path()[0] == ids
    o.path_commit(ids)
    pl.path_commit(ids)
    if case == "erased":
        o.path_transform(False, (1000.0, 0.0, 0.0))
        pl.path_transform(False, (1000.0, 0.0, 0.0))
    elif case == "collision":
        r = o.path_rows(len(ids) - 1)[-1]
        blocker = np.array([[r[0], r[1], 0.0, 2.0, 2.0, 0.0, 0.0]])
        o.set_obstacles(blocker)
        pl.set_obstacles(blocker)
    a, b = o.initialize_tree([0, 0, 0, 0.05, 1.5, 0.1]), pl.tree_init_from_path([0, 0, 0, 0.05, 1.5, 0.1])
    want = {"erased": abi.REINIT_ALL_ERASED, "collision": abi.REINIT_COLLISION, "kept": abi.REINIT_KEPT}[case]
    assert a == b == want, (case, a, b)
    _assert_same_tree(o, pl, case)
