"""Tree-level parity pinned to the REFERENCE'S OWN CODE (tests/ref_tree.py, tests/golden/ref_tree.npz).

The fixture holds the outputs of the reference's own sampleAroundVehicle, sortNodesExplore/Optimize,
Simulation, expandTree, initializeTree, extractBestPath and transformNodes* compiled from verbatim line
ranges of /root/reference (oracle/Makefile `ref`, CMake Release flags).  Bar: bit for bit everywhere
(headers, every trajectory row through its digest, candidate-list ids, RNG draws).
  * CPU: the product's host code (clrrt_draw_samples, clrrt_params_default) and the oracle against the
    fixture; when the reference build is present, a live re-run of the reference against the fixture.
  * GPU: the device (candidate lists under every search strategy, rollout batches, EXACT expansion,
    5 Hz re-initialisation) against the fixture.
"""
import os

import numpy as np
import pytest

import ref_tree as T
import ref_units as RU

FIX = np.load(T.FIXTURE, allow_pickle=False)
SORT_COLS = [0, 1, 2, 4, 6, 11, 16, 17, 18, 19, 20]  # tests/golden/make_ref_tree.py


def sort_tree(tag):
    h = FIX[f"sort_{tag}_tree"]
    H = np.zeros((len(h), T.NODE_W))
    H[:, SORT_COLS] = h
    H[:, 10] = -1
    H[:, 12] = H[:, 11]
    return H


def assert_headers(got, want, label):
    assert got.shape[0] == want.shape[0], f"{label}: {got.shape[0]} nodes vs {want.shape[0]}"
    bad = RU.mismatches(got[:, T.HDR_COLS], want[:, T.HDR_COLS])
    assert len(bad) == 0, f"{label}: {len(bad)} headers differ, first {bad[:5]}"


def assert_digests(got_rows, want, label):
    d = T.digests(got_rows)
    bad = np.nonzero(np.any(d != want, axis=1))[0]
    assert len(bad) == 0, f"{label}: {len(bad)} trajectories differ, first {bad[:5]}"


# ------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("gi", range(3))
def test_product_samples_match_reference(gi):
    """clrrt_draw_samples (the product's host sampler) draws the reference's samples and heuristics
    (sampleAroundVehicle rrtplanner.cpp:187-201 + :142-143) from the same glibc stream, bit for bit."""
    import clrrt
    g = tuple(FIX["sample_goals"][gi])
    p = T.params(0, g)
    for si, seed in enumerate(FIX["sample_seeds"]):
        want = FIX["sample_out"][gi, si]
        xy, ex = clrrt.samples_to_numpy(clrrt.Rng(int(seed)).draw_samples(p, len(want)))
        assert len(RU.mismatches(xy, want[:, :2])) == 0, (g, seed)
        assert np.array_equal(ex, (want[:, 2] <= 0.7).astype(np.int32)), (g, seed)


def test_product_ref_res_matches_reference():
    """clrrt_params_default's ref_res = updateReferenceResolution(v0) (controller.cpp:18-21)."""
    import clrrt
    for v, (dla, res) in zip(FIX["lookahead_v"], FIX["lookahead_out"]):
        assert clrrt.default_params(v0=float(v)).ref_res == res, v


@pytest.mark.parametrize("tag", ["a", "b"])
def test_oracle_candidate_lists_match_reference(tag):
    import ctypes as C
    from oracle_binding import Oracle
    H, S = sort_tree(tag), FIX[f"sort_{tag}_samples"]
    o = Oracle(T.params(0))
    o.L.orc_load_tree(o.h, T.node_array(H), len(H))
    ids, cnt = FIX[f"sort_{tag}_ids"], FIX[f"sort_{tag}_n"]
    for j in range(len(S)):
        oi = np.zeros(10, np.int32)
        ok = np.zeros(10, np.float32)
        m = o.L.orc_sort_nodes(o.h, S[j, 0], S[j, 1], int(S[j, 2]), 0, oi.ctypes.data_as(C.POINTER(C.c_int)),
                               ok.ctypes.data_as(C.POINTER(C.c_float)))
        assert m == cnt[j] and np.array_equal(oi[:m], ids[j, :m]), j


@pytest.mark.parametrize("tag", list(T.SIM_CASES))
def test_oracle_rollouts_match_reference(tag):
    from oracle_binding import Oracle
    Hp, J = FIX[f"sim_{tag}_parents"], FIX[f"sim_{tag}_jobs"]
    coll, (ns, nm), _ = T.SIM_CASES[tag]
    obs = T.scene(ns, nm)
    o = Oracle(T.sim_params(tag), obs if len(obs) else None)
    o.L.orc_load_tree(o.h, T.node_array(Hp), len(Hp))
    meta, rows = T.oracle_simulate(o, J)
    assert len(RU.mismatches(meta[:, T.SIM_META_COLS], FIX[f"sim_{tag}_meta"][:, T.SIM_META_COLS])) == 0
    assert_digests(rows, FIX[f"sim_{tag}_digest"], tag)


@pytest.mark.parametrize("case", T.EXPAND_CASES, ids=[c[0] for c in T.EXPAND_CASES])
def test_oracle_expand_matches_reference(case):
    from oracle_binding import Oracle
    name, coll, (ns, nm), seed, iters, goal = case
    o = Oracle(T.params(coll, goal), T.scene(ns, nm) if ns + nm else None)
    Oracle.srand(seed)
    o.init_tree()
    o.expand(iters)
    assert_headers(T.headers_from_numpy(o.nodes()), FIX[f"expand_{name}_hdr"], name)
    assert_digests([o.rows(i) for i in range(o.size())], FIX[f"expand_{name}_digest"], name)
    import ctypes as C
    buf = (C.c_long * 5)()
    o.L.orc_counters(o.h, buf)
    assert list(buf[:4]) == list(FIX[f"expand_{name}_counters"]), name  # sim_count and failure counters


def _oracle_replan():
    from clrrt import replan
    from oracle_binding import Oracle
    make = replan.default_make_params(0)
    o = Oracle(T.params(0), None)
    Oracle.srand(T.REPLAN_SEED)
    outcomes = []
    for q in range(T.REPLAN_QUERIES):
        pose = FIX["replan_poses"][q]
        gc = replan.goal_in_car_frame(T.REPLAN_GOAL, pose)
        o.set_params(make(pose[4], gc))
        o.set_obstacles(np.zeros((0, 7)))
        o.path_transform(False, pose)
        outcomes.append(o.initialize_tree([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]]))
        yield q, "init", o
        o.expand(T.REPLAN_ITERS)
        yield q, "tree", o
        ids = o.extract_best_path()
        o.path_commit(ids)
        o.path_transform(True, pose)
        yield q, "best", o


def test_oracle_replanning_matches_reference():
    """planMotion with commit_path = 1 (motionplanner.cpp:14-54): transformNodesWorldToCar ->
    initializeTree -> expandTree x REPLAN_ITERS -> extractBestPath -> transformNodesCarToworld; trees and
    committed paths equal the reference's after every step of 4 queries (re-init outcomes 0, 3, 3, 3)."""
    for q, step, o in _oracle_replan():
        if step in ("init", "tree"):
            assert_headers(T.headers_from_numpy(o.nodes()), FIX[f"replan_q{q}_{step}_hdr"], f"q{q} {step}")
            assert_digests([o.rows(i) for i in range(o.size())], FIX[f"replan_q{q}_{step}_digest"], f"q{q} {step}")
        else:
            from oracle_binding import nodes_to_numpy
            hb = T.headers_from_numpy(nodes_to_numpy(o.path_nodes()))
            assert_headers(hb, FIX[f"replan_q{q}_best_hdr"], f"q{q} best")
            rows = [o.path_rows(i) for i in range(len(hb))]
            assert np.array_equal(T.digest(np.concatenate(rows)), FIX[f"replan_q{q}_best_rows_digest"])
    assert list(FIX["replan_outcomes"]) == [0, 3, 3, 3]


_HAVE_REF = os.path.exists(os.path.join(RU.REF_DIR, "libref_units_O3.so"))
live = pytest.mark.skipif(not _HAVE_REF, reason="reference build absent (no /root/reference)")


@live
@pytest.mark.parametrize("case", T.EXPAND_CASES[:2], ids=[c[0] for c in T.EXPAND_CASES[:2]])
def test_reference_build_reproduces_fixture(case):
    """The reference's own expandTree, re-run here, still gives the committed fixture."""
    H, rows, cnt = T.ref_expand(T.ref_lib(), case)
    assert_headers(H, FIX[f"expand_{case[0]}_hdr"], case[0])
    assert_digests(rows, FIX[f"expand_{case[0]}_digest"], case[0])


# ------------------------------------------------------------------------------------------- GPU
def _planner(coll=0, goal=(40.0, 0.0, 0.0, 0.0), max_nodes=1 << 15, max_batch=512):
    import clrrt
    return clrrt.Planner(T.params(coll, goal), device=0, max_nodes=max_nodes, max_rows=1 << 20, max_batch=max_batch)


STRATEGIES = {"default": {}, "brute": {"nn_exact_fused": 0, "nn_walk_min": 1 << 40},
              "walk": {"nn_exact_fused": 0, "nn_walk_min": 0},
              "walk_stateless": {"nn_exact_fused": 0, "nn_walk_min": 0, "nn_walk_stateless": 1},
              "walk_split": {"nn_exact_fused": 0, "nn_walk_min": 0, "nn_walk_budget_tiles": 1, "nn_walk_budget_keys": 1}}


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", list(STRATEGIES))
@pytest.mark.parametrize("tag", ["a", "b"])
def test_device_candidate_lists_match_reference(tag, strategy):
    """sortNodesExplore / sortNodesOptimize (rrtplanner.cpp:227-268): the device's EXACT lists (ties in
    the reference's std::sort order, over hundreds of copies of the root) equal the reference's, under
    every nearest-node strategy; the keys equal the oracle's dubinsDistance."""
    import clrrt
    from clrrt import abi
    H, S = sort_tree(tag), FIX[f"sort_{tag}_samples"]
    pl = _planner(max_nodes=16384)
    try:
        for k, v in STRATEGIES[strategy].items():
            pl.set_option(k, v)
        pl.tree_load(T.node_array(H))
        samples = (abi.Sample * len(S))()
        for j, s in enumerate(S):
            samples[j].x, samples[j].y, samples[j].explore = s[0], s[1], int(s[2])
        ids, keys = pl.sort_nodes_batch(samples, exact=True)
        want, cnt = FIX[f"sort_{tag}_ids"], FIX[f"sort_{tag}_n"]
        for j in range(len(S)):
            m = int(cnt[j])
            assert np.array_equal(ids[j, :m], want[j, :m]), (j, ids[j], want[j])
            assert m == 10 or ids[j, m] < 0, (j, ids[j])
        # keys: dubinsDistance (+ costE for optimize) of the listed nodes, as the reference computes them
        x = np.zeros((int(cnt.sum()), 6))
        k = 0
        for j in range(len(S)):
            for i in want[j, :cnt[j]]:
                x[k] = [S[j, 0], S[j, 1], H[i, 0], H[i, 1], H[i, 2], H[i, 11]]
                k += 1
        rk = RU.run_oracle("dubins", x)
        k = 0
        for j in range(len(S)):
            col = 0 if S[j, 2] else 1
            m = int(cnt[j])
            assert np.array_equal(keys[j, :m].astype(np.float64), rk[k:k + m, col]), j
            k += m
    finally:
        pl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("tag", list(T.SIM_CASES))
def test_device_rollouts_match_reference(tag):
    """Simulation (simulation.cpp:36-143) from loaded parents: outcome, rows, costs, reference end and
    every trajectory row equal the reference's (stub_w2: the exp cost term; obb_bend: the lane cost)."""
    Hp, J = FIX[f"sim_{tag}_parents"], FIX[f"sim_{tag}_jobs"]
    coll, (ns, nm), _ = T.SIM_CASES[tag]
    pl = _planner(coll)
    try:
        pl.set_params(T.sim_params(tag))
        pl.set_obstacles(T.scene(ns, nm))
        pl.tree_load(T.node_array(Hp))
        meta, rows = T.device_simulate(pl, J)
        bad = RU.mismatches(meta[:, T.SIM_META_COLS], FIX[f"sim_{tag}_meta"][:, T.SIM_META_COLS])
        assert len(bad) == 0, (bad[:5], meta[bad[:2]], FIX[f"sim_{tag}_meta"][bad[:2]])
        assert_digests(rows, FIX[f"sim_{tag}_digest"], tag)
        full = FIX[f"sim_{tag}_rows"]
        for k in range(len(full)):
            n = int(FIX[f"sim_{tag}_meta"][k, 1])
            assert np.array_equal(rows[k].view(np.uint64), full[k, :n].view(np.uint64)), k
    finally:
        pl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", T.EXPAND_CASES, ids=[c[0] for c in T.EXPAND_CASES])
def test_device_expand_matches_reference(case):
    """expandTree (rrtplanner.cpp:123-174) EXACT mode: the device tree equals the reference's node for
    node (headers, float costs, every trajectory row) with the same glibc seed."""
    import clrrt
    name, coll, (ns, nm), seed, iters, goal = case
    pl = _planner(coll, goal, max_batch=128)
    try:
        pl.set_obstacles(T.scene(ns, nm))
        pl.tree_init()
        st = pl.expand(clrrt.Rng(seed), n_iters=iters, mode=clrrt.CLRRT_MODE_EXACT, batch=128)
        assert st["iterations"] == iters
        g = pl.nodes()
        assert_headers(T.headers_from_numpy(g), FIX[f"expand_{name}_hdr"], name)
        rows = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in range(len(g["parent"]))]
        assert_digests(rows, FIX[f"expand_{name}_digest"], name)
        c = pl.counters()
        want = FIX[f"expand_{name}_counters"]
        assert (c["sim_count"], c["fail_collision"], c["fail_acclimit"], c["fail_iterlimit"]) == tuple(want), (c, want)
    finally:
        pl.close()


@pytest.mark.gpu
def test_device_replanning_matches_reference():
    """Four 5 Hz queries (commit_path = 1) through the C-ABI: the re-initialised tree, the expanded tree
    and the committed path (world frame) equal the reference's after every query."""
    import clrrt
    from clrrt import replan
    make = replan.default_make_params(0)
    pl = _planner(0, max_batch=128)
    try:
        rng = clrrt.Rng(T.REPLAN_SEED)
        for q in range(T.REPLAN_QUERIES):
            pose = FIX["replan_poses"][q]
            gc = replan.goal_in_car_frame(T.REPLAN_GOAL, pose)
            pl.set_params(make(pose[4], gc))
            pl.set_obstacles(np.zeros((0, 7)))
            pl.path_transform(False, pose)
            oc = pl.tree_init_from_path([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])
            assert oc == FIX["replan_outcomes"][q]
            for step in ("init", "tree"):
                if step == "tree":
                    pl.expand(rng, n_iters=T.REPLAN_ITERS, mode=clrrt.CLRRT_MODE_EXACT, batch=128)
                g = pl.nodes()
                assert_headers(T.headers_from_numpy(g), FIX[f"replan_q{q}_{step}_hdr"], f"q{q} {step}")
                rows = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in range(len(g["parent"]))]
                assert_digests(rows, FIX[f"replan_q{q}_{step}_digest"], f"q{q} {step}")
            ids, _, _ = pl.extract_best_path()
            pl.path_commit(ids)
            pl.path_transform(True, pose)
            nodes, prow = pl.path_download()
            assert_headers(T.headers_from_numpy(clrrt.nodes_to_numpy(nodes)), FIX[f"replan_q{q}_best_hdr"], f"q{q} best")
            assert np.array_equal(T.digest(prow), FIX[f"replan_q{q}_best_rows_digest"]), q
    finally:
        pl.close()
