"""extractBestPath (rrtplanner.cpp:318-368): the node chain root -> goal of the
goal node the reference's std::sort puts first.

CPU tests pin the oracle's restatement on hand-built trees; GPU tests compare the C-ABI entry
(clrrt_extract_best_path) with the oracle on EXACT-mode trees and on trees with many tied costs
(more than 16 goal nodes, so std::sort's introsort -- not its insertion-sort tail alone -- decides
the order of equal costs). Index work: the id chain must be identical.
"""
import numpy as np
import pytest

import clrrt
from clrrt import abi
from oracle_binding import Oracle


def _grown(seed=2, iters=120):
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_STUB), None)
    Oracle.srand(seed)
    o.init_tree()
    o.expand(iters)
    return o


def _relabel(nodes, rs, frac, levels):
    """Mark a random subset of nodes as goal nodes with costs from `levels` distinct values."""
    for i in range(1, len(nodes)):
        nodes[i].goal = int(rs.random() < frac)
        nodes[i].costS = float(rs.integers(0, levels)) * 0.5 + 3.0
    return nodes


def _chain(nodes, leaf):
    out = [leaf]
    while nodes[out[0]].parent != -1:
        out.insert(0, nodes[out[0]].parent)
    return out


def test_oracle_no_goal_is_empty():
    o = _grown()
    raw = o.nodes_raw()
    for i in range(len(raw)):
        raw[i].goal = 0
    o.load_tree(raw)
    assert o.extract_best_path() == []


def test_oracle_unique_minimum():
    o = _grown()
    raw = _relabel(o.nodes_raw(), np.random.default_rng(1), 0.3, 1000)
    o.load_tree(raw)
    goal = [i for i in range(len(raw)) if raw[i].goal]
    best = min(goal, key=lambda i: (raw[i].costS, i))
    path = o.extract_best_path()
    assert path[0] == 0 and raw[path[-1]].goal and raw[path[-1]].costS == raw[best].costS
    assert path == _chain(raw, path[-1])


def test_oracle_small_ties_keep_tree_order():
    """Fewer than 17 goal nodes: std::sort is an insertion sort there, so equal costs keep tree order."""
    o = _grown()
    raw = o.nodes_raw()
    for i in range(len(raw)):
        raw[i].goal = 0
    picks = [40, 7, 90, 23]
    for i in picks:
        raw[i].goal, raw[i].costS = 1, 5.0
    o.load_tree(raw)
    assert o.extract_best_path() == _chain(raw, 7)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,seed,iters", [("obb200", 3, 300), ("moving", 4, 250), ("empty", 2, 300)])
def test_best_path_exact_tree(kind, seed, iters):
    from test_gpu_parity import _scene
    mode, obs = _scene(kind)
    o = Oracle(abi.default_params(collision_mode=mode), obs)
    Oracle.srand(seed)
    o.init_tree()
    o.expand(iters)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=mode), max_nodes=1 << 16, max_rows=1 << 20,
                       max_batch=256)
    if obs is not None:
        pl.set_obstacles(obs)
    pl.tree_init()
    pl.expand(clrrt.Rng(seed), n_iters=iters, mode=clrrt.CLRRT_MODE_EXACT, batch=256)
    path, cost, ng = pl.extract_best_path()
    ref = o.extract_best_path()
    on = o.nodes()
    print(f"{kind}: {int(on['goal'].sum())} goal nodes, path {path}")
    assert ng == int(on["goal"].sum())
    assert path == ref
    if ref:
        assert np.float32(cost) == on["costS"][ref[-1]]


@pytest.mark.gpu
@pytest.mark.parametrize("frac,levels", [(0.5, 3), (0.2, 1), (0.05, 7), (0.0, 1)])
def test_best_path_tied_costs(frac, levels):
    o = _grown(5, 400)
    raw = _relabel(o.nodes_raw(), np.random.default_rng(levels), frac, levels)
    o.load_tree(raw)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_STUB), max_nodes=1 << 16,
                       max_rows=1 << 20, max_batch=256)
    pl.tree_load(raw)
    path, cost, ng = pl.extract_best_path()
    assert ng == sum(raw[i].goal for i in range(len(raw)))
    assert path == o.extract_best_path()
    # a path cap shorter than the chain returns its root end and the full length
    if len(path) > 2:
        short, _, _ = pl.extract_best_path(cap=2)
        assert short == path[:2]


@pytest.mark.gpu
def test_best_path_large_batch_tree():
    """Full size: a BATCH tree of ~100k nodes; the GPU chain equals the oracle's on the same tree."""
    from test_gpu_parity import _scene
    mode, obs = _scene("obb200")
    pl = clrrt.Planner(clrrt.default_params(collision_mode=mode), max_nodes=1 << 20, max_rows=1 << 26,
                       max_batch=16384)
    pl.set_obstacles(obs)
    pl.tree_init()
    pl.expand(clrrt.Rng(9), n_iters=16384 * 8, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
    path, cost, ng = pl.extract_best_path()
    o = Oracle(abi.default_params(collision_mode=mode), obs)
    o.load_tree(pl.nodes_raw())
    print(f"{pl.size()[0]} nodes, {ng} goal nodes, best costS {cost}, path length {len(path)}")
    assert ng > 0 and path == o.extract_best_path()
