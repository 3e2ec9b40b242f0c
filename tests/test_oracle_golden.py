"""The CPU oracle against the reference's own outputs (tests/golden/survey_pins.json) and the
frozen oracle vectors.  CPU only."""
import json
import os

import numpy as np
import pytest

from clrrt import abi, scenes
from oracle_binding import Oracle, lib, obb_dist

HERE = os.path.dirname(os.path.abspath(__file__))
PINS = json.load(open(os.path.join(HERE, "golden", "survey_pins.json")))
VECS = json.load(open(os.path.join(HERE, "golden", "oracle_vectors.json")))


def test_obb_kat():
    for k in PINS["obb_kat"]:
        d = obb_dist(tuple(k["a"]), tuple(k["b"]))
        assert abs(d - k["dist"]) <= k["tol"], (d, k)


def test_empty_scene_seed1_pins():
    pin = PINS["empty_seed1_200"]
    o = Oracle(abi.default_params())
    Oracle.srand(pin["seed"])
    o.init_tree()
    o.expand(pin["iters"])
    n = o.nodes()
    assert o.size() == pin["tree"]
    assert int(n["goal"].sum()) == pin["goal_nodes"]
    assert o.counters()["sim_count"] == pin["sim_count"]
    n1 = pin["node1"]
    assert n["parent"][1] == n1["parent"]
    st = n["state"][1]
    for key, idx in (("x", 0), ("y", 1), ("theta", 2), ("v", 4), ("t", 6)):
        assert abs(st[idx] - n1[key]) < 5e-7, key
    assert abs(float(n["costE"][1]) - n1["costE"]) < 5e-5
    assert abs(float(n["costS"][1]) - n1["costS"]) < 5e-4
    assert n["nrows"][1] == n1["rows"]


def test_obstacle_scene_seed3_pins():
    pin = PINS["lcg200_seed3_300"]
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), scenes.urban_scene(pin["obstacles"]))
    Oracle.srand(pin["seed"])
    o.init_tree()
    o.expand(pin["iters"])
    c = o.counters()
    assert o.size() == pin["tree"]
    assert int(o.nodes()["goal"].sum()) == pin["goal_nodes"]
    for k in ("sim_count", "fail_collision", "fail_acclimit"):
        assert c[k] == pin[k], k


def test_rand_streams():
    for seed, vals in VECS["rand"].items():
        lib().orc_srand(int(seed))
        assert [lib().orc_rand() for _ in range(len(vals))] == vals


def test_oracle_vectors_stable():
    trees = {}
    for v in VECS["oracle_vectors"]:
        mode = v["collision_mode"]
        if mode not in trees:
            obs = scenes.urban_scene(200) if mode == abi.CLRRT_COLLISION_OBB else None
            o = Oracle(abi.default_params(collision_mode=mode), obs)
            Oracle.srand(v["tree_seed"])
            o.init_tree()
            o.expand(v["tree_iters"])
            trees[mode] = o
        o = trees[mode]
        if "parent" in v:
            r = o.simulate(v["parent"], 0, *v["sample"])
            assert r["outcome"] == v["outcome"] and r["nrows"] == v["nrows"]
            assert r["costE"] == v["costE"] and r["costS"] == v["costS"]
            assert list(r["final"]) == v["final"]
        else:
            ids, keys = o.sort_nodes(*v["sort_sample"], v["explore"])
            assert ids == v["ids"]
            assert np.allclose(keys, v["keys"], rtol=0, atol=0)


def test_batch_mode_b1_equals_sequential():
    """BATCH mode with one sample per round is the reference's sequential loop."""
    p = abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB)
    obs = scenes.urban_scene(50)
    a, b = Oracle(p, obs), Oracle(p, obs)
    Oracle.srand(5); a.init_tree(); a.expand(60)
    Oracle.srand(5); b.init_tree(); b.expand_batch(60, 1, stable=False)
    na, nb = a.nodes(), b.nodes()
    assert a.size() == b.size()
    assert np.array_equal(na["state"], nb["state"]) and np.array_equal(na["parent"], nb["parent"])


def test_scene_generator_shape():
    s = scenes.urban_scene(200, 20)
    assert s.shape == (220, 7)
    assert np.all(np.abs(s[:200, 1]) >= 3.0)
    assert np.all(s[:200, 5:] == 0) and np.any(s[200:, 5:] != 0)


@pytest.mark.parametrize("T", [0, 24])
def test_threaded_batch_defer_equals_sequential(T):
    """orc_expand_batch_defer_mt (each round's samples on host threads, keys without the by-value Node copy) grows
    the tree of the sequential orc_expand_batch_defer, bit for bit -- it is the checker the full-size deferred-sample
    tests (tests/test_full_size_parity.py) run at the benchmarked batch sizes."""
    obs = scenes.urban_scene(200)
    trees = []
    for threads in (0, 8):
        o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
        Oracle.srand(7)
        o.init_tree()
        nd = o.expand_batch(6 * 128, 128, stable=True, defer_steps=T, threads=threads)
        assert (nd > 0) == (T > 0)
        trees.append((bytes(o.nodes_raw()), o.counters(), nd,
                      b"".join(o.rows(i).tobytes() for i in range(1, o.size(), 5))))
    assert trees[0] == trees[1]
    assert len(trees[0][0]) > 160 * 100
