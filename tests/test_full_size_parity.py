"""Parity at the benchmarked sizes (BASELINE.json configs[1], configs[2], configs[4]) — GPU.

* cfg3 (200 static obstacles, B = 16384 samples per round): BATCH rounds through the multi-GPU round API
  (clrrt_round_eval / clrrt_round_commit, the path bench.py times).  On rounds 1, 3, 6 and 12, 512 (128)
  samples drawn at random from the round's 16384 are evaluated by the oracle against the same frozen
  tree (eval_iteration = one expandTree iteration, rrtplanner.cpp:123-174, BATCH tie order) and the
  records the GPU produced for them INSIDE the full batch must be identical: count, parent, nrows, goal
  flag, state bits and float cost bits; for 48 of them the committed trajectory rows too.
* cfg2 (50 static obstacles, B = 4096): two BATCH rounds, whole tree against the oracle's expand_batch,
  bit for bit (states, costs, rows).
* cfg3 at the tree sizes the bench reaches (test_cfg3_bench_size_tree): one query grown past 2.2 M nodes
  in pipelined BATCH rounds (clrrt_expand, the single-GPU bench path), where the large-tree search settings
  engage (walk search, narrowed rollout grid, the N/512 exact-key budget).  On the next round (a) the
  candidate lists of all 16384 samples from the default search equal brute force's, ids and key bits, and
  (b) 128 samples' records inside the full round equal the oracle's eval_iteration on the frozen tree.
The 20-mover config-5 scene runs in tests/test_replan.py (test_replanning_queries_parity[moving20],
test_moving20_batch_reinit_from_found_path).
"""
import numpy as np
import pytest

import clrrt
from clrrt import abi, scenes
from oracle_binding import Oracle

pytestmark = pytest.mark.gpu

REC = 160


def _records(raw, n):
    if n == 0:
        return None
    return clrrt.nodes_to_numpy((abi.Node * n).from_buffer_copy(raw[:n * REC]))


def _per_sample(rec, samples, picks):
    """Map the compacted round records back to their samples: a regular record's reference ends at its
    sample (the accumulated linspace's last point, within 1e-6 m); a goal-biased record (parent =
    CLRRT_PARENT_PREV) follows its regular record."""
    out = {j: [] for j in picks}
    if rec is None:
        return out
    sx = np.array([samples[j].x for j in picks])
    sy = np.array([samples[j].y for j in picks])
    for i in range(len(rec["parent"])):
        if rec["parent"][i] == abi.CLRRT_PARENT_PREV:
            continue
        d = np.hypot(sx - rec["ref_back"][i, 0], sy - rec["ref_back"][i, 1])
        k = int(np.argmin(d))
        if d[k] < 1e-6:
            out[picks[k]].append(i)
            if i + 1 < len(rec["parent"]) and rec["parent"][i + 1] == abi.CLRRT_PARENT_PREV:
                out[picks[k]].append(i + 1)
    return out


def _same_node(g, i, r):
    """GPU record i (numpy view) vs oracle node r (abi.Node): exact."""
    st = np.array(list(r.state), dtype=np.float64)
    return (int(g["parent"][i]) == r.parent and int(g["nrows"][i]) == r.nrows and int(g["goal"][i]) == r.goal
            and np.array_equal(g["state"][i].view(np.uint64), st.view(np.uint64))
            and float(g["costE"][i]) == r.costE and float(g["costS"][i]) == r.costS)


def test_cfg3_full_batch_rounds_match_oracle():
    import torch
    B = 16384
    obs = scenes.urban_scene(200)
    params = abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                       max_rows=1 << 26, max_batch=B)
    pl.set_obstacles(obs)
    pl.tree_init()
    o = Oracle(params, obs)
    out = torch.empty((2 * B, REC), dtype=torch.uint8, device="cuda")
    rng = clrrt.Rng(31)
    pick_rng = np.random.default_rng(5)
    checked = {"samples": 0, "nodes": 0, "rows": 0}
    check_rounds = {1: 512, 3: 512, 6: 512, 12: 128}
    for rnd in range(1, max(check_rounds) + 1):
        smp = rng.draw_samples(pl.params, B)
        n_before = pl.size()[0]
        n = pl.round_eval(smp, out.data_ptr())
        raw = out[:n].cpu().numpy().tobytes()
        rec = _records(raw, n)
        picks = sorted(pick_rng.choice(B, check_rounds.get(rnd, 0), replace=False).tolist())
        if picks:
            o.load_tree(pl.nodes_raw())
            mine = _per_sample(rec, smp, picks)
            bad = []
            for j in picks:
                want = o.eval_iteration(smp[j].x, smp[j].y, smp[j].explore, stable=True)
                got = mine[j]
                ok = len(got) == len(want) and all(_same_node(rec, i, r) for i, r in zip(got, want))
                checked["samples"] += 1
                checked["nodes"] += len(want)
                if not ok:
                    bad.append((j, len(want), len(got)))
            assert not bad, f"round {rnd} ({n_before} nodes): {len(bad)} of {len(picks)} samples differ {bad[:5]}"
        pl.round_commit(out.data_ptr(), n, 0, n)
        if picks:
            # committed trajectories (Node::tra) of 48 accepted regular nodes vs the oracle's Simulation
            g = pl.nodes()
            for j in picks[:48]:
                for i in mine[j][:1]:
                    par = int(rec["parent"][i])
                    want = o.simulate(par, 0, smp[j].x, smp[j].y, rows=True, rows_cap=600)
                    t = n_before + i
                    rows = pl.rows(int(g["row_offset"][t]), int(g["nrows"][t]))
                    assert np.array_equal(rows.view(np.uint64), want["rows"].view(np.uint64)), (rnd, j)
                    checked["rows"] += 1
    print(f"cfg3 full-batch rounds: {pl.size()[0]} nodes; oracle-checked {checked}")
    assert checked["nodes"] > 500 and checked["rows"] > 50
    pl.close()


def test_cfg3_bench_size_tree():
    import torch
    B = 16384
    target = 4096 * 512 + 100_000  # nn_walk_budget_keys' N/512 term exceeds its 4096 floor from 2.1 M nodes
    max_nodes = 5 << 19
    obs = scenes.urban_scene(200)
    params = clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB)
    pl = clrrt.Planner(params, max_nodes=max_nodes, max_rows=max_nodes * 64, max_batch=B)
    try:
        pl.set_obstacles(obs)
        pl.tree_init()
        rng = clrrt.Rng(41)
        while pl.size()[0] < target:
            st = pl.expand(rng, n_iters=64 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
            assert not st["capacity_stop"]
        n_tree = pl.size()[0]
        smp = rng.draw_samples(pl.params, B)
        # (a) the default large-tree search against brute force (node-index tie order in both)
        ids_w, keys_w = pl.sort_nodes_batch(smp, exact=False)
        pl.set_option("nn_walk_min", 1 << 40)
        ids_b, keys_b = pl.sort_nodes_batch(smp, exact=False)
        pl.set_option("nn_walk_min", 8192)
        bad = np.nonzero((ids_w != ids_b).any(axis=1) | (keys_w.view(np.uint32) != keys_b.view(np.uint32)).any(axis=1))[0]
        assert bad.size == 0, f"{n_tree} nodes: {bad.size} of {B} lists differ, e.g. {bad[:5]}"
        assert (ids_b[:, 0] >= 0).sum() > B // 2
        # (b) the round's records of 128 samples against the oracle
        out = torch.empty((2 * B, REC), dtype=torch.uint8, device="cuda")
        n = pl.round_eval(smp, out.data_ptr())
        rec = _records(out[:n].cpu().numpy().tobytes(), n)
        picks = sorted(np.random.default_rng(9).choice(B, 128, replace=False).tolist())
        o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
        o.load_tree(pl.nodes_raw())
        want = o.eval_iterations([smp[j].x for j in picks], [smp[j].y for j in picks],
                                 [smp[j].explore for j in picks], stable=True, threads=16)
        mine = _per_sample(rec, smp, picks)
        nodes, bad = 0, []
        for j, w in zip(picks, want):
            got = mine[j]
            nodes += len(w)
            if not (len(got) == len(w) and all(_same_node(rec, i, r) for i, r in zip(got, w))):
                bad.append((j, len(w), len(got)))
        print(f"cfg3 bench-size tree: {n_tree} nodes, {B} lists = brute force, 128 samples ({nodes} nodes) = oracle")
        assert not bad, f"{n_tree} nodes: {len(bad)} of 128 samples differ {bad[:5]}"
        assert nodes > 20
    finally:
        pl.close()


def test_cfg2_batch_tree_parity():
    B, rounds = 4096, 2
    obs = scenes.urban_scene(50)
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
    Oracle.srand(21)
    o.init_tree()
    o.expand_batch(B * rounds, B, stable=True)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 16,
                       max_rows=1 << 24, max_batch=B)
    pl.set_obstacles(obs)
    pl.tree_init()
    st = pl.expand(clrrt.Rng(21), n_iters=B * rounds, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
    assert st["rounds"] == rounds
    on, gn = o.nodes(), pl.nodes()
    print(f"cfg2 BATCH: oracle {len(on['parent'])} nodes, gpu {len(gn['parent'])}")
    assert len(on["parent"]) == len(gn["parent"]) > 500
    assert np.array_equal(on["parent"], gn["parent"]) and np.array_equal(on["goal"], gn["goal"])
    assert np.array_equal(gn["state"].view(np.uint64), on["state"].view(np.uint64))
    assert np.array_equal(gn["costE"].view(np.uint32), on["costE"].view(np.uint32))
    assert np.array_equal(gn["costS"].view(np.uint32), on["costS"].view(np.uint32))
    for i in range(1, len(on["parent"]), 7):
        rows = pl.rows(int(gn["row_offset"][i]), int(gn["nrows"][i]))
        assert np.array_equal(rows.view(np.uint64), np.ascontiguousarray(o.rows(i)).view(np.uint64)), i
    oc, gc = o.counters(), pl.counters()
    assert oc["rollouts"] > 0 and gc["rollouts"] > 0
    pl.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config", ["cfg3", "cfg2"])
def test_bench_settings_deferred_tree_matches_oracle(config):
    """The exact settings bench.py measures, whole tree against the oracle (verdict r04 item 1): BATCH rounds at
    the benchmarked batch with deferred samples (cfg3: 200 obstacles, B = 16384, defer_steps 128, the lag-2
    pipeline a 2 s query runs, 8 rounds; cfg2: 50 obstacles, B = 4096, defer_steps 64, lag 1 as a 200 ms query
    runs, 6 rounds) grow node for node, bit for bit (states, float costs, goal flags, parents, every trajectory row,
    the reference's counters) the tree of orc_expand_batch_defer's rule (each sample evaluated against its own
    round's frozen tree -- expandTree rrtplanner.cpp:123-174 -- and committed ceil(chain / T) - 1 rounds late,
    oldest round first), evaluated here on 16 host threads."""
    B, T, M, rounds, lag = {"cfg3": (16384, 128, 200, 8, 2), "cfg2": (4096, 64, 50, 6, 1)}[config]
    obs = scenes.urban_scene(M)
    seed = 31
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
    Oracle.srand(seed)
    o.init_tree()
    ndef = o.expand_batch(B * rounds, B, stable=True, defer_steps=T, threads=16)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                       max_rows=1 << 26, max_batch=B)
    try:
        pl.set_option("defer_steps", T)
        pl.set_option("nn_lag", lag)
        pl.set_obstacles(obs)
        pl.tree_init()
        st = pl.expand(clrrt.Rng(seed), n_iters=B * rounds, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        assert st["rounds"] == rounds and st["iterations"] == B * rounds, st
        on, gn = o.nodes(), pl.nodes()
        print(f"{config} bench settings: oracle {len(on['parent'])} nodes ({ndef} samples deferred), "
              f"gpu {len(gn['parent'])} nodes ({st['deferred']} deferred)")
        assert len(on["parent"]) == len(gn["parent"]) > rounds * B // 4
        bad = np.nonzero((on["parent"] != gn["parent"]) | (on["goal"] != gn["goal"]) | (on["nrows"] != gn["nrows"])
                         | (gn["state"].view(np.uint64) != on["state"].view(np.uint64)).any(axis=1)
                         | (gn["costE"].view(np.uint32) != on["costE"].view(np.uint32))
                         | (gn["costS"].view(np.uint32) != on["costS"].view(np.uint32)))[0]
        assert bad.size == 0, f"{bad.size} nodes differ, first {bad[:5]}"
        assert st["deferred"] == ndef > 0
        oc, gc = o.counters(), pl.counters()
        for k in ("sim_count", "fail_collision", "fail_acclimit", "fail_iterlimit", "rollouts"):
            assert oc[k] == gc[k], (k, oc[k], gc[k])
        nr = pl.size()[1]
        arena = pl.rows(0, nr)
        for i in range(1, len(on["parent"])):
            off, cnt = int(gn["row_offset"][i]), int(gn["nrows"][i])
            assert np.array_equal(arena[off:off + cnt].view(np.uint64), np.ascontiguousarray(o.rows(i)).view(np.uint64)), i
        assert pl.debug_counters()[61] == 0
    finally:
        pl.close()


@pytest.mark.timeout(900)
def test_late_query_deferred_rounds_match_oracle():
    """Deferral at the late-query tree sizes (verdict r05 item 4): a cfg3 tree grown past 2.2 M nodes with the bench's
    settings (B = 16384, defer_steps 128, the lag-2 pipeline) -- where the stateless half-precision walk format and the
    N/512 exact-key budget are live -- then 4 more deferring rounds from it.  For rounds 1-3 of those, 512 random
    samples each are evaluated by the oracle against their ORIGIN round's frozen tree (eval_iteration = expandTree,
    rrtplanner.cpp:123-174, BATCH tie order; the tree size before the round from clrrt_round_sizes): the records the
    GPU appended for each sample are identical (count, parent, nrows, goal flag, state and float cost bits) and were
    appended by the commit of round r + ceil(chain / T) - 1 (the deferred-sample rule, chain = the oracle's deciding
    rollout chain; the drain's commit when that is past the last round), and by no other commit."""
    B, T, lag, rounds, seed, per = 16384, 128, 2, 4, 43, 512
    target = 4096 * 512 + 100_000
    max_nodes = 5 << 19
    obs = scenes.urban_scene(200)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=max_nodes,
                       max_rows=max_nodes * 64, max_batch=B)
    try:
        pl.set_option("defer_steps", T)
        pl.set_option("nn_lag", lag)
        pl.set_obstacles(obs)
        pl.tree_init()
        rng = clrrt.Rng(seed)
        while pl.size()[0] < target:
            st = pl.expand(rng, n_iters=64 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
            assert not st["capacity_stop"]
        n0 = pl.size()[0]
        rng_at = clrrt.Rng()
        rng_at.state = abi.Rng.from_buffer_copy(bytes(rng.state))
        st = pl.expand(rng, n_iters=rounds * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        assert st["rounds"] == rounds and st["deferred"] > 0, st
        sizes = [n0] + [int(x) for x in pl.round_sizes()]  # sizes[c + 1]: after commit c (c = rounds: the drain)
        assert len(sizes) in (rounds + 1, rounds + 2), sizes
        smp = rng_at.draw_samples(pl.params, rounds * B)
        raw = pl.nodes_raw()
        g = clrrt.nodes_to_numpy(pl.nodes_raw(n0))
        o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
        o.load_tree(raw)
        del raw
        # appended: a goal-biased node's parent is the regular node just before it (k_append resolved it)
        idx = np.arange(len(g["parent"]), dtype=np.int64) + n0
        is_gb = np.zeros(len(g["parent"]), dtype=bool)
        is_gb[1:] = g["parent"][1:] == idx[:-1]
        gb_next = np.zeros(len(g["parent"]), dtype=bool)
        gb_next[:-1] = is_gb[1:]
        pick_rng = np.random.default_rng(11)
        checked = {"samples": 0, "nodes": 0, "deferred": 0}
        for r in range(1, rounds):
            picks = sorted(pick_rng.choice(B, per, replace=False).tolist())
            ss = [smp[r * B + j] for j in picks]
            want, chains = o.eval_iterations_upto([s.x for s in ss], [s.y for s in ss], [s.explore for s in ss],
                                                  sizes[r], stable=True, threads=16)
            bad = []
            for j, s, w, ch in zip(picks, ss, want, chains):
                D = (int(ch) + T - 1) // T - 1 if ch > 0 else 0
                c = min(r + D, len(sizes) - 2)  # the commit due (the drain's when past the last round)
                # the sample's regular record: its reference ends at the sample; the goal-biased one follows it
                hit = np.nonzero((np.abs(g["ref_back"][:, 0] - s.x) < 1e-6) & (np.abs(g["ref_back"][:, 1] - s.y) < 1e-6)
                                 & ~is_gb)[0]
                got = [int(i) for i in hit]
                got += [i + 1 for i in got if gb_next[i]]
                got.sort()
                lo, hi = sizes[c] - n0, sizes[c + 1] - n0
                ok = len(got) == len(w) and all(lo <= i < hi for i in got)
                for q, (i, rr) in enumerate(zip(got, w) if ok else ()):
                    if q == 1:  # the goal-biased record: the oracle leaves its parent unresolved (-2)
                        ok = ok and rr.parent == abi.CLRRT_PARENT_PREV and int(g["parent"][i]) == n0 + got[0]
                        rr.parent = int(g["parent"][i])
                    ok = ok and _same_node(g, i, rr)
                checked["samples"] += 1
                checked["nodes"] += len(w)
                checked["deferred"] += D > 0
                if not ok:
                    bad.append((r, j, D, len(w), got[:2], (lo, hi)))
            assert not bad, f"round {r}: {len(bad)} of {per} samples differ {bad[:4]}"
        print(f"late-query deferred rounds from {n0} nodes (commits {sizes[1:]}): oracle-checked {checked}")
        assert checked["nodes"] > 200 and checked["deferred"] > 0
    finally:
        pl.close()
