#!/usr/bin/env python3
"""Writes tests/golden/ref_tree.npz + ref_tree_meta.json: tree-level cases with the outputs of the
REFERENCE'S OWN CODE (oracle/_ref, `make -C oracle ref`; tests/ref_tree.py lists the functions).

Every record is checked against the oracle (bit for bit) before it is written; a difference stops the
script.  Trajectories are stored as per-rollout / per-node SHA-1 digests of their float64 bits (and in
full for a few), headers in full.  Run in the development container (needs /root/reference):
    python3 tests/golden/make_ref_tree.py
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import ref_tree as T  # noqa: E402
import ref_units as RU  # noqa: E402
from oracle_binding import Oracle, lib as olib  # noqa: E402

SEED = 20261017
SORT_SIZES = {"a": (3000, 400, 512), "b": (9000, 1500, 256)}  # nodes, root copies, samples
SIM_SETS = {tag: (c, o) for tag, (c, o, _) in T.SIM_CASES.items()}
N_PARENTS, N_JOBS, FULL_ROWS = 48, 480, 8
SORT_COLS = [0, 1, 2, 4, 6, 11, 16, 17, 18, 19, 20]  # header columns the candidate lists read (+ v, t)


def fail(msg):
    sys.exit("oracle differs from the reference: " + msg)


def eq_bits(a, b):
    return len(RU.mismatches(np.atleast_2d(a), np.atleast_2d(b))) == 0


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    L = T.ref_lib()
    O = olib()
    rng = np.random.default_rng(SEED)
    out, meta = {}, {"reference": "vdBerg93/cl-rrt at /root/reference (line ranges in oracle/Makefile)",
                     "flags": "-std=c++11 -O3 -DNDEBUG -ffp-contract=off (CMake Release)", "checks": {}}

    # a2/a3: sampleAroundVehicle + heuristic draw vs the oracle's glibc rand() stream
    S = np.zeros((len(T.SAMPLE_GOALS), len(T.SAMPLE_SEEDS), 2000, 3))
    for gi, g in enumerate(T.SAMPLE_GOALS):
        for si, s in enumerate(T.SAMPLE_SEEDS):
            S[gi, si] = T.ref_samples(L, g, s, 2000)
            o = Oracle(T.params(0, g))
            Oracle.srand(s)
            xy = np.zeros((2000, 2)); ex = np.zeros(2000, np.int32)
            import ctypes as C
            O.orc_draw_samples(o.h, 2000, T.dp(xy), ex.ctypes.data_as(C.POINTER(C.c_int)))
            if not eq_bits(xy, S[gi, si, :, :2]) or not np.array_equal(ex, (S[gi, si, :, 2] <= 0.7).astype(np.int32)):
                fail(f"samples goal {g} seed {s}")
    out["sample_out"] = S
    out["sample_goals"] = np.array(T.SAMPLE_GOALS)
    out["sample_seeds"] = np.array(T.SAMPLE_SEEDS)

    # a14: updateLookahead / updateReferenceResolution
    v = np.concatenate([rng.uniform(-12, 12, 600), [0.0, 10.0, -10.0, 9.999999999, 10.000000001, 3.0, 20.0]])
    la = np.zeros((len(v), 2))
    L.ref_lookahead_res(len(v), T.dp(v), T.dp(la))
    out["lookahead_v"] = v
    out["lookahead_out"] = la

    # a4: candidate lists over synthetic trees (std::sort tie order over copies of the root)
    for tag, (n, k, ns) in SORT_SIZES.items():
        H = T.sort_tree(rng, n, k)
        Ssm = T.sort_samples(rng, H, ns)
        ids, cnt = T.ref_sort(L, H, Ssm)
        o = Oracle(T.params(0))
        o.L.orc_load_tree(o.h, T.node_array(H), len(H))
        import ctypes as C
        for j in range(ns):
            oi = np.zeros(10, np.int32); ok = np.zeros(10, np.float32)
            m = O.orc_sort_nodes(o.h, Ssm[j, 0], Ssm[j, 1], int(Ssm[j, 2]), 0, oi.ctypes.data_as(C.POINTER(C.c_int)),
                                 ok.ctypes.data_as(C.POINTER(C.c_float)))
            if m != cnt[j] or not np.array_equal(oi[:m], ids[j, :m]):
                fail(f"sort {tag} sample {j}: {oi[:m]} vs {ids[j, :cnt[j]]}")
        out[f"sort_{tag}_tree"] = H[:, SORT_COLS]
        out[f"sort_{tag}_samples"] = Ssm
        out[f"sort_{tag}_ids"] = ids
        out[f"sort_{tag}_n"] = cnt
        meta["checks"][f"sort_{tag}"] = {"nodes": n, "root_copies": k, "samples": ns,
                                         "mean_list": float(cnt.mean())}

    # a5-a12: Simulation from parents toward samples / the goal
    for tag, (coll, (ns_, nm_)) in SIM_SETS.items():
        Hp = T.sim_parents(rng, N_PARENTS)
        J = T.sim_jobs(rng, Hp, N_JOBS)
        obs = T.scene(ns_, nm_)
        p = T.sim_params(tag)
        T.ref_configure(L, p, obs)
        rmeta, rrows = T.ref_simulate(L, Hp, J)
        o = Oracle(p, obs if len(obs) else None)
        o.L.orc_load_tree(o.h, T.node_array(Hp), len(Hp))
        ometa, orows = T.oracle_simulate(o, J)
        if not eq_bits(ometa[:, T.SIM_META_COLS], rmeta[:, T.SIM_META_COLS]):
            bad = RU.mismatches(ometa[:, T.SIM_META_COLS], rmeta[:, T.SIM_META_COLS])
            fail(f"simulate {tag} meta jobs {bad[:5]}: {ometa[bad[0]]} vs {rmeta[bad[0]]}")
        dg = T.digests(rrows)
        if not np.array_equal(T.digests(orows), dg):
            fail(f"simulate {tag} rows")
        out[f"sim_{tag}_parents"] = Hp
        out[f"sim_{tag}_jobs"] = J
        out[f"sim_{tag}_meta"] = rmeta
        out[f"sim_{tag}_digest"] = dg
        full = np.zeros((FULL_ROWS, 520, 10))
        for k in range(FULL_ROWS):
            full[k, :len(rrows[k])] = rrows[k]
        out[f"sim_{tag}_rows"] = full
        meta["checks"][f"sim_{tag}"] = {"jobs": N_JOBS, "outcomes": np.bincount(rmeta[:, 0].astype(int), minlength=5).tolist(),
                                        "steps": int(rmeta[:, 8].sum())}

    # a1: expandTree (sequential, EXACT) trees
    for case in T.EXPAND_CASES:
        name, coll, (ns_, nm_), seed, iters, goal = case
        H, rows, cnt = T.ref_expand(L, case)
        o = Oracle(T.params(coll, goal), T.scene(ns_, nm_) if ns_ + nm_ else None)
        Oracle.srand(seed)
        o.init_tree()
        o.expand(iters)
        Ho = T.headers_from_numpy(o.nodes())
        if len(Ho) != len(H) or not eq_bits(Ho[:, T.HDR_COLS], H[:, T.HDR_COLS]):
            fail(f"expand {name} headers ({len(Ho)} vs {len(H)} nodes)")
        if not np.array_equal(T.digests([o.rows(i) for i in range(len(H))]), T.digests(rows)):
            fail(f"expand {name} rows")
        out[f"expand_{name}_hdr"] = H
        out[f"expand_{name}_digest"] = T.digests(rows)
        out[f"expand_{name}_counters"] = cnt
        meta["checks"][f"expand_{name}"] = {"nodes": len(H), "goal_nodes": int(H[:, 13].sum()),
                                            "sim_count": int(cnt[0]), "fail_collision": int(cnt[1])}

    # f1/f2: planMotion queries (stub collision: the unity build's checkObsDistance), commit_path = 1
    from clrrt import replan
    make = replan.default_make_params(0)
    L.ref_best_clear()
    rb = T.ReferenceBackend(L, make)
    o = Oracle(T.params(0), None)

    class OB:
        def begin_query(self, pose, goal_car, obs_car):
            o.set_params(make(pose[4], goal_car)); o.set_obstacles(obs_car)
            o.path_transform(False, pose)
            return o.initialize_tree([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])

        def end_query(self, pose):
            ids = o.extract_best_path(); o.path_commit(ids); o.path_transform(True, pose)
            nodes = o.path_nodes()
            rows = [o.path_rows(i) for i in range(len(nodes))]
            return ids, (np.concatenate(rows) if rows else np.zeros((0, 10)))

    ob = OB()
    # the reference's sequence first, then the oracle's (both draw from the one glibc rand() state)
    L.ref_srand(T.REPLAN_SEED)
    pose = np.array([0.0, 0.0, 0.0, 0.0, 1.0, 0.0])
    poses = []
    for q in range(T.REPLAN_QUERIES):
        gc = replan.goal_in_car_frame(T.REPLAN_GOAL, pose)
        rb.begin_query(pose, gc, np.zeros((0, 7)))
        Hi, ri = T.ref_tree(L)
        out[f"replan_q{q}_init_hdr"] = Hi
        out[f"replan_q{q}_init_digest"] = T.digests(ri)
        L.ref_tree_expand(T.REPLAN_ITERS)
        He, re_ = T.ref_tree(L)
        out[f"replan_q{q}_tree_hdr"] = He
        out[f"replan_q{q}_tree_digest"] = T.digests(re_)
        Hb, rows_b = rb.end_query(pose)
        out[f"replan_q{q}_best_hdr"] = Hb
        out[f"replan_q{q}_best_rows_digest"] = T.digest(rows_b)
        poses.append(pose.copy())
        pose = replan.advance_pose(pose, rows_b)
    Oracle.srand(T.REPLAN_SEED)
    outcomes = []
    for q in range(T.REPLAN_QUERIES):
        pose = poses[q]
        gc = replan.goal_in_car_frame(T.REPLAN_GOAL, pose)
        outcomes.append(ob.begin_query(pose, gc, np.zeros((0, 7))))
        On = T.headers_from_numpy(o.nodes())
        if len(On) != len(out[f"replan_q{q}_init_hdr"]) or not eq_bits(On[:, T.HDR_COLS], out[f"replan_q{q}_init_hdr"][:, T.HDR_COLS]):
            fail(f"replan q{q} re-initialised tree")
        o.expand(T.REPLAN_ITERS)
        On = T.headers_from_numpy(o.nodes())
        if len(On) != len(out[f"replan_q{q}_tree_hdr"]) or not eq_bits(On[:, T.HDR_COLS], out[f"replan_q{q}_tree_hdr"][:, T.HDR_COLS]):
            fail(f"replan q{q} expanded tree ({len(On)} vs {len(out[f'replan_q{q}_tree_hdr'])} nodes)")
        if not np.array_equal(T.digests([o.rows(i) for i in range(len(On))]), out[f"replan_q{q}_tree_digest"]):
            fail(f"replan q{q} expanded tree rows")
        ids, rows_o = ob.end_query(pose)
        if len(ids) != len(out[f"replan_q{q}_best_hdr"]) or not np.array_equal(T.digest(rows_o), out[f"replan_q{q}_best_rows_digest"]):
            fail(f"replan q{q} best path")
    out["replan_poses"] = np.array(poses)
    out["replan_outcomes"] = np.array(outcomes)
    meta["checks"]["replan"] = {"outcomes": [int(v) for v in outcomes],
                                "best_path_lengths": [int(out[f"replan_q{q}_best_hdr"].shape[0]) for q in range(T.REPLAN_QUERIES)]}

    np.savez_compressed(T.FIXTURE, **out)
    with open(os.path.join(HERE, "ref_tree_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta["checks"], indent=1))
    print("wrote", T.FIXTURE, os.path.getsize(T.FIXTURE), "bytes")


if __name__ == "__main__":
    main()
