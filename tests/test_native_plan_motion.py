"""MotionPlanner::planMotion (rrt/src/motionplanner.cpp:8-77) through the C++
adapter's ROS-free MotionPlanner (include/clrrt_adapter.hpp), linked against libclrrt with no Python in
the loop (tests/native/plan_motion.cpp), against the CPU oracle running the same 5 Hz query sequence:
re-init outcome, tree size, committed path ids, the filtered MPC message (filterMPCmessage :130-151)
bit for bit, the fail counters of each query (:9, :45) and, with draw_tree on (rrtplanner.cpp:322-341),
every node's goal flag and trajectory (the rviz marker data) hash-equal to the oracle's tree."""
import os
import struct
import subprocess

import numpy as np
import pytest

from clrrt import abi, replan, scenes
from oracle_binding import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "plan_motion")
GOAL_W = (40.0, 0.0, 0.0, 0.0)


def _fnv1a(b):
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def test_plan_motion_program_compiles():
    """CPU: the adapter's MotionPlanner and the program compile (host C++ only)."""
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "plan_motion.cpp")], check=True)


def _oracle_sequence(mode, obs_world, seed, iters, nq):
    """The query sequence on the oracle (OracleBackend order of tests/test_replan.py); returns the
    per-query inputs and expected outputs."""
    make = replan.default_make_params(mode)
    o = Oracle(abi.default_params(collision_mode=mode), None)
    Oracle.srand(seed)
    pose = np.array([0.0, 0.0, 0.0, 0.0, 1.0, 0.0])
    inputs, want = [], []
    for q in range(nq):
        goal_c = replan.goal_in_car_frame(GOAL_W, pose)
        obs_c = replan.obstacles_in_car_frame(obs_world, q * replan.QUERY_PERIOD, pose)
        inputs.append((pose.copy(), goal_c, obs_c))
        o.reset_counters()
        o.set_params(make(pose[4], goal_c))
        o.set_obstacles(obs_c)
        o.path_transform(False, pose)
        oc = o.initialize_tree([0.0, 0.0, 0.0, pose[3], pose[4], pose[5]])
        o.expand(iters)
        n = o.size()
        nodes = o.nodes()
        markers = [(int(nodes["goal"][i]), _fnv1a(np.ascontiguousarray(o.rows(i)).tobytes())) for i in range(n)]
        ids = o.extract_best_path()
        o.path_commit(ids)
        o.path_transform(True, pose)
        msg = o.path_mpc_message(True)
        c = o.counters()
        want.append(dict(outcome=oc, tree=n, ids=list(ids), msg=msg, markers=markers,
                         counters=[c["sim_count"], c["fail_collision"], c["fail_acclimit"], c["fail_iterlimit"]]))
        rows = np.concatenate([o.path_rows(i) for i in range(len(ids))]) if ids else np.zeros((0, 10))
        pose = replan.advance_pose(pose, rows)
    return inputs, want


def _write_inputs(path, mode, inputs):
    with open(path, "wb") as f:
        f.write(b"CLPM" + struct.pack("<ii", mode, len(inputs)))
        for pose, goal_c, obs_c in inputs:
            f.write(np.asarray(pose, dtype="<f8").tobytes() + np.asarray(goal_c, dtype="<f8").tobytes())
            f.write(struct.pack("<i", len(obs_c)) + np.ascontiguousarray(obs_c, dtype="<f8").tobytes())


def _read_outputs(path):
    b = open(path, "rb").read()
    assert b[:4] == b"CLPO"
    off = 4
    def take(fmt):
        nonlocal off
        v = struct.unpack_from("<" + fmt, b, off)
        off += struct.calcsize("<" + fmt)
        return v if len(v) > 1 else v[0]
    out = []
    for _ in range(take("i")):
        r = dict(found=take("i"), outcome=take("i"), iterations=take("q"), tree=take("q"))
        n = take("i")
        r["ids"] = list(take(f"{n}i")) if n > 1 else ([take("i")] if n == 1 else [])
        r["published"] = take("i")
        m = take("i")
        r["msg"] = np.frombuffer(b, dtype="<f8", count=7 * m, offset=off).reshape(m, 7)
        off += 56 * m
        r["counters"] = [take("q") for _ in range(4)]
        k = take("i")
        r["markers"] = [(take("i"), take("Q")) for _ in range(k)]
        out.append(r)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["obb", "moving19", "moving20"])
def test_native_plan_motion_matches_oracle(kind, tmp_path):
    assert os.path.exists(EXE), "tests/native/plan_motion not built (make -C cl-rrt_amd/csrc)"
    mode = abi.CLRRT_COLLISION_OBB
    # obb: KEPT re-inits; moving19 (moving obstacle 208 removed, as in tests/test_replan.py): KEPT and
    # COLLISION re-inits; moving20: obstacle 208 blocks the lane, no query finds a path (:56-58)
    obs = {"obb": scenes.urban_scene(200), "moving19": np.delete(scenes.urban_scene(200, 20), 208, axis=0),
           "moving20": scenes.urban_scene(200, 20)}[kind]
    seed, iters, nq = 11, 150, 5
    inputs, want = _oracle_sequence(mode, obs, seed, iters, nq)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    _write_inputs(fin, mode, inputs)
    run = subprocess.run([EXE, str(fin), str(fout), str(seed), str(iters), "1"], capture_output=True, text=True,
                         timeout=300)
    print(run.stdout)
    assert run.returncode == 0, run.stdout + run.stderr
    got = _read_outputs(fout)
    assert len(got) == nq
    for q, (g, w) in enumerate(zip(got, want)):
        assert g["outcome"] == w["outcome"], q
        assert g["iterations"] == iters, q
        assert g["tree"] == w["tree"], q
        assert g["markers"] == w["markers"], q
        assert g["ids"] == w["ids"], q
        assert g["found"] == (len(w["ids"]) > 0), q
        assert g["counters"] == w["counters"], q
        # oracle message: x, y, theta, delta (NaN), v, a, a_cmd, d_cmd; the adapter's drops delta
        wm = np.delete(w["msg"], 3, axis=1) if len(w["msg"]) else np.zeros((0, 7))
        assert g["msg"].shape == wm.shape, q
        assert np.array_equal(g["msg"].view(np.uint64), np.ascontiguousarray(wm).view(np.uint64)), q
        assert g["published"] == int(len(wm) >= 3), q
    if kind == "moving20":
        assert not any(g["found"] for g in got)
    else:
        assert all(len(w["ids"]) for w in want), "a query without a path: the message comparison covers less"
