"""The C++ Simulation adapter and the reference-signature drop-ins (include/clrrt_adapter.hpp:
clrrt_adapter::Simulation / dropin::Simulation / dropin::expandTree) linked against libclrrt without
Python: tests/native/sim_adapter.cpp builds references as getReference / getGoalReference do
(reference.cpp:9-70), runs Simulation(RRT, state, ref, veh, GoalBiased, true, Vstart)
(simulation.h:18-19), and writes every stateArray, the costs, the flags and ref.v; they must equal the
CPU oracle's Simulation bit for bit.  The program also checks that expandTree reloads a tree whose
root changed at equal size and that a reference no getReference builds is refused."""
import ctypes as C
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import ref_tree as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "sim_adapter")


def test_native_sim_adapter_compiles_against_the_header():
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "sim_adapter.cpp")], check=True)


def _cases(seed=31, n=240):
    rng = np.random.default_rng(seed)
    H = T.sim_parents(rng, 40)
    J = T.sim_jobs(rng, H, n)
    return H, J


@pytest.mark.gpu
@pytest.mark.parametrize("coll", [0, 1])
def test_native_simulation_adapter_matches_oracle(coll):
    from oracle_binding import Oracle, lib as olib
    assert os.path.exists(EXE), "tests/native/sim_adapter not built (make -C cl-rrt_amd/csrc)"
    H, J = _cases(31 + coll)
    goal = (40.0, 0.0, 0.0, 0.0)
    obs = T.scene(200, 0) if coll else np.zeros((0, 7))
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            f.write(struct.pack("<iii", coll, len(obs), len(J)))
            f.write(np.array(goal, dtype="<f8").tobytes())
            f.write(np.ascontiguousarray(obs, dtype="<f8").tobytes())
            for j in J:
                h = H[int(j[0])]
                f.write(h[:10].astype("<f8").tobytes())
                f.write(np.array([h[18], h[19], j[2], j[3], h[20]], dtype="<f8").tobytes())
                f.write(struct.pack("<ii", int(j[1]), 0))
        out = subprocess.run([EXE, fin, fout], capture_output=True, text=True, timeout=120)
        print(out.stdout)
        assert out.returncode == 0, out.stdout + out.stderr
        buf = open(fout, "rb").read()
    o = Oracle(T.params(coll, goal), obs if coll else None)
    o.L.orc_load_tree(o.h, T.node_array(H), len(H))
    L = olib()
    pos = 0
    oc = C.c_int(); costs = (C.c_double * 2)(); fin10 = (C.c_double * 10)(); rb = (C.c_double * 3)(); rn = C.c_int()
    rows_o = np.zeros((520, 10))
    outcomes = []
    for k, j in enumerate(J):
        outcome, nrows, nv, flags = struct.unpack_from("<iiii", buf, pos); pos += 16
        cE, cS = struct.unpack_from("<dd", buf, pos); pos += 16
        v = np.frombuffer(buf, "<f8", nv, pos); pos += 8 * nv
        rows = np.frombuffer(buf, "<f8", 10 * nrows, pos).reshape(nrows, 10); pos += 80 * nrows
        nr = L.orc_simulate(o.h, int(j[0]), int(j[1]), j[2], j[3], C.byref(oc), costs, fin10, rb, C.byref(rn),
                            T.dp(rows_o), 520)
        assert (outcome, nrows) == (oc.value, nr), k
        assert flags == (outcome == 1) + 2 * (outcome == 2), k
        assert np.array_equal(np.array([cE, cS]).view(np.uint64), np.array(costs[:]).view(np.uint64)), k
        assert nv == rn.value and v[-1] == rb[2], k
        assert np.array_equal(rows.view(np.uint64), rows_o[:nr].view(np.uint64)), k
        outcomes.append(outcome)
    assert pos == len(buf)
    print("outcomes", np.bincount(outcomes, minlength=5))


@pytest.mark.gpu
def test_native_full_reference_nodes_match_oracle():
    """Engine::set_full_reference (include/clrrt_adapter.hpp): nodes grown by expandTree (EXACT) and by a
    BATCH expandBudget carry the reference's full Node::ref -- all N points of ref.x / ref.y / ref.v
    (getReference / getGoalReference, reference.cpp:9-70, and generateVelocityProfile, :72-170) -- equal
    to the oracle's, bit for bit, node for node."""
    from oracle_binding import Oracle
    assert os.path.exists(EXE), "tests/native/sim_adapter not built (make -C cl-rrt_amd/csrc)"
    goal = (40.0, 0.0, 0.0, 0.0)
    obs = T.scene(200, 0)
    root = np.array([0.0, 0.0, 0.0, 0.0, 2.0, 0.0, 0.0, 0.0, 0.0, 0.0])
    trees = [(5, 120, 0), (6, 512, 64)]  # BATCH rounds of the engine's max_batch (64)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        tin, tout = os.path.join(td, "t.bin"), os.path.join(td, "tout.bin")
        with open(fin, "wb") as f:
            f.write(struct.pack("<iii", 1, len(obs), 0))
            f.write(np.array(goal, dtype="<f8").tobytes())
            f.write(np.ascontiguousarray(obs, dtype="<f8").tobytes())
        with open(tin, "wb") as f:
            f.write(struct.pack("<i", len(trees)))
            for seed, iters, batch in trees:
                f.write(struct.pack("<iiii", seed, iters, batch, 0))
                f.write(root.astype("<f8").tobytes())
        out = subprocess.run([EXE, fin, fout, tin, tout], capture_output=True, text=True, timeout=300)
        print(out.stdout)
        assert out.returncode == 0, out.stdout + out.stderr
        buf = open(tout, "rb").read()
    pos = 0
    for seed, iters, batch in trees:
        o = Oracle(T.params(1, goal), obs)
        Oracle.srand(seed)
        o.init_tree(root)
        if batch:
            o.expand_batch(iters, batch, stable=True)
        else:
            o.expand(iters)
        (n,) = struct.unpack_from("<i", buf, pos); pos += 4
        assert n == o.size() and n > 20, (seed, n, o.size())
        on = o.nodes()
        full = 0
        for i in range(n):
            par, N = struct.unpack_from("<ii", buf, pos); pos += 8
            x = np.frombuffer(buf, "<f8", N, pos); pos += 8 * N
            y = np.frombuffer(buf, "<f8", N, pos); pos += 8 * N
            v = np.frombuffer(buf, "<f8", N, pos); pos += 8 * N
            assert par == on["parent"][i], (seed, i)
            ox, oy, ov = o.ref(i)
            assert N == len(ox), (seed, i, N, len(ox))
            for a, b in ((x, ox), (y, oy), (v, ov)):
                assert np.array_equal(a.view(np.uint64), np.ascontiguousarray(b, dtype=np.float64).view(np.uint64)), (seed, i)
            full += N > 2
        print(f"tree seed {seed} ({'BATCH' if batch else 'EXACT'}): {n} nodes, {full} with full references")
        assert full > 10
    assert pos == len(buf)

