#!/usr/bin/env python3
"""Writes tests/golden/capi_exact_obb200_s3.bin, the expected outputs for tests/native/capi_exact.cpp (the
C++ drop-in test linked against libclrrt): the CPU oracle's sequential expandTree on the 200-obstacle
scene (SURVEY.md §8(d) generator), srand(3), 300 iterations — node headers, an FNV-1a hash of every
node's trajectory rows, the counters — and checkObsDistance on 48 states.

Format (little endian): b"CLRF", int32 version 1, int32 n_obs, double[n_obs][7] obstacles, int32 n_nodes,
clrrt_node[n_nodes] (160 B), uint64[n_nodes] row hashes, int64[5] counters (sim_count, fail_collision,
fail_acclimit, fail_iterlimit, rollouts), int32 n_states, double[n_states][10] states,
double[n_states] distances.
Run from the repo root:  python3 tests/golden/make_capi_fixture.py
"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from clrrt import abi, scenes  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

SEED, ITERS = 3, 300


def fnv1a(b):
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def main():
    obs = scenes.urban_scene(200)
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
    Oracle.srand(SEED)
    o.init_tree()
    o.expand(ITERS)
    raw = o.nodes_raw()
    n = len(raw)
    hashes = [fnv1a(np.ascontiguousarray(o.rows(i)).tobytes()) for i in range(n)]
    cnt = o.counters()
    rng = np.random.default_rng(4)
    states = np.zeros((48, 10))
    states[:, 0] = rng.uniform(5, 60, 48)
    states[:, 1] = rng.uniform(-20, 20, 48)
    states[:, 2] = rng.uniform(-3.2, 3.2, 48)
    states[:, 6] = rng.uniform(0, 10, 48)
    dist = np.array([o.check_obs(s) for s in states])
    out = bytearray(b"CLRF") + struct.pack("<ii", 1, len(obs)) + np.ascontiguousarray(obs, dtype="<f8").tobytes()
    out += struct.pack("<i", n) + bytes(raw) + struct.pack(f"<{n}Q", *hashes)
    out += struct.pack("<5q", cnt["sim_count"], cnt["fail_collision"], cnt["fail_acclimit"], cnt["fail_iterlimit"],
                       cnt["rollouts"])
    out += struct.pack("<i", len(states)) + states.astype("<f8").tobytes() + dist.astype("<f8").tobytes()
    path = os.path.join(HERE, f"capi_exact_obb200_s{SEED}.bin")
    open(path, "wb").write(bytes(out))
    print(f"wrote {path}: {n} nodes, counters {cnt}, {int((dist == 0).sum())} of 48 states colliding")


if __name__ == "__main__":
    main()
