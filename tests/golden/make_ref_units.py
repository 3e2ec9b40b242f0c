#!/usr/bin/env python3
"""Writes tests/golden/ref_units.npz + ref_units_meta.json: hot-path unit cases with the outputs of the
REFERENCE'S OWN CODE (oracle/_ref, built by `make -C oracle ref` from verbatim line ranges of
/root/reference; see oracle/Makefile and tests/ref_units.py).

Before writing, it checks the oracle against the reference on LIVE_N fresh cases per unit (bit for
bit) and records the comparison between the reference's build flavours (-O3 Release, -O2, -O0) and
the collision decisions under every choice of the reference's unset normsY[3].  Run it in the
development container (needs /root/reference):  python3 tests/golden/make_ref_units.py
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
import ref_units as R  # noqa: E402

FIX_N = {"obb": 2048, "geom": 1024, "ode": 2048, "lateral": 2048, "profile": 160, "angle": 2048,
         "dubins": 4096, "feasible": 4096, "goalbias": 4096, "goalref": 160, "ctrl": 384}
LIVE_N = {"obb": 100000, "geom": 100000, "ode": 100000, "lateral": 100000, "profile": 20000, "angle": 100000,
          "dubins": 100000, "feasible": 100000, "goalbias": 100000, "goalref": 20000, "ctrl": 10000}
FIX_SEED, LIVE_SEED = 20261016, 7


def compare(unit, o, r):
    if unit == "geom":  # vertices, normals 0..2; the oracle's canonical ny[3] == the reference's normsX[3]
        cols = list(range(11)) + [12, 13, 14]
        return len(R.mismatches(o[:, cols], r[:, cols])) + len(R.mismatches(o[:, 15:16], r[:, 15:16]))
    return len(R.mismatches(o, r))


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    libs = {f: R.reference_lib(f) for f in ("O3", "O2", "O0")}
    ref = libs["O3"]
    meta = {"reference": "vdBerg93/cl-rrt at /root/reference (line ranges in oracle/Makefile)",
            "compiler": subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
            "flags": "-std=c++11 -O3 -DNDEBUG -ffp-contract=off (CMake Release), zero-fill padded operator new",
            "live": {}, "fixture_cases": FIX_N}
    for unit in FIX_N:
        x = R.cases(unit, LIVE_N[unit], LIVE_SEED)
        outs = {}
        for f, L in libs.items():
            y = R.run_reference(L, unit, x)
            outs[f] = y[0] if unit == "ode" else y
        o = R.run_oracle(unit, x)
        rec = {"cases": int(x.shape[0]), "oracle_vs_O3": compare(unit, o, outs["O3"]),
               "O2_vs_O3": compare(unit, outs["O2"], outs["O3"]), "O0_vs_O3": compare(unit, outs["O0"], outs["O3"])}
        if unit == "obb":
            dec = outs["O3"][:, 0] == 0
            rec["overlaps"] = int(dec.sum())
            rec["axis3_decision_flips"] = {
                str(m): int(((R.run_reference(ref, unit, x, m)[:, 0] == 0) != dec).sum()) for m in (1, 2, 3)}
        meta["live"][unit] = rec
        print(unit, rec, flush=True)
        if rec["oracle_vs_O3"]:
            sys.exit(f"oracle differs from the reference's {unit}: fix the oracle before writing fixtures")
    arrays = {}
    for unit, n in FIX_N.items():
        x = R.cases(unit, n, FIX_SEED)
        y = R.run_reference(ref, unit, x)
        if unit == "ode":
            y = y[0]
        if unit in ("profile", "goalref"):
            nmax = int(y[:, 0].max())
            assert nmax <= R.NMAX
            y = np.concatenate([y[:, :1 + nmax], y[:, 1 + R.NMAX:1 + R.NMAX + nmax],
                                y[:, 1 + 2 * R.NMAX:1 + 2 * R.NMAX + nmax]], 1)
            meta[f"{unit}_nmax"] = nmax
        arrays[f"{unit}_in"] = x
        arrays[f"{unit}_out"] = y
    arrays["prius"] = R.reference_prius(ref)
    np.savez_compressed(os.path.join(HERE, "ref_units.npz"), **arrays)
    with open(os.path.join(HERE, "ref_units_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote ref_units.npz / ref_units_meta.json")


if __name__ == "__main__":
    main()
