"""Regenerates tests/golden/oracle_vectors.json from the CPU oracle (oracle/liboracle.so) and glibc.

The oracle is itself pinned to the reference's outputs (survey_pins.json); these vectors freeze
small oracle outputs (rand() streams, rollout / sort known answers) so a change in the oracle or
in glibc shows up as a diff.  Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "cl-rrt_amd"))

from oracle_binding import Oracle, lib  # noqa: E402
from clrrt import abi, scenes  # noqa: E402


def main():
    out = {"rand": {}}
    for seed in range(1, 9):
        lib().orc_srand(seed)
        out["rand"][str(seed)] = [lib().orc_rand() for _ in range(32)]
    # rollouts from the root / early nodes, empty + 200-obstacle scenes
    vec = []
    for mode, obs in ((abi.CLRRT_COLLISION_STUB, None), (abi.CLRRT_COLLISION_OBB, scenes.urban_scene(200))):
        p = abi.default_params(collision_mode=mode)
        o = Oracle(p, obs)
        Oracle.srand(7)
        o.init_tree()
        o.expand(12)
        xy, ex = o.draw_samples(6)
        for j in range(6):
            ids, keys = o.sort_nodes(xy[j][0], xy[j][1], ex[j])
            for par in ids[:3]:
                r = o.simulate(par, 0, xy[j][0], xy[j][1])
                vec.append({"collision_mode": mode, "tree_seed": 7, "tree_iters": 12, "parent": par,
                            "sample": list(xy[j]), "outcome": r["outcome"], "nrows": r["nrows"],
                            "costE": r["costE"], "costS": r["costS"], "final": list(r["final"])})
            vec.append({"collision_mode": mode, "tree_seed": 7, "tree_iters": 12, "sort_sample": list(xy[j]),
                        "explore": int(ex[j]), "ids": ids, "keys": keys})
    out["oracle_vectors"] = vec
    with open(os.path.join(HERE, "oracle_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(vec), "vectors")


if __name__ == "__main__":
    main()
