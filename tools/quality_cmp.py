"""Best-path quality of BATCH vs EXACT expansion on cfg3's scene.

EXACT grows the reference's own sequential tree; BATCH evaluates B samples per round against the tree frozen
at the round's start.  For each seed and wall budget: nodes, goal (feasible) nodes and the costS of the path
extractBestPath picks (lower is better; inf = no path), for EXACT, BATCH at B = 16384 (the bench) and BATCH at
B = 256 with EXACT's iteration count (the same number of samples: what the frozen-tree rounds cost per sample)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: E402,F401
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

budgets = [float(x) for x in sys.argv[1:]] or [200.0, 2000.0]
seeds = [1, 2, 3, 4, 5]
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=6 << 20,
                   max_rows=1 << 30, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))


def run(mode, seed, budget=0.0, iters=0, batch=16384):
    pl.tree_init()
    t0 = time.perf_counter()
    st = pl.expand(clrrt.Rng(seed), n_iters=iters, budget_ms=budget, mode=mode, batch=batch)
    wall = (time.perf_counter() - t0) * 1e3
    ids, cost, ng = pl.extract_best_path()
    return dict(nodes=pl.size()[0], iters=st["iterations"], goal=ng, cost=cost if ids else float("inf"), ms=wall)


run(clrrt.CLRRT_MODE_BATCH, 99, budget=200.0)  # warm-up
for budget in budgets:
    rows = []
    for seed in seeds:
        ex = run(clrrt.CLRRT_MODE_EXACT, seed, budget=budget, batch=256)
        bb = run(clrrt.CLRRT_MODE_BATCH, seed, budget=budget)
        bs = run(clrrt.CLRRT_MODE_BATCH, seed, iters=ex["iters"], batch=256)
        rows.append((ex, bb, bs))
        print(f"budget {budget:6.0f} ms seed {seed}: EXACT {ex['nodes']} nodes {ex['goal']} goal cost {ex['cost']:.2f} | "
              f"BATCH {bb['nodes']} nodes {bb['goal']} goal cost {bb['cost']:.2f} | BATCH same samples "
              f"({ex['iters']}, B=256) {bs['nodes']} nodes {bs['goal']} goal cost {bs['cost']:.2f}", flush=True)
    med = lambda k, i: float(np.median([r[i][k] for r in rows]))
    print(f"budget {budget:6.0f} ms median: EXACT cost {med('cost', 0):.2f} ({med('nodes', 0):.0f} nodes), BATCH cost "
          f"{med('cost', 1):.2f} ({med('nodes', 1):.0f} nodes), BATCH same samples cost {med('cost', 2):.2f}", flush=True)
