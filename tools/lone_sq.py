"""Instruction mix of one lone rollout (a single lane on its SIMD: the makespan's tail and EXACT mode's
critical path), for SQ counter passes: the longest rollout of a cfg3 round run alone through k_rollout
(simulate_batch) 3 times, then 40 EXACT iterations at speculation width 1 (k_roll_run with one sample's
candidates).  Run under `rocprofv3 --pmc SQ_... --kernel-include-regex "k_roll"`; per-step figures are the
counters of one k_rollout dispatch over the printed step count."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                   max_rows=1 << 26, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=4 * 16384, budget_ms=1e9, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 1024))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, k]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) for k in range(4) if ids[s, k] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] for r in res])
i = int(np.argmax(nr))
print(f"tree {pl.size()[0]} nodes; longest rollout {nr[i] - 1} steps (outcome {res[i]['outcome']})", flush=True)
for rep in range(3):
    pl.reset_counters()
    r = pl.simulate_batch([jobs[i]])
    print(f"lone k_rollout: {r[0]['nrows'] - 1} steps, scan points {pl.debug_counters()[1]}, box tests "
          f"{pl.debug_counters()[2]}", flush=True)
pl.reset_counters()
pl.set_option("exact_min_width", 1)
st = pl.expand(clrrt.Rng(9), n_iters=40, budget_ms=1e9, mode=clrrt.CLRRT_MODE_EXACT, batch=1)
print(f"EXACT width 1: {st['iterations']} iterations in {st['rounds']} rounds, rollout steps {pl.debug_counters()[0]}",
      flush=True)
