"""Latency split of one rollout step for the makespan's stragglers: the longest rollouts of a cfg3 round
run alone (one lane on its SIMD: the kernel's tail) and as 64 copies (one dense wave), in the diagnostics
build (make -C cl-rrt_amd/csrc prof; CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so) whose k_rollout records shader
clocks per phase of the step.  Prints clocks per step and per phase."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

NAMES = ["loop", "waypoint (cos, sin, scan)", "lateral + control + ODE", "sincos + tan + cos/sin", "collision",
         "costs / end checks + row store", "-", "-"]
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 27, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=int(sys.argv[1]) if len(sys.argv) > 1 else 30 * 16384, budget_ms=1e9,
          mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 4096))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, k]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) for k in range(4) if ids[s, k] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] for r in res])
order = np.argsort(-nr)
print("tree", pl.size()[0], "jobs", len(jobs), "longest rollouts (steps):", nr[order[:8]].tolist(),
      "outcomes", [res[i]["outcome"] for i in order[:8]])
pl.enable_timing(True)
for label, jl in (("1 lane, longest", [jobs[order[0]]]), ("1 lane, 2nd", [jobs[order[1]]]),
                  ("1 lane, 8th", [jobs[order[7]]]), ("64 copies of the longest", [jobs[order[0]]] * 64),
                  ("1 lane, median", [jobs[order[len(order) // 2]]]),
                  ("64 distinct longest", [jobs[i] for i in order[:64]]),
                  ("64 distinct, random", [jobs[i] for i in np.random.default_rng(3).choice(len(jobs), 64, False)]),
                  ("longest + 63 random", [jobs[order[0]]] + [jobs[i] for i in
                                                              np.random.default_rng(4).choice(len(jobs), 63, False)])):
    pl.reset_counters()
    pl.enable_timing(True)  # resets the kernel timers (kernel_time accumulates)
    r = pl.simulate_batch(jl)
    ms, _ = pl.kernel_time(1)
    d = pl.debug_counters()
    steps = sum(x["nrows"] - 1 for x in r)
    lanes = len(jl)
    smax = max(x["nrows"] - 1 for x in r)
    ph = np.array(d[40:48], dtype=np.float64) / max(1, steps)  # per lane-step (per lane clocks)
    tot = ph.sum()
    print(f"{label:28s} kernel {ms:.3f} ms, {steps // lanes} steps/lane, {tot:,.0f} clk per step "
          f"({ms * 1e-3 * 2.4e9 / max(1, steps // lanes):,.0f} wall clk/step at 2.4 GHz; longest lane {smax} steps, "
          f"{ms * 1e-3 * 2.4e9 / max(1, smax):,.0f} wall clk per its step)")
    for nm, v in zip(NAMES, ph):
        if v > 0:
            print(f"    {nm:32s} {v:9,.0f} clk  {v / max(1, tot) * 100:5.1f}%")
    if label.startswith("1 lane, longest"):
        w = pl.work_counters()
        print(f"    scan points per step {w['scan_points'] / max(1, steps):.1f}, box tests per step "
              f"{w['box_tests'] / max(1, steps):.1f}")
