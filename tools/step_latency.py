"""Per-step latency of the rollout step (k_rollout, one lane per job) for the longest rollouts of a cfg3
round: one job alone (the makespan's tail: a single lane on its SIMD), 64 copies (one dense wave) and
4096 copies (every SIMD busy).  Prints us per step and clock cycles per step at 2.4 GHz."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes

pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 27, max_batch=16384)  # jobs <= 10 x max_batch
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=40 * 16384, budget_ms=1e9, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 4096))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, k]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) for k in range(4) if ids[s, k] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] for r in res])
longest = [jobs[i] for i in np.argsort(-nr)[:8]]
print("longest rollouts (steps):", sorted(nr)[-8:])
pl.enable_timing(True)
for label, jl in (("1 lane", longest[:1]), ("8 lanes, 8 jobs", longest[:8]), ("64 copies", longest[:1] * 64),
                  ("4096 copies", longest[:1] * 4096), ("16384 copies", longest[:1] * 16384),
                  ("65536 copies", longest[:1] * 65536), ("131072 copies", longest[:1] * 131072)):
    for rep in range(3):
        pl.reset_counters()
        pl.enable_timing(True)  # resets the kernel timers (kernel_time accumulates)
        r = pl.simulate_batch(jl)
        ms, n = pl.kernel_time(1)
    steps = max(x["nrows"] - 1 for x in r)
    print(f"{label:18s}: kernel {ms:.3f} ms for {steps} steps -> {ms * 1e3 / steps:.2f} us/step "
          f"({ms * 1e-3 / steps * 2.4e9:,.0f} clk/step)")
# the same for a typical (median) job
med = jobs[int(np.argsort(nr)[len(nr) // 2])]
for label, jl in (("median job, 1 lane", [med]), ("median, 4096 copies", [med] * 4096)):
    for rep in range(3):
        pl.enable_timing(True)
        r = pl.simulate_batch(jl)
        ms, n = pl.kernel_time(1)
    steps = max(x["nrows"] - 1 for x in r)
    print(f"{label:18s}: kernel {ms:.3f} ms for {steps} steps -> {ms * 1e3 / max(1, steps):.2f} us/step")
