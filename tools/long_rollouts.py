"""What the longest rollouts of a cfg3 round do (they set the rollout kernel's makespan): grow a tree for
argv[1] rounds, take 16384 samples' first 4 candidates, simulate them, and describe the jobs that run
longest (outcome, speed, waypoint progress, the last step at which the state changed)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 40
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 27, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=rounds * 16384, budget_ms=1e9, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, k]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) for k in range(4) if ids[s, k] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] for r in res])
oc = np.array([r["outcome"] for r in res])
print(f"jobs {len(jobs)}; steps mean {nr.mean() - 1:.1f}, p50 {np.percentile(nr, 50) - 1:.0f}, p99 {np.percentile(nr, 99) - 1:.0f}, "
      f"p99.9 {np.percentile(nr, 99.9) - 1:.0f}, max {nr.max() - 1}")
for o in sorted(set(oc.tolist())):
    m = oc == o
    print(f"  outcome {o}: {m.sum()} jobs, steps mean {nr[m].mean() - 1:.1f} max {nr[m].max() - 1}")
order = np.argsort(-nr)[:40]
long_jobs = [jobs[i] for i in order]
lr = pl.simulate_batch(long_jobs, rows=True)
if lr is None:
    # rows capped at 512 by simulate_batch; describe from the final state only
    for i in order[:20]:
        r = res[i]
        f = r["final"]
        print(f"  job {i}: outcome {r['outcome']} steps {r['nrows'] - 1} refN {r['ref_n']} v {f[4]:.4g} a {f[5]:.3g} "
              f"wp {f[7]:.0f} vback {r['ref_vback']:.3g} costE {r['costE']:.3g}")
else:
    for r in lr[:20]:
        rows = r["rows"]
        ch = np.nonzero(np.any(rows[1:, [0, 1, 2, 3, 4, 5, 7]] != rows[:-1, [0, 1, 2, 3, 4, 5, 7]], axis=1))[0]
        print(f"  outcome {r['outcome']} steps {r['nrows'] - 1} refN {r['ref_n']} v_end {rows[-1, 4]:.4g} "
              f"wp_end {rows[-1, 7]:.0f} last change at step {ch[-1] + 1 if len(ch) else 0}")
