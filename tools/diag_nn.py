"""Diagnose the nearest-node search on a bench-sized tree: node clustering and the time of the
explore / optimize halves of a 16384-sample batch (brute force vs grid)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0,
               mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
n = pl.nodes()
xy = n["state"][:, :2]
N = len(xy)
print("nodes", N, "rounds", st["rounds"])
d0 = np.hypot(xy[:, 0] - xy[0, 0], xy[:, 1] - xy[0, 1])
for r in (0.01, 0.1, 0.5, 1, 2, 5):
    print(f"  within {r} m of root: {int((d0 < r).sum())}")
u, cnt = np.unique(np.round(xy, 6), axis=0, return_counts=True)
print("  distinct positions", len(u), "max multiplicity", cnt.max())
print("  bbox", xy.min(0), xy.max(0))
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ex = np.array([s.explore for s in smp])
for label, sel in (("explore", ex == 1), ("optimize", ex == 0)):
    sub = [s for s, k in zip(smp, sel) if k]
    for grid in (False, True):
        pl.set_nn_grid_threshold(0 if grid else 1 << 40)
        pl.sort_nodes_batch(sub, exact=False)
        torch.cuda.synchronize()
        pl.reset_counters()
        t0 = time.perf_counter()
        pl.sort_nodes_batch(sub, exact=False)
        t = time.perf_counter() - t0
        print(f"  {label:8s} {len(sub)} samples grid={grid}: {t*1e3:.1f} ms", pl.nn_stats() if grid else "")
