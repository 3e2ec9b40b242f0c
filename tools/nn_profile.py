"""Nearest-node search on a bench-sized tree (cfg3 scene, BATCH expansion for `ms`): how many nodes a
sample's list actually depends on (Euclidean lower bound vs the 11th key) and the brute-force /
place-ordered / grid timings on one 16384-sample batch."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 26, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
n = pl.nodes()
N = len(n["state"])
x, y = n["state"][:, 0], n["state"][:, 1]
ce = n["costE"].astype(np.float64)
print("nodes", N, "rounds", st["rounds"], "x", np.percentile(x, [0, 5, 50, 95, 100]).round(1),
      "y", np.percentile(y, [0, 5, 50, 95, 100]).round(1))
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ex = np.array([s.explore for s in smp])
sx = np.array([s.x for s in smp]); sy = np.array([s.y for s in smp])
ids, keys = pl.sort_nodes_batch(smp, exact=False)
k10 = keys[:, 9].astype(np.float64)
for lab, m in (("explore", ex == 1), ("optimize", ex == 0)):
    print(f"{lab}: {m.sum()} samples, 10th key pct", np.percentile(k10[m][np.isfinite(k10[m])], [5, 50, 95]).round(2),
          "unfilled", int((~np.isfinite(k10[m])).sum()))
    sel = np.nonzero(m)[0][:300]
    need = []
    for s in sel:
        d = np.hypot(x - sx[s], y - sy[s])
        lb = d if lab == "explore" else ce + d
        need.append(int((lb <= k10[s]).sum()))
    print("   nodes with lower bound <= 10th key per sample: pct", np.percentile(need, [5, 50, 95, 100]))


def timed(modes, budget, ordered=False):
    pl.set_nn_grid(0 if modes else 1 << 40, modes, budget)
    pl.set_option("nn_ordered_min", 0 if ordered else 1 << 40)
    pl.sort_nodes_batch(smp, exact=False)
    torch.cuda.synchronize()
    pl.reset_counters()
    t0 = time.perf_counter()
    r, _ = pl.sort_nodes_batch(smp, exact=False)
    return (time.perf_counter() - t0) * 1e3, r, pl.nn_stats()


tb, rb, sb = timed(0, 0)
print(f"brute: {tb:.2f} ms {sb}")
to, ro, so = timed(0, 0, True)
print(f"ordered: {to:.2f} ms equal={np.array_equal(rb, ro)} {so}")
for modes in ():
    for b in (0, 2048, 8192):
        tg, rg, sg = timed(modes, b)
        print(f"grid modes={modes} budget={b}: {tg:.2f} ms equal={np.array_equal(rb, rg)} {sg}")
pl.set_option("nn_debug", 1)
td, _, sd = timed(0, 0)
pl.set_option("nn_debug", 0)
print(f"brute without the exact pass: {td:.2f} ms {sd}")
for lab, m in (("explore", ex == 1), ("optimize", ex == 0)):
    sub = [s for s, k in zip(smp, m) if k]
    pl.set_nn_grid(1 << 40, 0, 0); pl.set_option("nn_ordered_min", 1 << 40)
    pl.sort_nodes_batch(sub, exact=False); torch.cuda.synchronize(); pl.reset_counters()
    t0 = time.perf_counter(); pl.sort_nodes_batch(sub, exact=False)
    print(f"brute {lab} only ({len(sub)}): {(time.perf_counter() - t0) * 1e3:.2f} ms {pl.nn_stats()}")
