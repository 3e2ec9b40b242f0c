"""Diagnose the nearest-node search on a bench-sized tree: node clustering, brute force vs grid
search time (per sample mode, for several wave budgets) on a 16384-sample batch."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0
budgets = [int(b) for b in sys.argv[2].split(",")] if len(sys.argv) > 2 and sys.argv[2] else []
obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
pl.set_nn_grid(1 << 40, 0)
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
n = pl.nodes()
N = len(n["state"])
print("nodes", N, "rounds", st["rounds"])
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ex = np.array([s.explore for s in smp])


def timed(sub, modes, budget, ordered=False):
    pl.set_nn_grid(0 if modes else 1 << 40, modes, budget)
    pl.set_option("nn_ordered_min", 0 if ordered else 1 << 40)
    ref = pl.sort_nodes_batch(sub, exact=False)
    torch.cuda.synchronize()
    pl.reset_counters()
    t0 = time.perf_counter()
    ids, _ = pl.sort_nodes_batch(sub, exact=False)
    return (time.perf_counter() - t0) * 1e3, ids, pl.nn_stats()


for label, sel in (("explore", ex == 1), ("optimize", ex == 0), ("all", ex >= 0)):
    sub = [s for s, k in zip(smp, sel) if k]
    tb, ids_b, sb = timed(sub, 0, 0)
    to, ids_o, so = timed(sub, 0, 0, ordered=True)
    print(f"  {label:8s} {len(sub):5d} samples brute force: {tb:.1f} ms, place-ordered: {to:.1f} ms "
          f"equal={np.array_equal(ids_b, ids_o)} tiles {so['tiles_searched']}/{so['tiles_seen']}")
    print(f"      brute: queued {sb['pairs_queued']} exact {sb['exact_keys']}; ordered: queued {so['pairs_queued']} "
          f"exact {so['exact_keys']}")
    pl.set_option("nn_debug", 1)
    tn, _, _ = timed(sub, 0, 0)
    tno, _, _ = timed(sub, 0, 0, ordered=True)
    pl.set_option("nn_debug", 0)
    print(f"      without the exact pass: brute {tn:.1f} ms, ordered {tno:.1f} ms")
    for b in budgets:
        for modes in (1, 3):
            tg, ids_g, stt = timed(sub, modes, b)
            print(f"      grid modes={modes} budget={b}: {tg:.1f} ms equal={np.array_equal(ids_b, ids_g)} {stt}")
