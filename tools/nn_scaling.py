"""Walk search time vs the number of samples on one large tree (cfg3 scene grown for argv[1] ms): if the
time does not fall with the sample count, a round's search is bound by its slowest samples (latency),
not by throughput.  Also the per-sample cost spread (walk stats of single samples)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 6000.0
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=8 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
print("nodes", pl.size()[0], flush=True)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
pl.set_option("nn_walk_min", 0)


def t(sub, reps=3):
    pl.sort_nodes_batch(sub, exact=False)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        pl.sort_nodes_batch(sub, exact=False)
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


for lab, pick in (("explore", 1), ("optimize", 0)):
    sub = [s for s in smp if s.explore == pick]
    for n in (len(sub), 4096, 1024, 256, 64, 16, 1):
        print(f"{lab:8s} {n:6d} samples: {t(sub[:n]):8.2f} ms", flush=True)
# per-sample cost spread: exact keys and tiles of 400 single samples (optimize and explore)
for lab, pick in (("explore", 1), ("optimize", 0)):
    sub = [s for s in smp if s.explore == pick][:300]
    ex, ti, tm, qd = [], [], [], []
    for s in sub:
        pl.reset_counters()
        t0 = time.perf_counter()
        pl.sort_nodes_batch([s], exact=False)
        tm.append((time.perf_counter() - t0) * 1e3)
        st = pl.nn_stats()
        dc = pl.debug_counters()
        ex.append(st["walk_exact"]); ti.append(st["walk_tiles"])
        qd.append((st["walk_queued"], dc[28], dc[29], dc[30]))
    ex, ti, tm = np.array(ex), np.array(ti), np.array(tm)
    q = lambda a: [round(float(np.percentile(a, p)), 1) for p in (50, 90, 99, 100)]
    print(f"{lab}: single-sample exact keys p50/90/99/max {q(ex)}, tiles {q(ti)}, ms {q(tm)}")
    qd = np.array(qd)
    print(f"   per sample: queued {qd[:, 0].mean():.0f}, stage-1 undecided {qd[:, 1].mean():.0f}, surely feasible "
          f"{qd[:, 2].mean():.0f}, stage-2 dropped {qd[:, 3].mean():.0f}, exact {ex.mean():.0f}")
    far = np.argsort(-ex)[:3]
    for i in far:
        print(f"   costly sample ({sub[i].x:.2f}, {sub[i].y:.2f}): exact {ex[i]}, tiles {ti[i]}, {tm[i]:.2f} ms")
