"""Can the longest rollouts (iteration-limit orbits, the rollout kernel's tail) be told apart before they
run?  Grow a cfg3 tree for argv[1] rounds, simulate the first 4 candidates of 16384 samples and tabulate
steps against the initial geometry: the angle between the parent's heading and the direction to the
sample, and the sample's distance."""
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
nd = pl.nodes()
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, k]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) for k in range(4) if ids[s, k] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] - 1 for r in res])
oc = np.array([r["outcome"] for r in res])
par = np.array([j[0] for j in jobs])
sx = np.array([j[2] for j in jobs]); sy = np.array([j[3] for j in jobs])
st = nd["state"][par]
bx, by = nd["ref_back"][par, 0], nd["ref_back"][par, 1]
dx, dy = sx - st[:, 0], sy - st[:, 1]
dist = np.hypot(dx, dy)
ang = np.abs(np.mod(np.arctan2(dy, dx) - st[:, 2] + np.pi, 2 * np.pi) - np.pi)
v0 = st[:, 4]
rdist = np.hypot(sx - bx, sy - by)  # the new reference runs from the parent's ref.back() to the sample
long_ = nr >= 300
print(f"jobs {len(jobs)}, >= 300 steps: {long_.sum()} (outcomes {np.bincount(oc[long_], minlength=5).tolist()})")
print("angle bin (deg) x distance bin (m): long jobs / all jobs")
ab = [0, 30, 60, 90, 120, 150, 181]
db = [0, 2, 4, 6, 8, 12, 20, 1000]
print("          " + "".join(f"{f'{db[i]}-{db[i + 1]}':>12s}" for i in range(len(db) - 1)))
for a0, a1 in zip(ab[:-1], ab[1:]):
    row = []
    for d0, d1 in zip(db[:-1], db[1:]):
        m = (np.degrees(ang) >= a0) & (np.degrees(ang) < a1) & (dist >= d0) & (dist < d1)
        row.append(f"{int(long_[m].sum())}/{int(m.sum())}")
    print(f"{a0:3d}-{a1:3d}   " + "".join(f"{x:>12s}" for x in row))
for thr in (45, 60, 75, 90):
    for dmax in (6, 8, 12):
        m = (np.degrees(ang) >= thr) & (dist < dmax)
        print(f"predict long if angle >= {thr} deg and dist < {dmax} m: flags {m.sum()} jobs "
              f"({m.mean() * 100:.1f}%), catches {long_[m].sum()} of {long_.sum()} long, flagged steps "
              f"{nr[m].sum() / nr.sum() * 100:.1f}% of all")
print(f"reference length (m) of long jobs: p50 {np.median(rdist[long_]):.2f}, others p50 {np.median(rdist[~long_]):.2f}")
print(f"initial speed of long jobs p50 {np.median(v0[long_]):.2f}, others {np.median(v0[~long_]):.2f}")
