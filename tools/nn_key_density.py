"""How many nodes lie near a sample's 11th key (cfg3 scene grown for argv[1] ms)?  The walk must compute
the exact key of every feasible node whose key bound does not exceed the 11th key, so the count of
feasible nodes with key <= k11 + margin (and how many distinct key inputs they have) is the floor of its
exact-key work.  Keys in float32 numpy (tests/test_nnwalk_bounds.py), feasibility in float64."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes
from test_nnwalk_bounds import dubins_key_f32

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 3000.0
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=8 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
nd = pl.nodes()
N = len(nd["parent"])
x, y, th = nd["state"][:, 0], nd["state"][:, 1], nd["state"][:, 2]
c = np.cos(np.float32(-th)).astype(np.float32)
s = np.sin(np.float32(-th)).astype(np.float32)
bx, by, ap = nd["ref_back"][:, 0], nd["ref_back"][:, 1], nd["ang_par"]
ce = nd["costE"].astype(np.float32)
feas_len = 2.1 * pl.params.ref_res  # DevParams.feas_len (clrrt_capi.hip)
print(f"nodes {N}, distinct positions {len(np.unique(np.stack([x, y], 1), axis=0))}", flush=True)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
# argv[2:]: extra samples "x,y,explore" (e.g. the costly ones nn_scaling.py reports), analysed first
extra = []
for a in sys.argv[2:]:
    x_, y_, e_ = a.split(",")
    q = clrrt.abi.Sample() if hasattr(clrrt.abi, "Sample") else type(smp[0])()
    q.x, q.y, q.explore = float(x_), float(y_), int(e_)
    extra.append(q)
smp = extra + smp
deltas = (0.0, 1e-4, 1e-3, 1e-2, 0.1, 1.0)


def analyse(j):
    sx, sy, ex = smp[j].x, smp[j].y, smp[j].explore
    qx = (sx - x).astype(np.float32)
    qy = (sy - y).astype(np.float32)
    tx = c * qx - s * qy
    ty = np.abs(s * qx + c * qy)
    key = dubins_key_f32(tx, ty).astype(np.float32)
    if not ex:
        key = (ce + key).astype(np.float32)
    ang = np.arctan2(sy - by, sx - bx)
    d = np.mod(ang - ap + np.pi, 2 * np.pi) - np.pi
    feas = (np.abs(d) <= np.pi / 4) & (np.hypot(bx - sx, by - sy) >= feas_len)
    kf = key[feas].astype(np.float64)
    order = np.lexsort((np.nonzero(feas)[0], kf))
    k11 = kf[order[10]] if len(order) > 10 else np.inf
    cnt = [int(np.sum(kf <= k11 + dd)) for dd in deltas]
    near = feas & (key <= k11 + 1e-3)
    dist = len(np.unique(np.stack([x[near], y[near], th[near]], 1), axis=0))
    distc = len(np.unique(np.stack([x[near], y[near], th[near], ce[near].astype(np.float64)], 1), axis=0))
    rad = np.hypot(x[near], y[near])
    print(f"{'explore' if ex else 'optimize'} sample ({sx:.2f}, {sy:.2f}): k11 {k11:.4f}; feasible nodes with key "
          f"<= k11 + {deltas}: {cnt}; distinct (x, y, th) within 1e-3: {dist}, with costE {distc}; their |p| "
          f"p50 {np.median(rad) if len(rad) else -1:.2f}", flush=True)
    return cnt + [dist]


for j in range(len(extra)):
    analyse(j)
for lab, pick in (("explore", 1), ("optimize", 0)):
    rows = [analyse(j) for j in [k for k in range(len(extra), len(smp)) if smp[k].explore == pick][:8]]
    print(f"{lab} median counts {np.median(np.array(rows), 0).tolist()}", flush=True)
