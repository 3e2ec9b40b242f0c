"""Walk search vs brute force on a bench-sized tree (cfg3 scene, BATCH expansion for `ms`): identical
candidate lists and the time of one 16384-sample search each."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
walk_grow = len(sys.argv) > 2 and sys.argv[2] == "walk"
obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=8 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
pl.set_option("nn_walk_min", 8192 if walk_grow else 1 << 40)
pl.enable_timing(True)
t0 = time.perf_counter()
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
print(f"grown with {'walk' if walk_grow else 'brute'}: nodes {pl.size()} rounds {st['rounds']} nn {pl.kernel_time(0)} "
      f"roll {pl.kernel_time(1)}", flush=True)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))


def timed(walk):
    pl.set_option("nn_walk_min", 0 if walk else 1 << 40)
    pl.sort_nodes_batch(smp, exact=False)
    torch.cuda.synchronize()
    pl.reset_counters()
    t0 = time.perf_counter()
    r = pl.sort_nodes_batch(smp, exact=False)
    return (time.perf_counter() - t0) * 1e3, r, pl.nn_stats()


tb, (ib, kb), sb = timed(False)
tw, (iw, kw), sw = timed(True)
bad = np.nonzero(~np.all(ib == iw, axis=1))[0]
print(f"brute {tb:.2f} ms, walk {tw:.2f} ms; lists equal: {len(bad) == 0} ({len(bad)} differ); keys equal "
      f"{np.array_equal(kb.view(np.uint32), kw.view(np.uint32))}")
print("walk stats", {k: v for k, v in sw.items() if k.startswith("walk")})
# overflow budget sweep (tiles, exact keys; 0 = off): time and identity with the brute force
for bt, be in ((0, 0), (4096, 24576), (4096, 8192), (4096, 4096), (4096, 2048)):
    for nch in ((32,) if bt == 0 else (16, 32)):
        pl.set_option("nn_walk_budget_tiles", bt)
        pl.set_option("nn_walk_budget_keys", be)
        pl.set_option("nn_walk_chunks", nch)
        best = 1e9
        for _ in range(3):
            tx, (ix, kx), _ = timed(True)
            best = min(best, tx)
        nov = pl.debug_counters()[32]
        same = bool(np.all(ib == ix)) and np.array_equal(kb.view(np.uint32), kx.view(np.uint32))
        print(f"budget tiles {bt} keys {be} chunks {nch}: walk {best:.2f} ms, overflow records {nov}, "
              f"equal to brute {same}", flush=True)
pl.set_option("nn_walk_budget_tiles", 4096)
pl.set_option("nn_walk_budget_keys", 4096)
pl.set_option("nn_walk_chunks", 32)
for i in bad[:5]:
    print("sample", i, smp[i].x, smp[i].y, smp[i].explore, "\n  brute", ib[i], kb[i], "\n  walk ", iw[i], kw[i])
ex = np.array([s.explore for s in smp])
for lab, m in (("explore", ex == 1), ("optimize", ex == 0)):
    sub = [s for s, k in zip(smp, m) if k]
    pl.set_option("nn_walk_min", 0)
    pl.set_option("nn_debug", 2)
    pl.sort_nodes_batch(sub, exact=False); torch.cuda.synchronize(); pl.reset_counters()
    t0 = time.perf_counter(); pl.sort_nodes_batch(sub, exact=False)
    s = pl.nn_stats()
    print(f"walk {lab} only ({len(sub)}): {(time.perf_counter() - t0) * 1e3:.2f} ms "
          f"{ {k: round(v / len(sub), 1) for k, v in s.items() if k.startswith('walk')} } per sample")
    dc = pl.debug_counters()
    h = [dc[31], dc[33], dc[34], dc[35], dc[36], dc[37]]
    if sum(h[:5]):  # diagnostics build (CLRRT_WALK_PROFILE): exact keys by their gap above the 11th key
        print(f"   exact keys per sample by key - kth at the drain: <=0 {h[0] / len(sub):.1f}, <=1e-3 "
              f"{h[1] / len(sub):.1f}, <=1e-2 {h[2] / len(sub):.1f}, <=0.1 {h[3] / len(sub):.1f}, >0.1 "
              f"{h[4] / len(sub):.1f} (list not full: {h[5] / len(sub):.1f})")
