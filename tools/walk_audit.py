"""How tight the walk's tile bounds are, from a measured bound (verdict r05 item 2): on cfg3 trees grown to argv[1:]
million nodes, for the explore and optimize samples of a 16384-sample round (a subset of argv SUB each), compares

  visited   tiles the walk search actually visits per sample (clrrt_search_work, overflow split included),
  admiss.   tiles whose bound (the walk's own walk_lb, max'ed with the super-tile's) is <= the sample's TRUE 11th
            key kth -- every search over these bounds visits at least these, whatever its pass order,
  useful    admissible tiles that hold a list member (a feasible record whose (key, id) does not follow the 11th
            entry's): what a perfect per-tile bound would visit,

and the exact keys: computed by the walk, needed (feasible records with key <= kth), and what stage 1 would let
through if kth were known from the start (clrrt_walk_audit, a brute-force diagnostic).  visited / admissible is the
cost of the pass order (the 11th key shrinks while tiles are visited); admissible / useful is the looseness of the
bounds.  Usage: python tools/walk_audit.py 1.1 2.8 16   (env SUB: samples per kind, default 2048)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: E402,F401
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

targets = [float(x) for x in sys.argv[1:]] or [1.1, 2.8]
SUB = int(os.environ.get("SUB", "2048"))
cap = int(max(targets) * 1e6) + (1 << 20)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=cap,
                   max_rows=min(1 << 31, cap * 72), max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
rng = clrrt.Rng(5)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
kinds = (("explore", [s for s in smp if s.explore][:SUB]), ("optimize", [s for s in smp if not s.explore][:SUB]))


def q(a, p):
    return float(np.percentile(a, p)) if len(a) else 0.0


for tgt in targets:
    while pl.size()[0] < tgt * 1e6:  # fixed-count rounds: the same tree on every build
        st = pl.expand(rng, n_iters=16 * 16384, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        if st["capacity_stop"]:
            break
    n = pl.size()[0]
    print(f"{n / 1e6:6.2f} M nodes, {-(-n // 32)} tiles", flush=True)
    for lab, sub in kinds:
        pl.reset_counters()
        pl.sort_nodes_batch(sub, exact=False)
        w = pl.search_work()
        ns = max(1, w["samples"])
        a = pl.walk_audit(sub)
        adm, use, le, s1, sup, rec = a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], a[:, 7]
        inf, far, head, usele = a[:, 8], a[:, 9], a[:, 10], a[:, 11]
        print(f"  {lab:8s} {len(sub)} samples: tiles visited {w['tiles'] / ns:7.0f} | admissible mean {adm.mean():7.0f} "
              f"(p50 {q(adm, 50):.0f}, p90 {q(adm, 90):.0f}) | useful mean {use.mean():5.1f} (p50 {q(use, 50):.0f}, "
              f"p90 {q(use, 90):.0f}); visited/admissible {w['tiles'] / ns / max(1e-9, adm.mean()):.2f}, "
              f"admissible/useful {adm.mean() / max(1e-9, use.mean()):.1f}", flush=True)
        print(f"  {'':8s} exact keys computed {w['exact_keys'] / ns:7.0f} | needed (key <= kth) {le.mean():6.1f} | "
              f"stage 1 at the final kth {s1.mean():7.0f} of {rec.mean():7.0f} records in admissible tiles; "
              f"admissible super-tiles {sup.mean():.0f} of {-(-n // 1024)}", flush=True)
        r = max(1e-9, rec.mean())
        print(f"  {'':8s} records of admissible tiles that are no member: infeasible {inf.mean() / r:.1%}, feasible but "
              f"farther than kth {far.mean() / r:.1%}, within kth but key > kth (heading) {head.mean() / r:.1%}; "
              f"admissible tiles holding a key <= kth (ties included) {usele.mean():.1f}", flush=True)
        kth = a[:, 6].copy().view(np.float32)
        na = np.maximum(1, adm)
        print(f"  {'':8s} kth p10 {q(kth, 10):.2f} p50 {q(kth, 50):.2f} p90 {q(kth, 90):.2f}; admissible tiles: the sample "
              f"inside their ref.back() disc {(a[:, 12] / na).mean():.1%}, mean radius position {(a[:, 13] / na).mean() / 1e3:.2f} m "
              f"ref.back() {(a[:, 14] / na).mean() / 1e3:.2f} m, unbounded arc {(a[:, 15] / na).mean():.1%}; tiles inside one "
              f"run of equal records {a[:, 16].mean():.0f}, records in runs {a[:, 17].mean() / r:.1%}", flush=True)
