"""Where the walk's exact keys fall (diagnostics build, CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so, option nn_debug 2): each
exact key computed by a walk wave, by its distance above the sample's 11th key at the moment it is computed (<= 0: it
enters the list; (0, 1e-3]: within the stage-1 bracket's margin, a tighter bracket could not drop it; larger gaps: the
bound that queued it was loose, or the 11th key shrank later).  One 16384-sample cfg3 round per kind (explore / optimize)
on a grown tree of argv[1] million nodes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

tgt = float(sys.argv[1]) if len(sys.argv) > 1 else 2.4
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=int(tgt * 1e6) + (1 << 20),
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
rng = clrrt.Rng(5)
while pl.size()[0] < tgt * 1e6:
    pl.expand(rng, n_iters=0, budget_ms=1000.0, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
print(f"{pl.size()[0] / 1e6:.2f} M nodes", flush=True)
for lab, sub in (("explore", [s for s in smp if s.explore]), ("optimize", [s for s in smp if not s.explore])):
    pl.set_option("nn_debug", 2)
    pl.reset_counters()
    pl.sort_nodes_batch(sub, exact=False)
    d = pl.debug_counters()
    pl.set_option("nn_debug", 0)
    h = [d[31], d[33], d[34], d[35], d[36], d[37]]
    tot = max(1, sum(h[:5]))
    print(f"{lab:8s} {len(sub):5d} samples: exact keys/sample {tot / len(sub):.0f}; gap to the 11th key <= 0 {h[0] / tot:.1%}, "
          f"(0, 1e-3] {h[1] / tot:.1%}, (1e-3, 1e-2] {h[2] / tot:.1%}, (1e-2, 0.1] {h[3] / tot:.1%}, > 0.1 {h[4] / tot:.1%}; "
          f"11th key still inf {h[5] / tot:.1%}", flush=True)
