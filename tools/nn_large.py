"""Nearest-node search of one 16384-sample cfg3 round on the trees one rank sees in multi-GPU weak scaling
(the replicated tree grows N times faster with N ranks: ~2 M nodes per 2 s query at N = 1, ~16 M at N = 8).
Grows the cfg3 scene by BATCH expansion and, at each target size (millions of nodes, argv[1:]), times the
walk search of a fresh 16384-sample round (explore and optimize samples mixed as drawn) and reports its
tiles and exact keys per sample."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: E402,F401
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

targets = [float(x) for x in sys.argv[1:]] or [4.7, 8.0, 16.0]
cap = int(max(targets) * 1e6) + (1 << 20)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=cap,
                   max_rows=min(1 << 31, cap * 72), max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
rng = clrrt.Rng(5)
smp = clrrt.Rng(77).draw_samples(pl.params, 16384)
t_grow = time.perf_counter()
for tgt in targets:
    while pl.size()[0] < tgt * 1e6:
        st = pl.expand(rng, n_iters=0, budget_ms=1000.0, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        if st["capacity_stop"]:
            break
    n = pl.size()[0]
    pl.sort_nodes_batch(smp, exact=False)  # warm: index built for this tree
    best = 1e9
    for _ in range(3):
        pl.reset_counters()
        t0 = time.perf_counter()
        pl.sort_nodes_batch(smp, exact=False)
        best = min(best, time.perf_counter() - t0)
    w = pl.search_work()
    print(f"{n / 1e6:6.2f} M nodes (grown in {time.perf_counter() - t_grow:5.1f} s): 16384-sample search "
          f"{best * 1e3:7.2f} ms ({best * 1e3 / 16.384:.3f} us/sample); tiles/sample "
          f"{w['tiles'] / max(1, w['samples']):.0f}, exact keys/sample {w['exact_keys'] / max(1, w['samples']):.0f}",
          flush=True)
