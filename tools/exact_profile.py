"""EXACT mode (the reference's sequential expandTree tree, speculated in rounds) on cfg3's scene:
rounds, iterations committed per round, speculated samples, wall time per round and the device time
per kernel class.  Usage: python tools/exact_profile.py [budget_ms] [batch]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: F401  (one HIP runtime)
import clrrt
from clrrt import abi, scenes

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
widths = [int(w) for w in sys.argv[3].split(",")] if len(sys.argv) > 3 else [8]
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                   max_rows=1 << 25, max_batch=max(batch, 256))
pl.set_obstacles(scenes.urban_scene(200))
for label in ["warm-up"] + [f"min width {w}" for w in widths]:
    if label != "warm-up":
        pl.set_option("exact_min_width", int(label.split()[-1]))
    pl.tree_init()
    pl.reset_counters()
    pl.enable_timing(True)
    t0 = time.perf_counter()
    st = pl.expand(clrrt.Rng(1), n_iters=0, budget_ms=budget, mode=clrrt.CLRRT_MODE_EXACT, batch=batch)
    wall = (time.perf_counter() - t0) * 1e3
    r = max(1, st["rounds"])
    ks = {k: pl.kernel_time(i) for i, k in enumerate(("nn", "rollout", "commit"))}
    print(f"{label}: {st['nodes_added']} nodes in {wall:.0f} ms = {st['nodes_added'] / wall * 1e3:.0f} nodes/s; "
          f"{st['iterations']} iterations in {st['rounds']} rounds ({st['iterations'] / r:.1f} per round, "
          f"{st['speculated'] / r:.1f} speculated); {wall / r:.2f} ms per round; device ms per round: "
          + ", ".join(f"{k} {v[0] / r:.2f} ({v[1] / r:.1f} launches)" for k, v in ks.items()))
