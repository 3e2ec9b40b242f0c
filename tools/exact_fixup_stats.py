"""EXACT rounds on the cfg3 scene (200 obstacles), one 2 s query from a fresh tree, with and without fix-ups
(option exact_fixup): nodes/s, rounds, committed samples per round and why the rounds' prefixes ended
(clrrt_exact_stats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: E402,F401
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
sets = ({"exact_fixup": 0}, {"exact_fixup": 1}, {"exact_fixup": 1, "exact_fixup_cap": 48},
        {"exact_fixup": 1, "exact_fixup_cap": 96}, {"exact_fixup": 1, "exact_fixup_cap": 160},
        {"exact_fixup": 1, "exact_fixup_cap": 96, "exact_min_width": 16})
if len(sys.argv) > 2 and sys.argv[2] == "default":  # (kernel traces: the default settings only; k=v options after)
    sets = ({"exact_fixup": 1, **{kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[3:]}},)
for opts in sets:
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                       max_rows=1 << 26, max_batch=16384)
    pl.set_obstacles(scenes.urban_scene(200))
    for k, v in opts.items():
        pl.set_option(k, v)
    for q in range(2):  # warm-up query, then the measured one
        pl.tree_init()
        st = pl.expand(clrrt.Rng(1 + q), n_iters=0, budget_ms=ms if q else 200.0, mode=clrrt.CLRRT_MODE_EXACT,
                       batch=16384)
    x = pl.exact_stats()
    print(f"{opts}: {st['nodes_added'] / (st['elapsed_ms'] * 1e-3):7.0f} nodes/s, {st['iterations']} iterations in "
          f"{st['rounds']} rounds ({st['iterations'] / st['rounds']:.2f} per round, {st['speculated'] / st['rounds']:.1f} "
          f"speculated), {st['elapsed_ms'] / st['rounds']:.2f} ms per round; stats (both queries) {x}", flush=True)
    pl.close()
