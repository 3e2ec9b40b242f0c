"""Rollout lane utilisation split by phase (verdict r05 item 3; diagnostics build with -DCLRRT_LANE_STATS, run with
CLRRT_LIB=cl-rrt_amd/var_lane/libclrrt.so): cfg3 BATCH rounds (B = 16384, defer_steps 128, the lag-2 pipeline of a 2 s
query); per wave-step of k_roll_run, the lanes that step while the job queue still has jobs and after the wave found
it empty (the tail), and the share of wave-steps with at most 8 lanes stepping.  Early (first second of a query) and
late (a tree past 2 M nodes) rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

B = 16384
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=6 << 20,
                   max_rows=(6 << 20) * 64, max_batch=B)
pl.set_obstacles(scenes.urban_scene(200))
pl.set_option("defer_steps", 128)
pl.tree_init()
rng = clrrt.Rng(5)


def report(label, st):
    d = pl.debug_counters()
    w0, l0, s0, w1, l1, s1 = d[33:39]
    tot_w = max(1, w0 + w1)
    print(f"{label}: {st['rounds']} rounds, tree {pl.size()[0]} nodes; wave-steps: queue non-empty {w0} "
          f"({w0 / tot_w:.0%}), {l0 / max(1, w0):.1f} lanes, <= 8 lanes {s0 / max(1, w0):.0%}; tail {w1} ({w1 / tot_w:.0%}), "
          f"{l1 / max(1, w1):.1f} lanes, <= 8 lanes {s1 / max(1, w1):.0%}; all {(l0 + l1) / tot_w:.1f} lanes "
          f"(utilisation {(l0 + l1) / tot_w / 64:.2f}); lane-steps in the tail {l1 / max(1, l0 + l1):.0%}", flush=True)


pl.reset_counters()
st = pl.expand(rng, n_iters=0, budget_ms=1000.0, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
report("first second of a query", st)
while pl.size()[0] < 2_000_000:
    pl.expand(rng, n_iters=16 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
pl.reset_counters()
st = pl.expand(rng, n_iters=0, budget_ms=500.0, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
report("late rounds (tree past 2 M nodes)", st)
