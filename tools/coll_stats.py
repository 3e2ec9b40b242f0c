"""Wave-cooperative collision check statistics (diagnostics build: tools/variant.sh collstats -DCLRRT_COLL_STATS, run
with CLRRT_LIB pointing at it): cfg3 BATCH rounds, per wave-step of k_roll_run: lanes checked, candidate pairs
(grid-cell lists + moving obstacles), 64-pair windows, windows with a cull survivor, survivors (SAT tests)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=1000, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
pl.reset_counters()
st = pl.expand(clrrt.Rng(9), n_iters=0, budget_ms=500, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
d = pl.debug_counters()
ws, lanes, pairs, win, winv, surv = d[33:39]
print(f"tree {pl.size()[0]} nodes, {st['rounds']} rounds; rollout steps {d[0]}, box tests (reference count) {d[2]}")
print(f"per wave-step: lanes {lanes / ws:.1f}, pairs {pairs / ws:.1f}, windows {win / ws:.2f}, windows with a survivor "
      f"{winv / ws:.2f}, survivors {surv / ws:.1f}; per lane-step: pairs {pairs / lanes:.1f}, survivors {surv / lanes:.2f}")
