"""Per-phase wave time of the rollout kernel (build: make -C cl-rrt_amd/csrc prof; run with
CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so): cfg3 scene, BATCH expansion for `ms`."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.enable_timing(True)
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
d = pl.debug_counters()
names = ["loop / abandon", "waypoint (cos, sin, scan)", "lateral error + control + ODE", "sincos + tan",
         "collision", "costs / end checks + row store", "refill", "batched finish + goal-bias init"]
ph = d[32:40]
tot = sum(ph)
print(f"nodes {pl.size()[0]} rounds {st['rounds']} steps {d[0]} rollout ms {pl.kernel_time(1)} nn ms {pl.kernel_time(0)}")
for nm, v in zip(names, ph):
    print(f"  {nm:32s} {v / max(1, tot) * 100:5.1f}%  {v / max(1, d[0]):8.1f} clk/step")
print(f"scan: {d[30] / max(1, d[0]):.2f} points per lane-step, wave-level iterations {d[31]:,} "
      f"({d[31] * 64 / max(1, d[30]):.1f}x the lane average)")
print(f"active lanes per wave step {d[28] / max(1, d[29]):.1f}; wave steps {d[29]:,}, "
      f"{d[29] / max(1, d[27]):.0f} per wave")
print(f"waves {d[27]:,}: mean lifetime {d[24] / max(1, d[27]):,.0f} clk, max {d[25]:,} clk; busiest lane {d[26]} steps "
      f"(max over all launches)")
# one more round on the grown tree, alone: its rollout launch against its longest wave and busiest lane
for opt in (1, 0):
    pl.set_option("roll_coop", opt)
    pl.reset_counters()
    pl.enable_timing(True)
    pl.expand(clrrt.Rng(9), n_iters=16384, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
    d = pl.debug_counters()
    rms, rn = pl.kernel_time(1)
    ph = d[32:40]
    tot = sum(ph)
    print(f"single round (roll_coop={opt}): rollout launches {rn}, {rms:.3f} ms; longest wave {d[25] / 2.4e6:.3f} ms "
          f"({d[25]:,} clk), busiest lane {d[26]} steps -> {d[25] / max(1, d[26]):,.0f} clk per its step; "
          f"mean wave life {d[24] / max(1, d[27]) / 2.4e6:.3f} ms; active lanes per wave step {d[28] / max(1, d[29]):.1f}")
    for nm, v in zip(names, ph):
        print(f"  {nm:32s} {v / max(1, tot) * 100:5.1f}%  {v / max(1, d[0]):8.1f} clk/step")
