"""Rollout kernel timeline in bench conditions (build: make -C cl-rrt_amd/csrc prof; run with
CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so): cfg3 scene grown by BATCH expansion for `ms`, then single rounds
(no search beside them) with the wave-cooperative collision checks on and off: the rollout launch, its
longest wave, the longest chain (a regular rollout + its goal-biased follow-up), when the waves found the
job queue empty, and the busiest lane's steps after that (the tail)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0
CLK = 2.4e6  # shader clocks per ms
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.enable_timing(True)
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
print(f"grown: nodes {pl.size()[0]} rounds {st['rounds']} rollout ms {pl.kernel_time(1)} nn ms {pl.kernel_time(0)}")


def report(label, d, rms, rn):
    w = max(1, d[51])
    print(f"{label}: rollout launches {rn}, {rms / max(1, rn):.3f} ms each; longest wave {d[49] / CLK:.3f} ms, mean wave "
          f"{d[48] / w / CLK:.3f} ms over {d[51]} waves; longest chain {d[50]} steps -> {d[49] / max(1, d[50]):,.0f} "
          f"clk per step of the longest wave; queue empty after {d[52] / w / CLK:.3f} ms (mean), {d[53] / CLK:.3f} ms (max); "
          f"busiest lane's tail {d[54]} steps (mean over waves {d[55] / w:.0f})")
    names = ["loop top", "waypoint scan", "lateral error + control + ODE", "sincos + tan + cos/sin", "collision",
             "costs / end checks + row store", "refill / abandon check", "batched finish + goal-bias init"]
    ph = d[40:48]
    tot = max(1, sum(ph))
    for nm, v in zip(names, ph):
        print(f"    {nm:32s} {v / tot * 100:5.1f}%")


for opt in (1, 0):
    pl.set_option("roll_coop", opt)
    pl.reset_counters()
    pl.enable_timing(True)
    pl.expand(clrrt.Rng(9), n_iters=16384, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
    d = pl.debug_counters()
    rms, rn = pl.kernel_time(1)
    report(f"single round (roll_coop={opt})", d, rms, rn)
# a sparse round: 64 samples (<= 640 jobs over the persistent waves, ~2 per wave): the longest chain runs
# with almost no other lane in its wave
for nb in (64, 1024):
    pl.reset_counters()
    pl.enable_timing(True)
    pl.expand(clrrt.Rng(13), n_iters=nb, mode=clrrt.CLRRT_MODE_BATCH, batch=nb)
    d = pl.debug_counters()
    rms, rn = pl.kernel_time(1)
    report(f"sparse round ({nb} samples)", d, rms, rn)
# pipelined rounds (the bench's): the same statistics over 0.5 s
pl.set_option("roll_coop", 1)
pl.reset_counters()
pl.enable_timing(True)
st = pl.expand(clrrt.Rng(11), n_iters=0, budget_ms=500, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
d = pl.debug_counters()
rms, rn = pl.kernel_time(1)
report(f"pipelined rounds ({st['rounds']})", d, rms, rn)
