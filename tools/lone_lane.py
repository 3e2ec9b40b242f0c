"""Straggler step latency: the longest first-candidate rollouts of a cfg3 round run (a) alone in k_rollout
(one lane per job, the plain step loop) and (b) as the only live sample of a k_roll_run round (clrrt_round_eval
with that one sample: its candidates take <= 10 lanes of one persistent wave, the short ones end and the long
one runs on alone), so the two step loops' single-lane latency can be compared.  Diagnostics build
(make -C cl-rrt_amd/csrc prof; CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so) for the wave clocks of (b)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

CLK = 2.4e6  # shader clocks per ms
ms = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
print(f"tree {pl.size()[0]} nodes")
smp = list(clrrt.Rng(77).draw_samples(pl.params, 4096))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
jobs = [(int(ids[s, 0]), 0, smp[s].x, smp[s].y) for s in range(len(smp)) if ids[s, 0] >= 0]
sidx = [s for s in range(len(smp)) if ids[s, 0] >= 0]
res = pl.simulate_batch(jobs)
nr = np.array([r["nrows"] for r in res])
order = np.argsort(-nr)[:4]
out = torch.empty((2 * 16, 160), dtype=torch.uint8, device="cuda")  # clrrt_node records
for i in order:
    job, s = jobs[i], sidx[i]
    # (a) k_rollout, one lane
    for rep in range(2):
        pl.enable_timing(True)
        r = pl.simulate_batch([job])
        a_ms, _ = pl.kernel_time(1)
    st = r[0]["nrows"] - 1
    # (b) k_roll_run, the sample alone in a round (rows of the round are not committed)
    for opt in (1, 0):
        pl.set_option("roll_coop", opt)
        for rep in range(2):
            pl.reset_counters()
            pl.enable_timing(True)
            pl.round_eval((abi.Sample * 1)(smp[s]), out.data_ptr())
            b_ms, nb = pl.kernel_time(1)
            d = pl.debug_counters()
        chain = max(1, d[50])
        print(f"job {i} (sample {s}, outcome {r[0]['outcome']}, {st} steps): k_rollout {a_ms:.3f} ms = "
              f"{a_ms * CLK / st:,.0f} clk/step | k_roll_run coop={opt}: {b_ms:.3f} ms ({nb} launches), longest wave "
              f"{d[49] / CLK:.3f} ms, chain {d[50]} -> {d[49] / chain:,.0f} clk/step; waves {d[51]}")
    pl.set_option("roll_coop", 1)
