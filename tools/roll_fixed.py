"""Fixed-workload (argv[1] = rN: N growth rounds) timing of one round's evaluation (nearest-node search + rollouts) on a cfg3 tree:
grow the tree for `ms`, then evaluate the same 16384 samples `reps` times without committing and
report the per-launch kernel times (for A/B builds: CLRRT_LIB=...)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch
import clrrt
from clrrt import abi, scenes

arg = sys.argv[1] if len(sys.argv) > 1 else "1000"
# "r40": grow for exactly 40 rounds (same tree for every build); otherwise a wall budget in ms
rounds = int(arg[1:]) if arg.startswith("r") else 0
ms = 1e9 if rounds else float(arg)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=8 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
st = pl.expand(clrrt.Rng(5), n_iters=rounds * 16384, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
print("grown:", st, flush=True)
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
arr = (abi.Sample * len(smp))(*smp)
out = torch.empty(2 * len(smp) * C_NODE if (C_NODE := 160) else 0, dtype=torch.uint8, device="cuda")
n = pl.round_eval(arr, out.data_ptr())
torch.cuda.synchronize()
pl.enable_timing(True)
pl.reset_counters()
for _ in range(reps):
    n = pl.round_eval(arr, out.data_ptr())
torch.cuda.synchronize()
nn_ms, k0 = pl.kernel_time(0)
ro_ms, k1 = pl.kernel_time(1)
w = pl.work_counters()
print(f"tree {pl.size()[0]} nodes; accepted {n}; nn {nn_ms / k0:.3f} ms/launch, rollout {ro_ms / k1:.3f} ms/launch, "
      f"steps/launch {w['steps'] / reps:.0f}")
