"""Rollout cost per simulated step with and without the collision check (BATCH rounds, B = 16384)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes

for mode, obs in ((abi.CLRRT_COLLISION_STUB, None), (abi.CLRRT_COLLISION_OBB, scenes.urban_scene(200))):
    pl = clrrt.Planner(clrrt.default_params(collision_mode=mode), max_nodes=1 << 21, max_rows=1 << 27,
                       max_batch=16384)
    if obs is not None:
        pl.set_obstacles(obs)
    for persistent in (1, 0):
        pl.set_option("roll_persistent", persistent)
        pl.tree_init()
        pl.expand(clrrt.Rng(3), n_iters=16384 * 2, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        pl.enable_timing(True)
        pl.reset_counters()
        pl.expand(clrrt.Rng(4), n_iters=16384 * 6, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        ms, n = pl.kernel_time(1)
        w = pl.work_counters()
        print(f"mode {mode} persistent {persistent}: rollout {ms / n:.2f} ms/launch, {w['steps'] / n / 1e6:.2f} M steps/launch, "
              f"{ms * 1e6 / w['steps']:.2f} ns/step, scan {w['scan_points'] / w['steps']:.1f}/step, "
              f"box {w['box_tests'] / w['steps']:.1f}/step")
