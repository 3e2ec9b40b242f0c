"""Grow a bench-like BATCH tree on the GPU and save its node records (gpurun_out/tree_<ms>.bin)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa
import clrrt
from clrrt import abi, scenes
ms = float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0
obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 28, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
st = pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
raw = pl.nodes_raw()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", f"tree_{int(ms)}.bin"), "wb").write(bytes(raw))
print("nodes", len(raw), st)
