"""Dump a bench-sized tree (cfg3 scene, BATCH expansion for `ms`) plus one sample batch and its
candidate lists to gpurun_out/nn_tree.npz for offline analysis of nearest-node pruning."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes

ms = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
obs = scenes.urban_scene(200)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=4 << 20,
                   max_rows=1 << 26, max_batch=16384)
pl.set_obstacles(obs)
pl.tree_init()
pl.expand(clrrt.Rng(5), n_iters=0, budget_ms=ms, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
n = pl.nodes()
smp = list(clrrt.Rng(77).draw_samples(pl.params, 16384))
ids, keys = pl.sort_nodes_batch(smp, exact=False)
xy, ex = clrrt.samples_to_numpy(smp)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/nn_tree.npz", state=n["state"][:, :3], ref_back=n["ref_back"],
                    ang_par=n["ang_par"], costE=n["costE"], parent=n["parent"], sxy=xy, ex=ex, ids=ids,
                    keys=keys, feas_len=np.array([2.1 * pl.params.ref_res if hasattr(pl.params, "ref_res") else 0.42]))
print("nodes", len(n["parent"]))
