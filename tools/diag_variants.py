"""Time one 6-round cfg3 BATCH expansion per option variant (diagnostics; prints as it goes)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
from clrrt import abi, scenes
obs = scenes.urban_scene(200)
variants = [dict(nn_pipeline=0), dict(nn_pipeline=1), dict(nn_lag=1), dict(nn_lag=2), dict(nn_lag=2, stream_prio=0),
            dict(roll_priority=0, roll_blocks=512), dict(roll_coop=0), dict(rows_deferred=0), dict(nn_walk_double=0),
            dict(defer_steps=64), dict(defer_steps=64, nn_lag=2)]
sel = sys.argv[1:] 
for i, opts in enumerate(variants):
    if sel and str(i) not in sel:
        continue
    t0 = time.time()
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=1 << 20,
                       max_rows=1 << 26, max_batch=16384)
    for k, v in opts.items():
        pl.set_option(k, v)
    pl.set_obstacles(obs)
    pl.tree_init()
    print(f"{i} {opts}: setup {time.time() - t0:.2f} s", flush=True)
    for r in range(6):
        t1 = time.time()
        st = pl.expand(clrrt.Rng(12 + r), n_iters=16384, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        print(f"   round {r}: {time.time() - t1:.3f} s nodes {pl.size()[0]} deferred {st['deferred']}", flush=True)
    pl.close()
