"""Round time of cfg3 BATCH rounds (B = 16384, 200 obstacles) against tree size, for several widths of
the persistent rollout grid (option roll_blocks): the tree grows in chunks of 16 pipelined rounds and
each chunk's wall time is recorded (the pipeline drains at chunk ends, same for every width).
Prints ms per round by tree-size bucket; decides how the grid should split the GPU between the
rollouts and the side stream's nearest-node search as the tree grows."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

B = 16384
CHUNK = 16
widths = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "96,128,160,192")]
buckets = [0, 300_000, 700_000, 1_100_000, 1_500_000, 1_900_000, 2_400_000]
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=6 << 20,
                   max_rows=400 << 20, max_batch=B)
pl.set_obstacles(scenes.urban_scene(200))
table = {}
for w in widths:
    pl.set_option("roll_blocks", w)
    pl.tree_init()
    rng = clrrt.Rng(1)
    pl.expand(rng, n_iters=2 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)  # warm-up
    pl.tree_init()
    rng = clrrt.Rng(1)
    acc = {}
    while True:
        n0 = pl.size()[0]
        if n0 >= buckets[-1]:
            break
        t0 = time.perf_counter()
        pl.expand(rng, n_iters=CHUNK * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        dt = (time.perf_counter() - t0) * 1e3 / CHUNK
        bi = max(i for i in range(len(buckets) - 1) if buckets[i] <= n0)
        acc.setdefault(bi, []).append(dt)
    table[w] = {k: sum(v) / len(v) for k, v in acc.items()}
    print(f"roll_blocks {w}: " + ", ".join(f"{buckets[k] // 1000}k+: {v:.2f} ms" for k, v in sorted(table[w].items())),
          flush=True)
