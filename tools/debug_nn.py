import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "cl-rrt_amd")
import torch
torch.cuda.init(); print("torch devices", torch.cuda.device_count(), flush=True)
x = torch.ones(4, device="cuda"); print("torch ok", float(x.sum()), flush=True)
import numpy as np
import clrrt
from clrrt import abi
from oracle_binding import Oracle
o = Oracle(abi.default_params()); Oracle.srand(4); o.init_tree(); o.expand(150)
pl = clrrt.Planner(clrrt.default_params(), max_nodes=1<<16, max_rows=1<<20, max_batch=2048)
pl.tree_load(o.nodes_raw())
smp = list(clrrt.Rng(21).draw_samples(pl.params, 400))
ids, keys = pl.sort_nodes_batch(smp)
y = torch.ones(4, device="cuda"); print("torch after clrrt ok", float(y.sum()), flush=True)
shown = 0
for j, s in enumerate(smp):
    cid, ckey = o.sort_nodes(s.x, s.y, s.explore)
    gid = [int(i) for i in ids[j] if i >= 0]
    if gid != cid and shown < 6:
        shown += 1
        print("sample", j, s.x, s.y, "explore", s.explore)
        print("  cpu", cid, [f"{k:.7g}" for k in ckey])
        print("  gpu", gid, [f"{k:.7g}" for k in keys[j][:len(gid)]])
        for nid in set(cid) ^ set(gid):
            print("   node", nid, "dubins cpu", o.dubins(s.x, s.y, nid))
