"""Find the first row/column where a GPU rollout departs from the oracle's (bitwise)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "cl-rrt_amd")
import numpy as np
import clrrt
from clrrt import abi
from oracle_binding import Oracle

o = Oracle(abi.default_params()); Oracle.srand(1); o.init_tree()
o.expand(104)
n0 = o.size()
pre = o.nodes_raw()
ref = clrrt.Rng(1)
for _ in range(3 * 104): ref.next()
s = ref.draw_samples(clrrt.default_params(), 1)[0]
o.expand(1)
alln = o.nodes_raw()
pl = clrrt.Planner(clrrt.default_params(), max_nodes=1 << 12, max_rows=1 << 18, max_batch=8)
def first_diff(g, c, label):
    n = min(len(g), len(c))
    d = (g[:n].view(np.uint64) != c[:n].view(np.uint64))
    if d.any():
        r, col = np.argwhere(d)[0]
        print(f"{label}: first bit difference at row {r} col {col}: gpu {g[r,col]!r} cpu {c[r,col]!r}; rows g {len(g)} c {len(c)}")
        print("   gpu row", list(g[r])); print("   cpu row", list(c[r]))
        if r > 0: print("   prev row equal:", np.array_equal(g[r-1], c[r-1]))
    else:
        print(f"{label}: identical ({n} rows)")
pl.tree_load(pre)
for c in (49, 99):
    g = pl.simulate_batch([(c, 0, s.x, s.y)], rows=True)[0]
    oo = Oracle(abi.default_params()); oo.load_tree(pre)
    cr = oo.simulate(c, 0, s.x, s.y, rows=True)
    first_diff(g["rows"], cr["rows"], f"regular from {c}")
# goal-biased from the new node n0
arr = (abi.Node * (n0 + 1))(*alln[:n0 + 1])
pl.tree_load(arr)
g = pl.simulate_batch([(n0, 1, 0.0, 0.0)], rows=True)[0]
oo = Oracle(abi.default_params()); oo.load_tree(arr)
cr = oo.simulate(n0, 1, rows=True)
first_diff(g["rows"], cr["rows"], f"goal-biased from {n0}")
print("ref_n", g["ref_n"], cr["ref_n"], "ref_back", g["ref_back"], cr["ref_back"], "vback", g["ref_vback"], cr["ref_vback"])
