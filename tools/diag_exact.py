"""Per-iteration diagnosis of EXACT-mode divergence: for each iteration of a sequential oracle run,
load the oracle's tree as it was before the iteration, run that single iteration on the GPU in EXACT
mode, and compare the appended nodes; on a mismatch print the candidate lists and rollouts."""
import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "cl-rrt_amd")
import numpy as np
import clrrt
from clrrt import abi, scenes
from oracle_binding import Oracle

kind, seed, iters = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
mode = abi.CLRRT_COLLISION_OBB if kind != "empty" else abi.CLRRT_COLLISION_STUB
obs = scenes.urban_scene(200) if kind != "empty" else None
o = Oracle(abi.default_params(collision_mode=mode), obs)
Oracle.srand(seed); o.init_tree()
sizes = [o.size()]
snap = [o.nodes_raw()]
xs = []
for it in range(iters):
    o.expand(1)
    sizes.append(o.size())
all_nodes = o.nodes_raw()
pl = clrrt.Planner(clrrt.default_params(collision_mode=mode), max_nodes=1 << 14, max_rows=1 << 20, max_batch=64)
if obs is not None:
    pl.set_obstacles(obs)
ref = clrrt.Rng(seed)
bad = 0
for it in range(iters):
    n0, n1 = sizes[it], sizes[it + 1]
    pre = (abi.Node * n0)(*all_nodes[:n0])
    pl.tree_load(pre)
    rng = clrrt.Rng(1); rng.state = abi.Rng.from_buffer_copy(bytes(ref.state))
    smp = ref.draw_samples(pl.params, 1)  # advances ref by one iteration
    pl.expand(rng, n_iters=1, mode=clrrt.CLRRT_MODE_EXACT, batch=1)
    g = pl.nodes()
    got = g["state"][n0:], g["parent"][n0:]
    exp = clrrt.nodes_to_numpy((abi.Node * (n1 - n0))(*all_nodes[n0:n1])) if n1 > n0 else None
    ok = (len(got[1]) == n1 - n0) and (n1 == n0 or (np.array_equal(got[1], exp["parent"]) and np.allclose(got[0], exp["state"], rtol=1e-12, atol=1e-12)))
    if not ok:
        bad += 1
        s = smp[0]
        print(f"iter {it}: sample ({s.x:.6f},{s.y:.6f}) explore {s.explore}; oracle appended {n1-n0} parents {list(exp['parent']) if exp else []}, gpu {len(got[1])} parents {list(got[1])}")
        oo = Oracle(abi.default_params(collision_mode=mode), obs); oo.load_tree(pre)
        cid, ck = oo.sort_nodes(s.x, s.y, s.explore)
        gid, gk = pl.sort_nodes_batch([s])
        print("   oracle cand", cid, [f"{k:.9g}" for k in ck])
        print("   gpu    cand", [int(i) for i in gid[0] if i >= 0], [f"{k:.9g}" for k in gk[0][:len(cid)]])
        jobs = [(c, 0, s.x, s.y) for c in cid]
        gr = pl.simulate_batch(jobs)
        for c, r in zip(cid, gr):
            orr = oo.simulate(c, 0, s.x, s.y)
            print(f"   cand {c}: oracle {orr['outcome']} {orr['nrows']}  gpu {r['outcome']} {r['nrows']}  dfinal {np.abs(r['final']-orr['final']).max():.3g}")
        if bad >= 4:
            break
print(f"{kind} seed {seed}: {iters} iterations, mismatching {bad}")
