"""Nearest-node search of one 16384-sample cfg3 round on the trees one rank sees in multi-GPU weak scaling
(the replicated tree grows N times faster with N ranks: ~2 M nodes per 2 s query at N = 1, ~16 M at N = 8).
Grows the cfg3 scene by BATCH expansion and, at each target size (millions of nodes, argv[1:]), times the
walk search of a fresh 16384-sample round (explore and optimize samples mixed as drawn, then each kind
alone) and reports its tiles, exact keys and overflow records per sample.  With CLRRT_WALK_PHASES=1 and the
diagnostics build (CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so) also the walk's per-phase shader clocks."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import torch  # noqa: E402,F401
import clrrt  # noqa: E402
from clrrt import abi, scenes  # noqa: E402

targets = [float(x) for x in sys.argv[1:]] or [4.7, 8.0, 16.0]
phases = os.environ.get("CLRRT_WALK_PHASES") == "1"
cap = int(max(targets) * 1e6) + (1 << 20)
pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), max_nodes=cap,
                   max_rows=min(1 << 31, cap * 72), max_batch=16384)
pl.set_obstacles(scenes.urban_scene(200))
pl.tree_init()
for kv in os.environ.get("CLRRT_OPTS", "").split(","):
    if kv:
        k, v = kv.split("=")
        pl.set_option(k, int(v))
rng = clrrt.Rng(5)
smp = clrrt.Rng(77).draw_samples(pl.params, 16384)
kinds = (("mixed", list(smp)), ("explore", [s for s in smp if s.explore]), ("optimize", [s for s in smp if not s.explore]))
t_grow = time.perf_counter()


def timed(sub):
    pl.sort_nodes_batch(sub, exact=False)  # warm: index built for this tree
    best = 1e9
    for _ in range(3):
        pl.reset_counters()  # the counters below are those of the last repetition
        t0 = time.perf_counter()
        pl.sort_nodes_batch(sub, exact=False)
        best = min(best, time.perf_counter() - t0)
    return best


for tgt in targets:
    while pl.size()[0] < tgt * 1e6:  # fixed-count rounds: the same tree on every build (A/B runs compare)
        st = pl.expand(rng, n_iters=16 * 16384, mode=clrrt.CLRRT_MODE_BATCH, batch=16384)
        if st["capacity_stop"]:
            break
    n = pl.size()[0]
    print(f"{n / 1e6:6.2f} M nodes (grown in {time.perf_counter() - t_grow:5.1f} s)", flush=True)
    ab = [x for x in os.environ.get("CLRRT_OPTS_AB", "").split(";") if x]  # option sets timed one after another
    for kv in ab:
        for o in kv.split(","):
            k, v = o.split("=")
            pl.set_option(k, int(v))
        best = timed(kinds[0][1])
        w = pl.search_work()
        print(f"   [{kv}] mixed: {best * 1e3:7.2f} ms; tiles/sample {w['tiles'] / max(1, w['samples']):.0f}, exact keys/sample "
              f"{w['exact_keys'] / max(1, w['samples']):.0f}, overflow records {pl.debug_counters()[32]}", flush=True)
    for lab, sub in kinds:
        if phases:
            pl.set_option("nn_debug", 0)
        best = timed(sub)
        w = pl.search_work()
        dc = pl.debug_counters()
        ns = max(1, w["samples"])
        q = pl.nn_stats()
        line = (f"   {lab:8s} {len(sub):5d} samples: {best * 1e3:7.2f} ms; tiles/sample {w['tiles'] / ns:.0f}, "
                f"exact keys/sample {w['exact_keys'] / ns:.0f}, overflow records/round {dc[32]:.0f}; per sample: "
                f"super visits {q['walk_supers'] / len(sub):.0f}, prefilter passes {q['walk_queued'] / len(sub):.0f}")
        if phases:
            pl.set_option("nn_debug", 2)
            pl.reset_counters()
            pl.sort_nodes_batch(sub, exact=False)
            s = pl.nn_stats()
            tot = max(1, s["walk_clk_total"])
            line += (f"; clk/sample {tot / len(sub) / 1e3:.0f} k: bounds {s['walk_clk_bounds'] / tot:.0%}, supers "
                     f"{s['walk_clk_super'] / tot:.0%} (visits {s['walk_clk_visit'] / tot:.0%}, drains "
                     f"{s['walk_clk_drain'] / tot:.0%})")
            pl.set_option("nn_debug", 0)
        print(line, flush=True)
