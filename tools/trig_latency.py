"""Latency of the rollout step's trig (glibc sincos + cos + sin + tan restatements) and of a plain FP64
multiply-add chain, one lane and 64 lanes, via clrrt_selftest_math fn 18 / 19 (diagnostics)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
import clrrt
pl = clrrt.Planner(clrrt.default_params(), max_nodes=4, max_rows=4, max_batch=1)
for fn, label, per in ((18, "trig step (sincos+cos+sin+tan)", 1), (19, "100 dependent FP64 FMA", 100)):
    for lanes in (1, 64, 4096):
        for iters in (10, 2010):
            a = np.full(lanes, 0.3) + np.arange(lanes) * 1e-6
            b = np.full(lanes, float(iters))
            for rep in range(3):
                t0 = time.perf_counter()
                pl.selftest_math(fn, a, b)
                dt = time.perf_counter() - t0
            if iters == 10:
                base = dt
        per_it = (dt - base) / 2000
        print(f"{label:34s} {lanes:5d} lanes: {per_it * 1e6:8.3f} us/iteration = {per_it * 2.4e9 / per:8.1f} clk per unit")
