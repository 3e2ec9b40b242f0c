"""Serial time between consecutive rollout kernels (k_roll_run) of a pipelined BATCH run, from a
rocprofv3 --kernel-trace CSV: per gap, the kernels that ran in it (any stream), their summed busy time
and the idle time, aggregated over all gaps; and the mean gap per quarter of each query (queries are
separated by gaps > 5 ms).  Usage: python tools/round_gaps.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
roll = [(s, e) for s, e, n in ev if "k_roll_run" in n]
print(f"{len(roll)} rollout kernels, mean {sum(e - s for s, e in roll) / max(1, len(roll)) / 1e3:.1f} us")
gaps, per = [], defaultdict(float)
for (s0, e0), (s1, e1) in zip(roll, roll[1:]):
    g = s1 - e0
    if g <= 0 or g > 5e6:  # overlapping or a query boundary
        continue
    gaps.append(g)
    for s, e, n in ev:
        if e <= e0 or s >= s1:
            continue
        per[n.split("(")[0][:60]] += (min(e, s1) - max(s, e0)) / 1e3
ng = max(1, len(gaps))
print(f"{len(gaps)} gaps, mean {sum(gaps) / ng / 1e3:.1f} us, median {sorted(gaps)[len(gaps) // 2] / 1e3:.1f} us")
busy = 0.0
for n, t in sorted(per.items(), key=lambda x: -x[1])[:25]:
    print(f"  {n:60s} {t / ng:8.1f} us per gap")
    busy += t
print(f"  kernel time inside gaps {busy / ng:.1f} us per gap (streams overlap, so this can exceed the gap)")
# mean gap by query quarter (the search grows with the tree through a query)
queries, cur = [], []
for (s0, e0), (s1, e1) in zip(roll, roll[1:]):
    g = s1 - e0
    if g > 5e6:
        if cur:
            queries.append(cur)
        cur = []
    elif g > 0:
        cur.append(g)
if cur:
    queries.append(cur)
for qi, q in enumerate(queries):
    n = len(q)
    if n < 8:
        continue
    qs = [q[i * n // 4:(i + 1) * n // 4] for i in range(4)]
    print(f"query {qi}: {n} gaps, mean by quarter " + ", ".join(f"{sum(x) / len(x) / 1e3:.0f} us" for x in qs))
