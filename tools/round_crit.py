"""Critical path between consecutive rollout kernels of a pipelined BATCH run (rocprofv3 --kernel-trace CSV):
for every gap, the kernels that end inside it, the last one (what the next round waited for) and how long the
walk search of later rounds (k_walk_search, side streams) ran relative to the rollout kernel.  Prints totals
per quarter of each query.  Usage: python tools/round_crit.py <kernel_trace.csv>"""
import csv
import sys
from collections import Counter, defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:48])
            for r in rows)
roll = [(s, e) for s, e, n in ev if "k_roll_run" in n]
# queries: separated by gaps > 20 ms between rollout kernels
queries, cur = [], [roll[0]]
for a, b in zip(roll, roll[1:]):
    if b[0] - a[1] > 20e6:
        queries.append(cur)
        cur = []
    cur.append(b)
queries.append(cur)
print(f"{len(roll)} rollout kernels in {len(queries)} queries")
for qi, q in enumerate(queries):
    n = len(q)
    stats = [defaultdict(float) for _ in range(4)]
    last = [Counter() for _ in range(4)]
    for i, ((s0, e0), (s1, e1)) in enumerate(zip(q, q[1:])):
        k = min(3, 4 * i // max(1, n - 1))
        st = stats[k]
        st["rounds"] += 1
        st["roll_ms"] += (e0 - s0) / 1e6
        st["gap_ms"] += (s1 - e0) / 1e6
        ends = [(e, nm) for s, e, nm in ev if e0 < e <= s1 and "k_roll_run" not in nm]
        if ends:
            last[k][max(ends)[1]] += 1
        walks = [(s, e) for s, e, nm in ev if "k_walk_search" in nm and s < s1 and e > s0]
        if walks:
            st["walk_end_after_roll_ms"] += max(0, max(e for _, e in walks) - e0) / 1e6
            st["walk_busy_ms"] += sum(min(e, s1) - max(s, s0) for s, e in walks) / 1e6
    for k in range(4):
        st = stats[k]
        r = max(1, st["rounds"])
        print(f"query {qi} quarter {k}: {int(st['rounds'])} rounds, rollout {st['roll_ms'] / r:.2f} ms, gap {st['gap_ms'] / r:.2f} ms, "
              f"walk ends {st['walk_end_after_roll_ms'] / r:.2f} ms after the rollout kernel; last to end in the gap: "
              f"{', '.join(f'{nm} {c}' for nm, c in last[k].most_common(3))}")
