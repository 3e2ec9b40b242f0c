"""The main stream's timeline between consecutive rollout kernels of a pipelined BATCH run (rocprofv3 --kernel-trace
CSV, plain or .gz): for each gap, the kernels the rollout kernel's stream ran in it, in order, and the stream's idle
time before each (the stream waiting for the host or for an event of another stream).  Prints, over the rounds of
the last query (or of `--query k`), the median start offset / duration / preceding idle of each kernel position and
the share of the gap each kind of kernel holds.  Usage: python tools/round_timeline.py <kernel_trace.csv[.gz]>"""
import csv
import gzip
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
qsel = int(sys.argv[sys.argv.index("--query") + 1]) if "--query" in sys.argv else -1
f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = list(csv.DictReader(f))
ev = []
for r in rows:
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "rocprim" in nm:
        nm = "rocprim::" + nm.split("detail::")[-1].split("<")[1].split(",")[0].replace("rocprim::ROCPRIM_400200_NS::detail::", "")[:40] \
            if "<" in nm else nm
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm[:60], r["Stream_Id"], r["Queue_Id"]))
ev.sort()
roll = [e for e in ev if "k_roll_run" in e[2]]
main = roll[-1][3]
mev = [e for e in ev if e[3] == main]
# queries: separated by gaps > 20 ms between rollout kernels
queries, cur = [], [roll[0]]
for a, b in zip(roll, roll[1:]):
    if b[0] - a[1] > 20e6:
        queries.append(cur)
        cur = []
    cur.append(b)
queries.append(cur)
q = queries[qsel]
print(f"{len(roll)} rollout kernels in {len(queries)} queries; main stream {main}; query {qsel}: {len(q)} rounds")
pos = defaultdict(lambda: defaultdict(list))
share = defaultdict(float)
idle_tot, gap_tot, roll_tot, n = 0.0, 0.0, 0.0, 0
for (s0, e0, *_), (s1, e1, *_) in zip(q, q[1:]):
    ks = [e for e in mev if e0 <= e[0] < s1]
    t = e0
    for i, (s, e, nm, *_r) in enumerate(ks):
        d = pos[i]
        d["name"].append(nm)
        d["start"].append((s - e0) / 1e3)
        d["dur"].append((e - s) / 1e3)
        d["idle"].append(max(0, s - t) / 1e3)
        share[nm] += (e - s) / 1e3
        idle_tot += max(0, s - t) / 1e3
        t = max(t, e)
    idle_tot += max(0, s1 - t) / 1e3
    share["(idle before the rollout kernel)"] += max(0, s1 - t) / 1e3
    gap_tot += (s1 - e0) / 1e3
    roll_tot += (e0 - s0) / 1e3
    n += 1
print(f"per round: rollout kernel {roll_tot / n:.0f} us, gap {gap_tot / n:.0f} us, main stream idle in the gap "
      f"{idle_tot / n:.0f} us")
print("position: most frequent kernel | median start after the rollout kernel, duration, idle before it (us) | rounds")
for i in sorted(pos):
    d = pos[i]
    nm = max(set(d["name"]), key=d["name"].count)
    print(f"  {i:2d} {nm:60s} start {statistics.median(d['start']):7.0f} dur {statistics.median(d['dur']):6.0f} "
          f"idle {statistics.median(d['idle']):6.0f} | {len(d['name'])}")
print("share of the gap (us per round):")
for nm, v in sorted(share.items(), key=lambda x: -x[1])[:20]:
    print(f"  {v / n:7.0f}  {nm}")
