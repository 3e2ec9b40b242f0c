"""Kernels around a few late-query gaps between rollout kernels (start/end relative to the gap start, per
stream) from a rocprofv3 --kernel-trace CSV: which kernel holds the critical path.  Usage: python tools/gap_detail.py <kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ","").replace("clrrt::","")[:34], r["Stream_Id"]) for r in rows)
roll = [(s, e) for s, e, n, st in ev if "k_roll_run" in n]
gaps = [(e0, s1) for (s0, e0), (s1, e1) in zip(roll, roll[1:]) if 0 < s1 - e0 < 5e6]
# pick gaps of the first query's last quarter
q = gaps[:270]
for e0, s1 in q[200:203] + q[-3:]:
    print(f"--- gap {(s1-e0)/1e3:.0f} us")
    for s, e, n, st in ev:
        if e > e0 - 3e6 and s < s1 and "k_roll_run" not in n:
            if e < e0 - 0: 
                if e < e0 - 200000: continue
            print(f"  st{st} {n:34s} {(s-e0)/1e3:8.0f} .. {(e-e0)/1e3:8.0f} us")
