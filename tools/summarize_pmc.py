#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel: dispatches, sum and mean per dispatch
of each counter.  Usage: summarize_pmc.py run_counter_collection.csv [more.csv ...] > summary.json"""
import collections
import csv
import json
import sys

out = collections.defaultdict(lambda: {"dispatches": 0, "counters": collections.defaultdict(float)})
for path in sys.argv[1:]:
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        out[k]["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
        seen[k].add(r["Dispatch_Id"])
    for k, d in seen.items():
        out[k]["dispatches"] = max(out[k]["dispatches"], len(d))
res = {}
for k, v in out.items():
    n = max(1, v["dispatches"])
    res[k] = {"dispatches": v["dispatches"],
              "per_dispatch": {c: x / n for c, x in v["counters"].items()},
              "total": dict(v["counters"])}
json.dump(res, sys.stdout, indent=1, sort_keys=True)
