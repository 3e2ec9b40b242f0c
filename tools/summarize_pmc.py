#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel: dispatches, sum and mean per dispatch
of each counter.  Usage: summarize_pmc.py [--build COMMIT] run_counter_collection.csv [more.csv ...] > summary.json
(--build records the profiled build's commit under "_build", which bench.py quotes in traffic_note; "_src" is the
sources' fingerprint, by which bench.py picks the pass of the build it runs on)."""
import collections
import csv
import json
import sys

args = sys.argv[1:]
build = None
if args and args[0] == "--build":
    build, args = args[1], args[2:]
out = collections.defaultdict(lambda: {"dispatches": 0, "counters": collections.defaultdict(float)})
for path in args:
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
if build:
    res["_build"] = build
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bench import source_fingerprint  # noqa: E402
res["_src"] = source_fingerprint()  # bench.py names the pass of the build it runs on
json.dump(res, sys.stdout, indent=1, sort_keys=True)
