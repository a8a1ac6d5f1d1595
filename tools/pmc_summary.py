"""Averages rocprofv3 --pmc counter_collection.csv values per kernel."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
only = sys.argv[2] if len(sys.argv) > 2 else "rollout"
agg = collections.defaultdict(list)
for r in rows:
    if only in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v) / len(v):16.1f}")
