"""per-wave SQ counters per kernel from a rocprofv3 counter_collection.csv"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"].split("(")[0][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    w = d.get("SQ_WAVES", 0)
    if w:
        print(k, {c.replace("SQ_", ""): round(v / w, 1) for c, v in sorted(d.items()) if c != "SQ_WAVES"}, "waves", w)
