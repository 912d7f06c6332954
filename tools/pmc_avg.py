"""average counter value per kernel over a rocprofv3 counter_collection csv: python tools/pmc_avg.py <csv>..."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print("%-60s %-14s %14.1f  (n=%d)" % (k[:60], c, sum(v) / len(v), len(v)))
