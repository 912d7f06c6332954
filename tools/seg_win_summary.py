"""Summarise tools/exp_place_seg.py output (one JSON line per file): per option value, the mean
over workloads (placements) and rounds, and the per-workload range.
    python tools/seg_win_summary.py gpurun_out/segwin_reasm.json ..."""
import json
import sys
from collections import defaultdict

for f in sys.argv[1:]:
    d = json.load(open(f))
    by = defaultdict(list)
    per = defaultdict(list)
    for k, v in d["ms"].items():
        wl, val = k.split("_", 1)
        by[val].append(sum(v) / len(v))
        per[val].extend(v)
    print("%s (%s, %s): " % (f, d["op"], d["option"]) + "; ".join(
        "%s mean %.4f ms (workloads %.4f-%.4f)" % (val, sum(m) / len(m), min(m), max(m)) for val, m in sorted(by.items())))
