"""A/B: spec kernel (and its copy-floor variant) at several blocks-per-CU caps (piece_lds), cfg2"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

dev = torch.device("cuda", 0)
W.set_option("path", 3)
wl = bench.Workload.make("cfg2", dev)
wl.decode()
torch.cuda.synchronize()
out = {}
for mode, dbg in [("classic", 0), ("spec", 0), ("copy", 5)]:
    W.set_option("piece_spec", 0 if mode == "classic" else 2)
    W.set_option("spec_dbg", dbg)
    for lds in [int(x) for x in sys.argv[1].split(",")]:
        W.set_option("piece_lds", lds)
        for _ in range(4):
            wl.decode()
        torch.cuda.synchronize()
        out["%s/%d" % (mode, lds)] = round(bench.timed_region(wl.decode, 20, 1)[1], 4)
W.set_option("spec_dbg", 0)
W.set_option("piece_lds", 0)
print(json.dumps(out))
