"""TEMPORARY: run the speculative kernel's debug variants on cfg2 (timings + for PMC)"""
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
W.set_option("piece_spec", 2)
out = {}
for d in [0, 1, 2, 3, 4]:
    W.set_option("spec_dbg", d)
    for _ in range(4):
        wl.decode()
    torch.cuda.synchronize()
    _, ms = bench.timed_region(wl.decode, 20, 1)
    out[d] = round(ms, 4)
W.set_option("spec_dbg", 0)
print(json.dumps(out))
