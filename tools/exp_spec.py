"""A/B: the speculative piece path vs the classic one (scan + unmask) on one workload, in
one process, interleaved rounds (GPU box). python tools/exp_spec.py [cfg] [rounds] [calls]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 40
dev = torch.device("cuda", 0)
W.set_option("path", 3)
wl = bench.Workload.make(cfg, dev)
res = {}
variants = [("classic", 0, 2048), ("spec", 2, 2048)]
if os.environ.get("SPINS0"):
    variants.append(("spec_spins0", 2, 0))
wl.decode()                                       # the device's frame-length hint
torch.cuda.synchronize()
for r in range(rounds):
    for name, mode, spins in variants:
        W.set_option("piece_spec", mode)
        W.set_option("spec_spins", spins)
        for _ in range(6):
            wl.decode()
        torch.cuda.synchronize()
        _, ms = bench.timed_region(wl.decode, calls, 1)
        res.setdefault(name, []).append(round(ms, 4))
W.set_option("spec_spins", 2048)
W.set_option("piece_spec", 0)
wl.decode()
bad = wl.verify(expect_plain=(wl.decodes % 2 == 1))
print(json.dumps({"cfg": cfg, "ms": res, "verify_mismatch": bad, "spec_calls": W.get_stat("piece_spec_calls")}))
