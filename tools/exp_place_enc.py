"""Experiment only (placement): K encode workloads of one config in ONE process
(each its own source and wire buffers), every (enc_win, workload) pair timed with `iters`
back-to-back encode calls, rounds interleaved.
    GPU box: python tools/exp_place_enc.py [config] [K] [rounds] [iters]   (EXP_WIN=0,1,2)
The swept options (enc_win, enc_xg) were removed from the library after the measurement (round 5,
commit ff92800 has them): EXP_OPT=enc_front still works."""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
wins = [int(x) for x in os.environ.get("EXP_WIN", "0,1,2").split(",")]
opt = os.environ.get("EXP_OPT", "enc_win")                    # or enc_xg
dev = torch.device("cuda", 0)
wls = [bench.EncodeWorkload(cfg, dev, seed_offset=k) for k in range(K)]
torch.cuda.synchronize()
out = {"config": cfg, "ms": {}}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for win in wins:
        W.set_option(opt, win)
        for k, w in enumerate(wls):
            for _ in range(2):
                w.step()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                w.step()
            e1.record()
            torch.cuda.synchronize()
            out["ms"].setdefault("wl%d_win%d" % (k, win), []).append(round(e0.elapsed_time(e1) / iters, 4))
W.set_option(opt, 0)
assert all(w.verify() == 0 for w in wls)
print(json.dumps(out))
