"""spec vs classic over uniform frame sizes (cfg2's layout, ~4 GiB, 16-frame segments):
python tools/exp_spec_sweep.py 2048,8192,..."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

dev = torch.device("cuda", 0)
W.set_option("path", 3)
for plen in [int(x) for x in sys.argv[1].split(",")]:
    wl = bench.Workload.make("cfg2", dev, nframes=(4 << 30) // plen, plen=plen)
    wl.decode()
    torch.cuda.synchronize()
    res = {}
    for r in range(2):
        for name, mode in (("classic", 0), ("spec", 2)):
            W.set_option("piece_spec", mode)
            for _ in range(4):
                wl.decode()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(bench.timed_region(wl.decode, 12, 1)[1], 4))
    print(json.dumps({"plen": plen, "ms": res}), flush=True)
    del wl
    torch.cuda.empty_cache()
