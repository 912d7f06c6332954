"""Experiment only (placement): K cfg5 workloads in ONE process (each its own
wire and output buffers, so its own placement); an option swept per workload, `iters` calls per
(value, workload, round): the fused reassembly (op reasm) or the segfuse decode (op decode).
    GPU box: python tools/exp_place_seg.py <reasm|decode> <option> <v1,v2,..> [K] [rounds] [iters]"""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

op, opt = sys.argv[1], sys.argv[2]
vals = [int(x) for x in sys.argv[3].split(",")]
K = int(sys.argv[4]) if len(sys.argv) > 4 else 3
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 2
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda", 0)
wls = []
for k in range(K):
    w = bench.Workload.make("cfg5", dev)
    w.out = torch.empty(w.wire_bytes + 64, dtype=torch.uint8, device=dev)
    w.msg = torch.empty(w.nseg * w.fps * 32, dtype=torch.uint8, device=dev)
    w.nmsg = torch.empty(w.nseg, dtype=torch.int32, device=dev)
    wls.append(w)


def call(w):
    if op == "reasm":
        W.batch_reassemble_device(w.buf, w.seg_off, w.seg_len, w.fps, w.desc, w.res, w.out, w.msg, w.nmsg)
    else:
        W.batch_decode_device(w.buf, w.seg_off, w.seg_len, w.fps, w.desc, w.res)


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
out = {"op": op, "option": opt, "ms": {}}
for r in range(rounds):
    for v in vals:
        W.set_option(opt, v)
        for k, w in enumerate(wls):
            for _ in range(2):
                call(w)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                call(w)
            e1.record()
            torch.cuda.synchronize()
            out["ms"].setdefault("wl%d_%s%d" % (k, opt, v), []).append(round(e0.elapsed_time(e1) / iters, 4))
print(json.dumps(out))
