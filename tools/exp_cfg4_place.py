"""Experiment only (DESIGN §4, cfg4's two modes): one cfg4 round (1 M x 64 KiB masked frames,
68.7 GB of wire) generated into each of K separately allocated buffers in ONE process, then
decoded `iters` times per buffer, buffers interleaved for `rounds` rounds. If the per-buffer
times differ by a stable factor, the decode's rate depends on where its buffer lies in
physical memory (not on the process, the box's clocks or its history).
    GPU box: python tools/exp_cfg4_place.py [K] [rounds] [iters]"""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
from util_amd import synth  # noqa: E402
from util_amd import wsframe as W  # noqa: E402
import numpy as np  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda", 0)
nf, fps = 1 << 20, 16
fl = int(os.environ.get("EXP_FL", "65536"))                  # 4096: cfg2's frames (4.3 GB buffers)
wirelen = int(synth.wirelens(np.array([fl], np.uint64))[0])
nseg = nf // fps
foff = torch.arange(nf, dtype=torch.int64, device=dev) * wirelen
so = foff[::fps].contiguous()
sl = torch.full((nseg,), fps * wirelen, dtype=torch.int64, device=dev)
desc = torch.empty(nf * 32, dtype=torch.uint8, device=dev)
res = torch.empty(nseg * 16, dtype=torch.uint8, device=dev)
bufs = []
for k in range(K):
    b = torch.empty(nf * wirelen + 256, dtype=torch.uint8, device=dev)
    b[nf * wirelen:].zero_()
    W.synth_device(b, foff, nf, 0, fl, 0, 4 if fl == 65536 else 2, first_frame=0)
    bufs.append(b)
torch.cuda.synchronize()
# EXP_WIN: the unmask kernel's window counts to try per buffer (option piece_win, log2)
wins = [int(x) for x in os.environ.get("EXP_WIN", "1").split(",")]
out = {"buffers": [hex(b.data_ptr()) for b in bufs], "ms": {}}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for w in wins:
        W.set_option("piece_win", w)
        for k, b in enumerate(bufs):
            for _ in range(2):
                W.batch_decode_device(b, so, sl, fps, desc, res)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                W.batch_decode_device(b, so, sl, fps, desc, res)
            e1.record()
            torch.cuda.synchronize()
            out["ms"].setdefault("buf%d_win%d" % (k, w), []).append(round(e0.elapsed_time(e1) / iters, 3))
W.set_option("piece_win", -1)
print(json.dumps(out))
