"""Experiment only (placement): K workloads of one bench config in ONE process (each
its own buffer, so its own physical placement), every (window count, workload) pair timed with
`iters` back-to-back decode calls, rounds interleaved.
    GPU box: python tools/exp_place_win.py <config> [K] [rounds] [iters]   (EXP_WIN=1,2)
EXP_STREAM=1: the raw-stream decode of each workload's wire instead (option stream_win)."""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
wins = [int(x) for x in os.environ.get("EXP_WIN", "1,2").split(",")]
opt = os.environ.get("EXP_OPT", "piece_win")                  # seg_win: the segment kernels (cfg5)
dflt = {"piece_win": -1, "seg_win": -1, "piece_dir": 0, "stream_win": 2}.get(opt, 0)
stream = os.environ.get("EXP_STREAM") == "1"
dev = torch.device("cuda", 0)
wls = [bench.Workload.make(cfg, dev) for _ in range(K)]
res = torch.zeros(16, dtype=torch.uint8, device=dev)


def call(w):
    if stream:
        W.stream_decode_device(w.buf, w.wire_bytes, w.nframes, w.desc, res)
    else:
        W.batch_decode_device(w.buf, w.seg_off, w.seg_len, w.fps, w.desc, w.res)



torch.cuda.synchronize()
out = {"config": cfg, "buffers": [hex(w.buf.data_ptr()) for w in wls], "ms": {}}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for win in wins:
        W.set_option(opt, win)
        for k, w in enumerate(wls):
            for _ in range(2):
                call(w)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                call(w)
            e1.record()
            torch.cuda.synchronize()
            out["ms"].setdefault("buf%d_win%d" % (k, win), []).append(round(e0.elapsed_time(e1) / iters, 4))
W.set_option(opt, dflt)
print(json.dumps(out))
