"""Experiment only: the raw stream's K2 against the batch K2 on the SAME buffer in
ONE process (so both meet the same HBM placement), alternating: `iters` batch decodes, then
`iters` raw-stream decodes of the same bytes (the stream call's own walk in front), K2's launch
times from the library's k2_timing events, plus each call's event time.
    GPU box: python tools/exp_stream_vs_batch_k2.py [config] [rounds] [iters]"""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
w = bench.Workload.make(cfg, dev)
n = w.wire_bytes
sdesc = torch.empty(w.nframes * 32 + 32, dtype=torch.uint8, device=dev)
sres = torch.empty(16, dtype=torch.uint8, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def batch():
    W.batch_decode_device(w.buf, w.seg_off, w.seg_len, w.fps, w.desc, w.res)


def stream():
    W.stream_decode_device(w.buf, n, w.nframes + 1, sdesc, sres)


out = {"config": cfg, "batch_step_ms": [], "batch_k2_ms": [], "stream_step_ms": [], "stream_k2_ms": []}
for r in range(rounds):
    for name, f in (("batch", batch), ("stream", stream)):
        for _ in range(4):
            f()
        torch.cuda.synchronize()
        W.set_option("k2_timing", 1)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_step_ms"].append(round(e0.elapsed_time(e1) / iters, 4))
        out[name + "_k2_ms"].append(round(W.get_stat("k2_ns") / max(1, W.get_stat("k2_calls")) / 1e6, 4))
        W.set_option("k2_timing", 0)
print(json.dumps(out))
