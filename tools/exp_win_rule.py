"""Experiment only (DESIGN §4 "Buffer placement"): the K2 window count for
batches >= 16 GiB chosen by the batch size alone (four windows: option piece_win=2) against the
current advice rule (piece_win=-1: four only when the previous call on the stream advised frames
of one length, so FIRST calls and CAPTURED calls take two), on K buffers of one config in ONE
process (each its own HBM placement):
  first_k2  one call on a fresh HIP stream (no advice yet): its K2 (library option k2_timing)
  captured  one call captured in a HIP graph, `iters` replays
  steady    the bench protocol: 2 warm-up calls, `iters` timed calls on one stream
    GPU box: python tools/exp_win_rule.py <config> [K] [rounds] [iters]"""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda", 0)
wls = [bench.Workload.make(cfg, dev) for _ in range(K)]
torch.cuda.synchronize()
out = {"config": cfg, "buffers": [hex(w.buf.data_ptr()) for w in wls], "ms": {},
       "rules": {"advice": -1, "size": 2}}


def call(w, st=None):
    W.batch_decode_device(w.buf, w.seg_off, w.seg_len, w.fps, w.desc, w.res, stream=st)


def timed(fn, st, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for r in range(rounds):
    for rule, val in (("advice", -1), ("size", 2)):
        W.set_option("piece_win", val)
        for k, w in enumerate(wls):
            key = "buf%d_%s" % (k, rule)
            st = torch.cuda.Stream(dev)                       # a fresh stream: a slot with no advice
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                call(w, st)                                   # (allocates the slot's workspace)
            torch.cuda.synchronize()
            # a first call's K2 (its workspace is allocated before K2 is launched: the library's
            # k2_timing events around the K2 launch leave that host work out)
            st2 = torch.cuda.Stream(dev)
            W.set_option("k2_timing", 1)
            with torch.cuda.stream(st2):
                call(w, st2)
            torch.cuda.synchronize()
            out["ms"].setdefault(key + "_first_k2", []).append(round(W.get_stat("k2_ns") / 1e6, 4))
            W.set_option("k2_timing", 0)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                call(w)
            cs = torch.cuda.current_stream()
            g.replay()
            out["ms"].setdefault(key + "_captured", []).append(round(timed(g.replay, cs, iters), 4))
            del g
            for _ in range(2):
                call(w)
            out["ms"].setdefault(key + "_steady", []).append(round(timed(lambda: call(w), cs, iters), 4))
        torch.cuda.synchronize()
W.set_option("piece_win", -1)
print(json.dumps(out))
