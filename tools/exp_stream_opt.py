"""Experiment only: raw-stream decode of one config's wire (ONE buffer, so one placement) with an
option alternated in-process: `iters` calls per (value, round), rounds interleaved; also the
calls' chunk-walk stats.
    GPU box: python tools/exp_stream_opt.py <config> <option> <v1,v2,...> [rounds] [iters]
(round 5 swept stream_rw_cmax and stream_rw_hm; the latter was removed after it measured neutral,
commit fcd51c2 has it)"""
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
from util_amd import wsframe as W  # noqa: E402

cfg, opt = sys.argv[1], sys.argv[2]
vals = [int(x) for x in sys.argv[3].split(",")]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = torch.device("cuda", 0)
w = bench.Workload.make(cfg, dev)
n = w.wire_bytes
desc = torch.empty(w.nframes * 32 + 32, dtype=torch.uint8, device=dev)
res = torch.empty(16, dtype=torch.uint8, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
out = {"config": cfg, "option": opt, "ms": {}, "chunk_walks": {}, "chunks": {}}
for r in range(rounds):
    for v in vals:
        W.set_option(opt, v)
        for _ in range(3):
            W.stream_decode_device(w.buf, n, w.nframes + 1, desc, res)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            W.stream_decode_device(w.buf, n, w.nframes + 1, desc, res)
        e1.record()
        torch.cuda.synchronize()
        out["ms"].setdefault(str(v), []).append(round(e0.elapsed_time(e1) / iters, 4))
        out["chunk_walks"][str(v)] = W.get_stat("stream_rw_chunk_walks")
        out["chunks"][str(v)] = W.get_stat("stream_rw_chunks")
r = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
out["last_result"] = [int(r["consumed"]), int(r["n_frames"]), int(r["status"])]
print(json.dumps(out))
