"""debug: the golden segment cases through the fused launch, byte ranges that differ from the oracle"""
import json, sys, os
import numpy as np
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import torch
from util_amd import wsframe as W
from oracle_lib import oracle_segments
from test_gpu_parity import gpu_decode
dev = torch.device("cuda:0")
cases = json.load(open("tests/golden/decode_segments.json"))["cases"]
for fused in (0, 1):
    W.set_option("path", 3)
    W.set_option("piece_fused", fused)
    for c in cases:
        wire = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
        gb, gd, gr = gpu_decode(dev, wire.copy(), c["seg_off"], c["seg_len"], c["max_frames"])
        ob = wire.copy()
        od, orr = oracle_segments(ob, c["seg_off"], c["seg_len"], c["max_frames"])
        bad = np.nonzero(gb != ob)[0]
        runs = []
        if len(bad):
            st = bad[0]; pv = bad[0]
            for x in bad[1:]:
                if x != pv + 1:
                    runs.append((int(st), int(pv) + 1)); st = x
                pv = x
            runs.append((int(st), int(pv) + 1))
        print(fused, c["name"], "res_eq", bool(np.array_equal(gr, orr)), "bad bytes", len(bad), runs[:8],
              "unchanged" if len(bad) and np.array_equal(gb[bad], wire[bad]) else "", "fails", W.get_stat("fused_fails"),
              "fused_calls", W.get_stat("fused_calls"), flush=True)
