"""Streaming ceilings on this GPU (websocketframeGpuCalibrate) at the decode's byte count.

    python tools/calib.py [--gib 4.0] [--iters 10]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=4303355904)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="", help="comma list of mode[:blocks]")
    args = ap.parse_args()
    import torch
    from util_amd._lib import load_bench_lib as load_lib
    lib = load_lib()
    n = args.bytes // 16 * 16
    a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    b = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    if args.modes:
        names = {16: "buf256x4_nt_nt", 17: "buf256x4_plain", 18: "buf256x4_nt_sc1", 19: "buf256x4_nt_plain",
                 20: "buf256x4_plain_nt", 21: "buf256x8_nt", 22: "buf512x4_nt", 23: "buf1024x4_nt",
                 24: "buf256x2_nt", 25: "buf256x16_nt", 26: "buf256x4_sc0nt", 27: "buf256x4_nt_sc1nt",
                 28: "buf128x4_nt", 29: "buf64x4_nt", 30: "buf256x4_sc1nt_sc1nt", 31: "buf256x4_sc0nt_sc1nt",
                 32: "buf256x4_sc0sc1nt_sc1nt", 33: "buf256x4_sc1_sc1nt", 34: "buf256x4_nt_sc0sc1nt", 5: "rounds1", 4: "oneshot",
                 40: "ldspipe512x6_c3", 41: "ldspipe512x8_c3", 42: "ldspipe256x12_c3", 43: "ldspipe1024x3_c3",
                 44: "ldspipe512x6_c1", 45: "ldspipe512x6_c7", 46: "ldspipe256x8_c3", 47: "ldspipe512x6_il",
                 48: "ldspipe256x8_il", 49: "ldspipe1024x3_il", 60: "dep256x4_d0", 61: "dep256x4_d1",
                 62: "dep256x4_d2", 63: "dep256x4_d4", 64: "dep256x8_d2", 65: "dep512x8_d2"}
        res = {}
        for r in range(3):
            for spec in args.modes.split(","):
                mode, _, blocks = spec.partition(":")
                mode, blocks = int(mode), int(blocks or 0)
                ts = []
                for i in range(args.iters + 1):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rc = lib.websocketframeGpuCalibrate(a.data_ptr(), b.data_ptr(), n, mode, 1, blocks, st)
                    e1.record()
                    assert rc == 0, lib.websocketframeGpuLastError()
                    torch.cuda.synchronize()
                    if i:
                        ts.append(e0.elapsed_time(e1))
                res.setdefault(spec, []).extend(ts)
        for spec, ts in res.items():
            med = float(np.median(ts))
            mode = int(spec.partition(":")[0])
            print(json.dumps({"kernel": names.get(mode, mode), "mode": spec, "median_ms": round(med, 4),
                              "GBps": round(2 * n / med / 1e6, 1)}), flush=True)
        return
    for mode, name, traffic in ((0, "inplace_xor", 2 * n), (3, "inplace_xor_pipelined", 2 * n),
                                (4, "inplace_xor_oneshot", 2 * n), (5, "rounds1", 2 * n), (6, "rounds2", 2 * n),
                                (7, "rounds4", 2 * n), (8, "rounds16", 2 * n), (1, "copy", 2 * n), (2, "read", n)):
        for nt in (0, 1):
            if mode >= 5 and nt == 0:
                continue
            for blocks in ((0,) if mode >= 4 else (1024, 2048, 4096)):
                ts = []
                for i in range(args.iters + 2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rc = lib.websocketframeGpuCalibrate(a.data_ptr(), b.data_ptr(), n, mode, nt, blocks, st)
                    e1.record()
                    assert rc == 0
                    torch.cuda.synchronize()
                    if i >= 2:
                        ts.append(e0.elapsed_time(e1))
                med = float(np.median(ts))
                print(json.dumps({"kernel": name, "nt": nt, "blocks": blocks, "bytes": traffic,
                                  "median_ms": round(med, 4), "GBps": round(traffic / med / 1e6, 1)}), flush=True)
    # torch's own elementwise ops for comparison
    for name, fn, traffic in (("torch_xor_inplace_i64", lambda: a.view(torch.int64).bitwise_xor_(0x5A5A), 2 * n),
                              ("torch_copy", lambda: b.copy_(a), 2 * n)):
        ts = []
        for i in range(args.iters + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e0.elapsed_time(e1))
        med = float(np.median(ts))
        print(json.dumps({"kernel": name, "bytes": traffic, "median_ms": round(med, 4),
                          "GBps": round(traffic / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
