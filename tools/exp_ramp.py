"""How the headline decode's per-call time evolves in a FRESH process after bench.py's prelude
(workload generation, the CPU-baseline host sample, the plain-XOR reference of N calls), then
`warmup` decodes and 200 decodes with events between calls: means of each 10-call group.

    python tools/exp_ramp.py --xor 100 [--idle-ms 0] [--no-sample]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--xor", type=int, default=100)
    ap.add_argument("--xor-ms", type=float, default=0.0, help="run the XOR reference for at least this long instead")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--idle-ms", type=float, default=0.0)
    ap.add_argument("--no-sample", action="store_true")
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--pre-decode", type=int, default=0, help="decode calls on the same batch before the idle gap")
    ap.add_argument("--pre-other", type=int, default=0, help="decode calls on a second batch (other memory) before")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    wl = bench.Workload.make("cfg2", dev)
    torch.cuda.synchronize()
    if not args.no_sample:
        wl.host_sample(262144)
    lib = wl.W.load_bench_lib()
    nb = wl.wire_bytes // 16 * 16
    st = torch.cuda.current_stream().cuda_stream
    nx = 0
    tx = time.perf_counter()
    while nx < args.xor or (time.perf_counter() - tx) * 1e3 < args.xor_ms:
        for _ in range(10):
            lib.websocketframeGpuCalibrate(wl.buf.data_ptr(), wl.buf.data_ptr(), nb, 72, 1, 2, st)
        nx += 10
        if args.xor_ms:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    xor_s = time.perf_counter() - tx
    for _ in range(args.pre_decode):
        wl.decode()
    if args.pre_other:
        wl2 = bench.Workload.make("cfg2", dev, first_frame=1 << 22)
        for _ in range(args.pre_other):
            wl2.decode()
        torch.cuda.synchronize()
        del wl2
    torch.cuda.synchronize()
    if args.idle_ms:
        time.sleep(args.idle_ms / 1e3)
    for _ in range(args.warmup):
        wl.decode()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.n + 1)]
    s = torch.cuda.current_stream()
    evs[0].record(s)
    hs = []
    for i in range(args.n):
        h0 = time.perf_counter()
        wl.decode()
        evs[i + 1].record(s)
        hs.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    d = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.n)]
    groups = [round(sum(d[i:i + 10]) / 10, 4) for i in range(0, args.n, 10)]
    print(json.dumps({"xor_calls": nx, "xor_s": round(xor_s, 3), "idle_ms": args.idle_ms, "warmup": args.warmup,
                      "sample": not args.no_sample, "pre_decode": args.pre_decode, "pre_other": args.pre_other, "first20_mean": round(sum(d[:20]) / 20, 4), "first10": [round(x, 4) for x in d[:10]],
                      "group_means": groups, "host_us_first10": [round(x * 1e6) for x in hs[:10]], "prelude_s": round(tx - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
