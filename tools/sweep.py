"""In-process A/B sweep of decode-kernel launch variants (interleaved rounds,
one process, same buffer; cdna_hip_programming.md §5.4 rule 24).

    python tools/sweep.py --config cfg2 --rounds 5 --iters 10 \
        --variants "dyn=1,unroll=4,nt=1" "dyn=0,unroll=4,nt=1" ...
Prints one JSON line per variant: median / min kernel ms and GB/s (algorithmic).
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def parse(v):
    out = {}
    for kv in v.split(","):
        if kv:
            k, x = kv.split("=")
            out[k] = int(x)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", nargs="+", default=["dyn=1,unroll=4,nt=1"])
    args = ap.parse_args()
    import torch
    import bench
    from util_amd import wsframe as W
    dev = torch.device("cuda:0")
    wl = bench.Workload.make(args.config, dev, nframes=args.frames)
    variants = [parse(v) for v in args.variants]
    # the library defaults (WsTuning in ws_api.hip); every variant starts from these
    defaults = {"path": 3, "piece_scan": 3, "dyn": 0, "unroll": 4, "nt": 1, "blocks_per_cu": 64}
    times = {i: [] for i in range(len(variants))}
    for r in range(args.rounds):
        for i, v in enumerate(variants):
            cfg = dict(defaults, **v)
            for k, x in cfg.items():
                W.set_option(k, x)
            wl.decode()  # warm this variant
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
            for a, b in ev:
                a.record()
                wl.decode()
                b.record()
            torch.cuda.synchronize()
            times[i] += [a.elapsed_time(b) for a, b in ev]
    for k, x in defaults.items():
        W.set_option(k, x)
    ok = wl.verify(expect_plain=(wl.decodes % 2 == 1)) == 0
    for i, v in enumerate(variants):
        t = np.array(times[i])
        med = float(np.median(t))
        print(json.dumps({"config": args.config, "variant": args.variants[i], "median_ms": round(med, 4),
                          "min_ms": round(float(t.min()), 4), "GBps_median": round(wl.algo_bytes / med / 1e6, 1),
                          "frac_8TBs": round(wl.algo_bytes / med / 1e6 / 8000, 4), "verified": ok}), flush=True)


if __name__ == "__main__":
    main()
