"""Is the decode's rate set by power/clock headroom? Per-call device time of the decode
back to back vs with an idle gap (torch.cuda._sleep: one spinning wave) between calls.

    python tools/exp_gap.py --config cfg4 --frames 358400 [--plen N] [--gaps 0,100000,1000000]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--frames", type=int, default=358400)
    ap.add_argument("--plen", type=int, default=None)
    ap.add_argument("--calls", type=int, default=12)
    ap.add_argument("--gaps", default="0,200000,2000000", help="sleep cycles between calls")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    wl = bench.Workload.make(args.config, dev, nframes=args.frames, plen=args.plen)
    for _ in range(4):
        wl.decode()
    torch.cuda.synchronize()
    for gap in (int(g) for g in args.gaps.split(",")):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.calls)]
        for e0, e1 in ev:
            if gap:
                torch.cuda._sleep(gap)
            e0.record()
            wl.decode()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        med = ts[len(ts) // 2]
        print("%s frames %d plen %s gap %d cycles: median %.3f ms  %.1f%% of 8 TB/s" % (
            args.config, wl.nframes, args.plen, gap, med, wl.algo_bytes / (med / 1e3) / 1e9 / 8000 * 100), flush=True)


if __name__ == "__main__":
    main()
