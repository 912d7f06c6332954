"""PCIe ceilings on the GPU box vs the host path (websocketframeBatchDecodeHost).

    python tools/exp_pcie.py [--gib 4]

Pinned host <-> HBM copies of the headline batch size: H2D alone, D2H alone, both at once on
two streams (what the host path overlaps), then the host path at several group sizes."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=4303355904)
    args = ap.parse_args()
    import torch
    import bench
    n = args.bytes
    h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)

    def both():
        h2d()
        d2h()
    for name, fn in (("h2d", h2d), ("d2h", d2h), ("both", both)):
        dt = timed(fn)
        print(json.dumps({"copy": name, "ms": round(dt * 1e3, 2), "GBps_per_direction": round(n / dt / 1e9, 1)}),
              flush=True)
    del h1, h2, d1, d2
    from util_amd import wsframe as W
    wl = bench.Workload.make("cfg2", torch.device("cuda:0"))
    for mb in (16, 64, 256, 1024):
        W.set_option("host_chunk_mb", mb)
        r, _ = bench.end_to_end(wl, runs=2)
        print(json.dumps({"host_path_chunk_mb": mb, "GiBps_payload": r["value"], "ms": r["ms"],
                          "GBps_per_direction": round(wl.wire_bytes / (r["ms"] / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
