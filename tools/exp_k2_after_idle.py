"""K2's own duration (k2_timing events) when each decode call follows a long low-activity
period (torch.cuda._sleep: one spinning wave) vs back to back: is K2's slowdown after long
walks (one big segment, stream path) a device power-state effect?"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    wl = bench.Workload.make("cfg2", dev)
    W = wl.W
    for cycles in (0, 2_000_000, 20_000_000, 160_000_000, 0):
        for _ in range(3):
            wl.decode()
        torch.cuda.synchronize()
        W.set_option("k2_timing", 1)
        for _ in range(20):
            if cycles:
                torch.cuda._sleep(cycles)
            wl.decode()
        torch.cuda.synchronize()
        n, ns = W.get_stat("k2_calls"), W.get_stat("k2_ns")
        W.set_option("k2_timing", 0)
        print(json.dumps({"sleep_cycles_before_each_call": cycles, "k2_ms": round(ns / n / 1e6, 4)}), flush=True)


if __name__ == "__main__":
    main()
