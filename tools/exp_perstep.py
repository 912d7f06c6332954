"""Per-step device times of the headline decode over a 20-step region (events between
calls): how the first calls after a short warm-up differ from steady state, after the
decode's own warm-up only, after a stream of plain XOR calls, and after a 200 ms idle gap."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def region(wl, n=20):
    st = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record(st)
    for i in range(n):
        wl.decode()
        evs[i + 1].record(st)
    torch.cuda.synchronize()
    return [round(evs[i].elapsed_time(evs[i + 1]), 4) for i in range(n)]


def main():
    dev = torch.device("cuda:0")
    wl = bench.Workload.make("cfg2", dev)
    lib = wl.W.load_bench_lib()
    nb = wl.wire_bytes // 16 * 16
    st = torch.cuda.current_stream().cuda_stream
    for case in ("warmup5", "xor100_then_warmup5", "idle200ms_then_warmup5", "warmup60"):
        if case.startswith("xor"):
            for _ in range(100):
                lib.websocketframeGpuCalibrate(wl.buf.data_ptr(), wl.buf.data_ptr(), nb, 72, 1, 2, st)
        if case.startswith("idle"):
            torch.cuda.synchronize()
            time.sleep(0.2)
        for _ in range(60 if case == "warmup60" else 5):
            wl.decode()
        torch.cuda.synchronize()
        d = region(wl)
        print(json.dumps({"case": case, "first5": d[:5], "last5": d[-5:], "mean": round(sum(d) / len(d), 4)}),
              flush=True)


if __name__ == "__main__":
    main()
