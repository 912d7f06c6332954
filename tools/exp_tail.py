"""Tail / ramp cost of one-shot streaming grids (DESIGN §4 'batches in flight').

    python tools/exp_tail.py [--bytes 4303355904] [--iters 30]

In-place XOR of the headline's byte count, back-to-back calls, HIP events at the two
ends only: (a) the one-shot grid (mode 4) on one stream; (b) the same grid on two
buffers alternating between two streams (the next grid fills the chip while the previous
one drains); (c) persistent grids over 16 KiB pieces, static (71) and work-stealing
from a ticket counter (70), at several grid sizes.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=4303355904)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    import torch
    from util_amd._lib import load_bench_lib as load_lib
    lib = load_lib()
    n = args.bytes // 16384 * 16384
    a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    b = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    ctr = [torch.zeros(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(2)]
    base = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]

    def call(buf, mode, blocks, stream, c):
        rc = lib.websocketframeGpuCalibrate(buf.data_ptr(), c.data_ptr(), n, mode, 1, blocks, stream.cuda_stream)
        assert rc == 0, lib.websocketframeGpuLastError()

    def run(name, fn):
        for _ in range(3):
            fn(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(base)
        for s in side:
            s.wait_event(e0)
        for i in range(args.iters):
            fn(i)
        for s in side:
            base.wait_stream(s)
        e1.record(base)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        print(json.dumps({"variant": name, "ms_per_call": round(ms, 4), "TBps": round(2 * n / ms / 1e9, 3),
                          "frac": round(2 * n / ms / 1e9 / 8.0, 4)}), flush=True)

    half = n // 2
    ha, hb = a[:half], a[half:]

    def call_n(buf, nbytes, mode, blocks, stream, c):
        rc = lib.websocketframeGpuCalibrate(buf.data_ptr(), c.data_ptr(), nbytes, mode, 1, blocks, stream.cuda_stream)
        assert rc == 0, lib.websocketframeGpuLastError()

    for rep in range(2):
        run("oneshot_1stream", lambda i: call(a, 4, 0, base, ctr[0]))
        run("oneshot_2streams_2bufs", lambda i: call((a, b)[i % 2], 4, 0, side[i % 2], ctr[i % 2]))
        # one call = two half grids on two streams at once (same bytes as one call of (a))
        run("halves_2streams", lambda i: (call_n(ha, half, 4, 0, side[0], ctr[0]),
                                          call_n(hb, half, 4, 0, side[1], ctr[1])))
        def forkjoin(i):                 # what one API call could do: fork from and join back to its stream
            ev = torch.cuda.Event()
            ev.record(base)
            for s in side:
                s.wait_event(ev)
            call_n(ha, half, 4, 0, side[0], ctr[0])
            call_n(hb, half, 4, 0, side[1], ctr[1])
            for s in side:
                base.wait_stream(s)
        run("halves_forkjoin", forkjoin)
        run("halves_1stream", lambda i: (call_n(ha, half, 4, 0, base, ctr[0]),
                                         call_n(hb, half, 4, 0, base, ctr[1])))
        for w in (2, 4, 8, 16):
            run("windows_%d" % w, lambda i, w=w: call(a, 72, w, base, ctr[0]))
        for mode, name in ((6, "rounds2"), (7, "rounds4"), (22, "buf512x4"), (23, "buf1024x4")):
            run(name, lambda i, m=mode: call(a, m, 0, base, ctr[0]))
        if rep == 0:
            run("persist_static_2048", lambda i: call(a, 71, 2048, base, ctr[0]))


if __name__ == "__main__":
    main()
