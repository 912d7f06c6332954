"""Experiment: does the in-place one-shot stream rate depend on where a 4.3 GB buffer sits
inside a larger allocation? (websocketframeGpuCalibrate mode 5 = one-shot in-place XOR)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from util_amd._lib import load_bench_lib as load_lib  # noqa: E402

lib = load_lib()
n = 4303355904 // 16 * 16
st = torch.cuda.current_stream().cuda_stream
for total_gb in (0, 18, 36):
    big = torch.empty(int(total_gb * 2**30) if total_gb else n, dtype=torch.uint8, device="cuda")
    offs = [0] if not total_gb else [0, (big.numel() - n) // 2 // 4096 * 4096, big.numel() - n]
    for off in offs:
        a = big[off:off + n]
        ts = []
        for i in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.websocketframeGpuCalibrate(a.data_ptr(), a.data_ptr(), n, 5, 1, 0, st) == 0
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e0.elapsed_time(e1))
        ts.sort()
        print("alloc %d GiB, offset %.1f GiB: median %.4f ms = %.0f GB/s" %
              (total_gb, off / 2**30, ts[len(ts) // 2], 2 * n / ts[len(ts) // 2] / 1e6), flush=True)
    del big, a
    torch.cuda.empty_cache()
