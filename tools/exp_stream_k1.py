"""Does the batch K1 in front speed up the raw stream's K2 (tools/exp_k1k2.hip
exp_stream_batchk1_k2)? cfg3, ms per (K1 +) K2 step, minus the K1 alone. GPU box."""
import ctypes as C
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
wl = bench.Workload.make("cfg3", dev)
lib = C.CDLL(os.path.join(here, "libexp_k1k2.so"))
vp, u64 = C.c_void_p, C.c_ulonglong
f = lib.exp_stream_batchk1_k2
f.restype = C.c_int
f.argtypes = [vp, u64, C.c_uint, vp, vp, vp, vp, C.c_uint, C.c_uint, vp, vp, C.c_int, C.c_int, vp]
res = torch.zeros(16, dtype=torch.uint8, device=dev)
sdesc = torch.empty(wl.nframes * 32, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream()
out = {}
for r in range(2):
    for k1 in (1, 0):
        ts = []
        for n in (1, 7):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = f(wl.buf.data_ptr(), wl.wire_bytes, wl.nframes, sdesc.data_ptr(), res.data_ptr(), wl.seg_off.data_ptr(),
                   wl.seg_len.data_ptr(), wl.nseg, wl.fps, wl.desc.data_ptr(), wl.res.data_ptr(), n, k1,
                   st.cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            ts.append(e0.elapsed_time(e1))
        out.setdefault("batchK1+streamK2" if k1 else "streamK2", []).append(round((ts[1] - ts[0]) / 6, 4))
print(json.dumps(out))
