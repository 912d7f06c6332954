"""The raw-stream K2 re-run on the stream call's own workspace vs the stream call and vs the
batch K1 + K2 / K2 alone on the same wire (tools/exp_k1k2.hip). GPU box:
    python tools/exp_stream_k2.py [cfg] [rounds] [iters]"""
import ctypes as C
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 6
dev = torch.device("cuda", 0)
wl = bench.Workload.make(cfg, dev)
lib = C.CDLL(os.path.join(here, os.environ.get("EXP_LIB", "libexp_k1k2.so")))
vp, u64 = C.c_void_p, C.c_ulonglong
f = lib.exp_stream_k2
f.restype = C.c_int
f.argtypes = [vp, u64, C.c_uint, vp, vp, C.c_int, C.c_int, vp, u64, vp]
h = lib.exp_batch_touch_k2
h.restype = C.c_int
h.argtypes = [vp, u64, vp, vp, C.c_uint, C.c_uint, vp, vp, vp, u64, C.c_int, vp]
g = lib.exp_k1k2_run
g.restype = C.c_int
g.argtypes = [vp, u64, vp, vp, C.c_uint, C.c_uint, vp, vp, vp, u64, u64, u64, C.c_int, C.c_int, C.c_longlong, vp]
res = torch.zeros(16, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream()


def timed(fn):
    fn(2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn(iters)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


out = {}
for r in range(rounds):
    # stream call alone (per call); stream call + iters K2 re-runs (minus one call) per K2
    t_call = timed(lambda n: f(wl.buf.data_ptr(), wl.wire_bytes, wl.nframes, wl.desc.data_ptr(), res.data_ptr(), 1, n,
                               wl.frame_off.data_ptr(), wl.nframes, st.cuda_stream)) / iters
    if os.environ.get("EXP_QUICK"):
        out.setdefault("stream_call", []).append(round(t_call, 4))
        continue
    t_k2 = (timed(lambda n: f(wl.buf.data_ptr(), wl.wire_bytes, wl.nframes, wl.desc.data_ptr(), res.data_ptr(), 0, n,
                              wl.frame_off.data_ptr(), wl.nframes, st.cuda_stream)) - t_call) / iters
    t_k2t = (timed(lambda n: f(wl.buf.data_ptr(), wl.wire_bytes, wl.nframes, wl.desc.data_ptr(), res.data_ptr(), 2, n,
                               wl.frame_off.data_ptr(), wl.nframes, st.cuda_stream)) - t_call) / iters
    t_bk2t = timed(lambda n: h(wl.buf.data_ptr(), wl.wire_bytes, wl.seg_off.data_ptr(), wl.seg_len.data_ptr(), wl.nseg,
                               wl.fps, wl.desc.data_ptr(), wl.res.data_ptr(), wl.frame_off.data_ptr(), wl.nframes, n,
                               st.cuda_stream)) / iters
    t_b = timed(lambda n: g(wl.buf.data_ptr(), wl.wire_bytes, wl.seg_off.data_ptr(), wl.seg_len.data_ptr(), wl.nseg,
                            wl.fps, wl.desc.data_ptr(), wl.res.data_ptr(), wl.buf.data_ptr(), wl.wire_bytes,
                            wl.nframes, 4104, 0, n, 0, st.cuda_stream)) / iters
    out.setdefault("stream_touch_k2", []).append(round(t_k2t, 4))
    out.setdefault("batch_touch_k2", []).append(round(t_bk2t, 4))
    out.setdefault("batch_k1_k2", []).append(round(t_b, 4))
    t_bk2 = timed(lambda n: g(wl.buf.data_ptr(), wl.wire_bytes, wl.seg_off.data_ptr(), wl.seg_len.data_ptr(), wl.nseg,
                              wl.fps, wl.desc.data_ptr(), wl.res.data_ptr(), wl.buf.data_ptr(), wl.wire_bytes,
                              wl.nframes, 4104, 1, n, 0, st.cuda_stream)) / iters
    out.setdefault("stream_call", []).append(round(t_call, 4))
    out.setdefault("stream_k2_rerun", []).append(round(t_k2, 4))
    out.setdefault("batch_k2_alone", []).append(round(t_bk2, 4))
print(json.dumps({"cfg": cfg, "ms": out}))
