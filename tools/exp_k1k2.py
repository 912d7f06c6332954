"""Why K2 streams faster right behind K1 (tools/exp_k1k2.hip): cfg2 batch, every sequence
timed as one event region of `iters` steps, rounds interleaved. GPU box:
    python tools/exp_k1k2.py [rounds] [iters]"""
import ctypes as C
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda", 0)
wl = bench.Workload.make(os.environ.get("EXP_CFG", "cfg2"), dev)
lib = C.CDLL(os.path.join(here, os.environ.get("EXP_LIB", "libexp_k1k2.so")))
lib.websocketframeGpuSetOption.argtypes = [C.c_char_p, C.c_longlong]
ldsv = [int(x) for x in os.environ.get("EXP_LDS", "0").split(",")]
for kv in filter(None, os.environ.get("EXP_OPTS", "").split(",")):    # e.g. EXP_OPTS=scan_alpha=0
    k, _, v = kv.partition("=")
    assert lib.websocketframeGpuSetOption(k.encode(), int(v)) == 0, kv
f = lib.exp_k1k2_run
f.restype = C.c_int
vp, u64 = C.c_void_p, C.c_ulonglong
f.argtypes = [vp, u64, vp, vp, C.c_uint, C.c_uint, vp, vp, vp, u64, u64, u64, C.c_int, C.c_int, C.c_longlong, vp]
other = torch.zeros(wl.wire_bytes, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream()
nframes = wl.nframes
stride = int(os.environ.get("EXP_STRIDE", "4104"))
names = {0: "K1+K2", 1: "K2", 2: "spin40+K2", 3: "hdrtouch+K2", 4: "midtouch+K2", 5: "othertouch+K2",
         6: "hdrtouch", 7: "K1", 8: "spin40", 9: "K1g+K2", 10: "K1g", 11: "chase+K2", 12: "chase", 13: "K1+xor+K2", 14: "wsread+K2", 15: "K1K1+K2", 16: "alu+K2", 17: "alu", 18: "xor+K2", 19: "xor",
         20: "ntxor+K2", 21: "wr+K2", 22: "ntwr+K2", 23: "rd+K2", 30: "ntxor", 31: "wr", 32: "ntwr", 33: "rd", 40: "K1v", 41: "K1v+K2"}
seq = [(0, 0), (1, 0), (2, 40), (3, 0), (4, 2048), (5, 0), (6, 0), (7, 0), (8, 40), (2, 10)]
if os.environ.get("EXP_MODES"):
    seq = [tuple(int(y) for y in x.split(":")) for x in os.environ["EXP_MODES"].split(",")]
buflen = wl.wire_bytes


def run(mode, arg, it):
    rc = f(wl.buf.data_ptr(), buflen, wl.seg_off.data_ptr(), wl.seg_len.data_ptr(), wl.nseg, wl.fps,
           wl.desc.data_ptr(), wl.res.data_ptr(), other.data_ptr(), other.numel(), nframes, stride, mode, it, arg,
           st.cuda_stream)
    assert rc == 0, rc


res = {}
for r in range(rounds):
  for lds in ldsv:
    assert lib.websocketframeGpuSetOption(b"piece_lds", lds) == 0
    for mode, arg in seq:
        run(mode, arg, 8)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(mode, arg, iters)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault("%s(%d)lds%d" % (names[mode], arg, lds), []).append(round(e0.elapsed_time(e1) / iters, 4))
print(json.dumps(res))
