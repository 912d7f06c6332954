"""ctypes driver of oracle/_ref/libwsref_reactor.so — TEST INFRASTRUCTURE ONLY.

Runs the reference's own rx stack (NetReactor_handle -> reactor_stream_readev ->
on_read_stream -> fragment cache -> on_recv, compiled from /root/reference sources by
`make -C oracle ref`) over one connection's byte stream, fed through a socketpair in
`chunk`-byte writes. Exists only in this container (the reference does not travel): the
GPU box checks against tests/golden/reassemble.json, which tests/golden/make_reasm_golden.py
produced with this driver.
"""
import ctypes as C
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
HARNESS = os.path.join(REF_DIR, "libwsref_reactor.so")
CODEC = os.path.join(REF_DIR, "libwsref.so")
_h = None


def available():
    return os.path.exists(HARNESS) and os.path.exists(CODEC)


def _load():
    global _h
    if _h is None:
        h = C.CDLL(HARNESS)
        codec = C.CDLL(CODEC)      # RTLD_LOCAL: its websocketframeDecode is reached by pointer only
        vp, u64, u32 = C.c_void_p, C.c_ulonglong, C.c_uint
        h.ref_reactor_deliver.restype = C.c_int
        h.ref_reactor_deliver.argtypes = [vp, u64, u32, u32, vp, vp, vp, u64, vp, u32, C.POINTER(u32),
                                          C.POINTER(u64), C.POINTER(u64), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                          C.POINTER(u32)]
        _h = (h, codec, C.cast(codec.websocketframeDecode, vp))
    return _h


def reactor_deliver(wire, chunk=65536, readcache_max=0, on_decode=None, max_msgs=1 << 20):
    """Deliveries of the reference reactor for one connection's stream `wire` (uint8 array).
    on_decode: None = the reference glue around the reference's websocketframeDecode; else a
    C function pointer (int) used as NetChannelExProc_t.on_decode.
    Returns dict(lens=[message lengths], bodies=uint8 concatenation, consumed, frames, detach_error,
    pending = fragments still cached at the end, cached = their cache_recv_bytes)."""
    h, _, dec = _load()
    wire = np.ascontiguousarray(wire, dtype=np.uint8)
    out = np.empty(max(1, len(wire)), np.uint8)
    lens = np.zeros(max_msgs, np.uint64)
    n, cons, frames, det = C.c_uint(), C.c_ulonglong(), C.c_ulonglong(), C.c_int()
    pend, cached = C.c_int(), C.c_uint()
    rc = h.ref_reactor_deliver(wire.ctypes.data if len(wire) else None, len(wire), chunk, readcache_max, dec,
                               on_decode, out.ctypes.data, len(out), lens.ctypes.data, max_msgs, C.byref(n),
                               C.byref(cons), C.byref(frames), C.byref(det), C.byref(pend), C.byref(cached))
    if rc:
        raise RuntimeError("ref_reactor_deliver failed: %d" % rc)
    ls = [int(x) for x in lens[:n.value]]
    return dict(lens=ls, bodies=out[:sum(ls)].copy(), consumed=int(cons.value), frames=int(frames.value),
                detach_error=int(det.value), pending=int(pend.value), cached=int(cached.value))
