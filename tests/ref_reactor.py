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


def reactor_deliver_batched(wires, chunk=1500, readcache_max=0, max_frames=64, gpu_fn=None, oracle_fn=None,
                            replay_fn=None, max_msgs=1 << 16):
    """The GPU batch binding at the reactor over the reference's own
    reactor and stream hook, several connections at once (oracle/reactor_harness.c:
    ref_reactor_deliver_batched): every round, each peer writes `chunk` bytes, the reactor
    recv()s them, ONE batch decode runs over every readable channel's whole m_inbuf (the
    previous read's undecoded tail first), and each channel's on_read loop replays that batch
    through replay_fn (websocketframeOnDecodeBatch). gpu_fn: websocketframeBatchDecodeHost
    (C pointer); else oracle_fn: ws_oracle_decode_segments. Returns (per-connection dicts as
    reactor_deliver's, number of batch decodes)."""
    h, _, _ = _load()
    if not hasattr(h, "_batched"):
        vp, u64, u32 = C.c_void_p, C.c_ulonglong, C.c_uint
        f = h.ref_reactor_deliver_batched
        f.restype = C.c_int
        f.argtypes = [u32, vp, vp, u32, u32, u32, vp, vp, vp, vp, u64, vp, u32, vp, vp, vp, vp, vp, vp, C.POINTER(u32)]
        h._batched = f
    n = len(wires)
    arrs = [np.ascontiguousarray(w, dtype=np.uint8) for w in wires]
    ptrs = (C.c_void_p * n)(*[a.ctypes.data if len(a) else None for a in arrs])
    lens = np.array([len(a) for a in arrs], np.uint64)
    per = max(1, max(len(a) for a in arrs))
    out = np.empty(per * n, np.uint8)
    msg_len = np.zeros(max_msgs * n, np.uint64)
    n_msgs = np.zeros(n, np.uint32)
    cons = np.zeros(n, np.uint64)
    frames = np.zeros(n, np.uint64)
    det = np.zeros(n, np.int32)
    pend = np.zeros(n, np.int32)
    cached = np.zeros(n, np.uint32)
    nb = C.c_uint()
    rc = h._batched(n, ptrs, lens.ctypes.data, chunk, readcache_max, max_frames, gpu_fn, oracle_fn, replay_fn,
                    out.ctypes.data, len(out), msg_len.ctypes.data, max_msgs * n, n_msgs.ctypes.data, cons.ctypes.data,
                    frames.ctypes.data, det.ctypes.data, pend.ctypes.data, cached.ctypes.data, C.byref(nb))
    if rc:
        raise RuntimeError("ref_reactor_deliver_batched failed: %d" % rc)
    res = []
    for c in range(n):
        ls = [int(x) for x in msg_len[c * max_msgs:c * max_msgs + n_msgs[c]]]
        res.append(dict(lens=ls, bodies=out[c * per:c * per + sum(ls)].copy(), consumed=int(cons[c]),
                        frames=int(frames[c]), detach_error=int(det[c]), pending=int(pend[c]), cached=int(cached[c])))
    return res, nb.value
