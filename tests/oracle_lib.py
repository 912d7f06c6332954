"""ctypes binding of the oracle (oracle/libws_oracle.so) — test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle", "libws_oracle.so")
_lib = None


def load_oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        lib = C.CDLL(ORACLE)
        vp, u64, i32, u32 = C.c_void_p, C.c_ulonglong, C.c_int, C.c_uint
        P = C.POINTER
        lib.ws_oracle_decode.restype = i32
        lib.ws_oracle_decode.argtypes = [vp, u64, P(vp), P(u64), P(i32), P(i32)]
        lib.ws_oracle_encode_headlen.restype = u32
        lib.ws_oracle_encode_headlen.argtypes = [u64]
        lib.ws_oracle_encode.argtypes = [vp, i32, i32, i32, u64]
        lib.ws_oracle_decode_segments.restype = None
        lib.ws_oracle_decode_segments.argtypes = [vp, vp, vp, u32, u32, vp, vp, vp]
        lib.ws_oracle_sec_accept.restype = vp
        lib.ws_oracle_sec_accept.argtypes = [C.c_char_p, u32, vp]
        _lib = lib
    return _lib


def oracle_segments(buf, seg_off, seg_len, max_frames, desc_base=None):
    """run the a5 loop oracle; buf (numpy uint8) modified in place. Returns (desc, res)."""
    from util_amd.wsframe import DESC_DTYPE, SEGRES_DTYPE
    lib = load_oracle()
    nseg = len(seg_off)
    so = np.ascontiguousarray(seg_off, dtype=np.uint64)
    sl = np.ascontiguousarray(seg_len, dtype=np.uint64)
    nslots = int(max(desc_base) + max_frames) if desc_base is not None and nseg else nseg * max_frames
    desc = np.zeros(max(1, nslots), dtype=DESC_DTYPE)
    res = np.zeros(max(1, nseg), dtype=SEGRES_DTYPE)
    db = None if desc_base is None else np.ascontiguousarray(desc_base, dtype=np.uint64)
    lib.ws_oracle_decode_segments(buf.ctypes.data, so.ctypes.data, sl.ctypes.data, nseg, max_frames,
                                  None if db is None else db.ctypes.data, desc.ctypes.data, res.ctypes.data)
    return desc, res[:nseg]


def used_descs(desc, res, max_frames, desc_base=None):
    """concatenate the used descriptor slots of every segment"""
    out = []
    for s in range(len(res)):
        b = int(desc_base[s]) if desc_base is not None else s * max_frames
        out.append(desc[b:b + int(res[s]["n_frames"])])
    return np.concatenate(out) if out else desc[:0]


def oracle_encode_frames(src, frames):
    """Reference composition of a batch encode: websocketframeEncode's header (the
    oracle restatement, pinned to the reference's golden vectors), then for masked
    (client) frames the MASK bit, the 4 key bytes and the payload XORed with the key
    (RFC 6455 §5.2-5.3). Returns (wire bytes, wire offsets incl. the total)."""
    lib = load_oracle()
    out = bytearray()
    offs = []
    for f in frames:
        offs.append(len(out))
        n = int(f["len"])
        hl = lib.ws_oracle_encode_headlen(n)
        h = (C.c_ubyte * 10)()
        lib.ws_oracle_encode(h, int(f["is_fin"]), int(f["prev_is_fin"]), int(f["type"]), n)
        hb = bytearray(bytes(h)[:hl])
        body = np.frombuffer(bytes(src[int(f["src_off"]):int(f["src_off"]) + n]), dtype=np.uint8).copy()
        if f["masked"]:
            hb[1] |= 0x80
            key = int(f["mask_key"]).to_bytes(4, "little")
            hb += key
            body ^= np.resize(np.frombuffer(key, dtype=np.uint8), n)
        out += hb + body.tobytes()
    offs.append(len(out))
    return bytes(out), np.array(offs, dtype=np.uint64)


def cache_overflow(already, add, max_limit):
    """check_cache_overflow (net_channel_ex.c:45-53), u32 operands"""
    if max_limit == 0:
        return False
    if max_limit < add:
        return True
    return already > max_limit - add


def oracle_reassemble(wire, seg_off, seg_len, max_frames, open_in=None, out_off=None, readcache_max=0,
                      cached_in=None):
    """Checker for websocketframeBatchReassembleDevice(Ex), composed from the decode oracle
    (pinned to the reference's golden vectors): the a5 loop runs on a copy of the wire
    (unmasking in place, as websocketframeDecode does), then the stream hook's delivery rule
    (net_channel_ex.c:110-157, pinned to the reference's own reactor by
    tests/golden/reassemble.json) is applied per segment — the bodies of consecutive consumed
    frames form the pending message, a FIN frame closes it; a frame that is cached (arriving
    while a message is pending, or non-FIN) and would take the cached bytes (u32, as
    cache_recv_bytes) past readcache_max stops the segment: WEBSOCKET_SEG_ERR_CACHE_OVERFLOW,
    its descriptor counted, not consumed.
    Returns (desc, res, msgs[s] = [(out_off, len, first, n, complete, continued)],
    regions[s] = (out_off, expected body bytes), open_out, cached_out)."""
    buf = np.asarray(wire, dtype=np.uint8).copy()
    desc, res = oracle_segments(buf, seg_off, seg_len, max_frames)
    res = res.copy()
    msgs, regions, open_out, cached_out = [], [], [], []
    for s in range(len(seg_off)):
        ob = int(out_off[s]) if out_off is not None else int(seg_off[s])
        opened = int(open_in[s]) if open_in is not None else 0
        cached = int(cached_in[s]) & 0xFFFFFFFF if (cached_in is not None and opened) else 0
        cont, first, q, q0 = opened, 0, 0, 0
        bodies, ms = [], []
        for k in range(int(res[s]["n_frames"])):
            d = desc[s * max_frames + k]
            if int(d["ret"]) <= 0:
                break
            n = int(d["datalen"])
            if n > int(seg_len[s]) - q:
                res[s]["status"] = -3
                break
            fin = int(d["is_fin"])
            cache_it = bool(opened) or not fin                          # net_channel_ex.c:129
            if cache_it and cache_overflow(cached, n & 0xFFFFFFFF, readcache_max):
                res[s]["status"] = -4
                res[s]["consumed"] = int(d["frame_off"]) - int(seg_off[s])
                res[s]["n_frames"] = k + 1
                break
            a = int(d["data_off"])
            bodies.append(buf[a:a + n] if n else buf[:0])
            q += n
            if cache_it:
                cached = (cached + (n & 0xFFFFFFFF)) & 0xFFFFFFFF
            opened = 1
            if fin:
                ms.append((ob + q0, q - q0, first, k + 1 - first, 1, cont))
                first, q0, cont, opened, cached = k + 1, q, 0, 0, 0
        if opened and len(bodies) > first:
            ms.append((ob + q0, q - q0, first, len(bodies) - first, 0, cont))
        msgs.append(ms)
        regions.append((ob, np.concatenate(bodies) if bodies else np.zeros(0, np.uint8)))
        open_out.append(opened)
        cached_out.append(cached if opened else 0)
    return desc, res, msgs, regions, np.array(open_out, dtype=np.uint8), np.array(cached_out, dtype=np.uint32)


def reactor_view(msgs, regions, res, open_out, cached_out, s=0):
    """What the reference reactor reports for segment s (one connection's stream), from a
    reassembly result: (complete message lengths, their bodies back to back, bytes consumed,
    frames consumed, detach error, pending, cached) — the fields of tests/golden/reassemble.json."""
    ob, body = regions[s]
    lens, parts = [], []
    for (o, n, _first, _nf, complete, _cont) in msgs[s]:
        if complete:
            lens.append(int(n))
            parts.append(body[int(o) - ob:int(o) - ob + int(n)])
    st = int(res[s]["status"])
    nf = int(res[s]["n_frames"]) - (1 if st in (-1, -4) else 0)
    return (lens, np.concatenate(parts) if parts else np.zeros(0, np.uint8), int(res[s]["consumed"]), nf,
            7 if st == -4 else 0, int(open_out[s]), int(cached_out[s]))
