"""Generate golden vectors from the REFERENCE build (run in the dev container only).

    make -C oracle ref && python tests/golden/make_golden.py

Calls hujianzhe/util's own websocketframeDecode / handshake functions, compiled
from /root/reference sources into oracle/_ref/libwsref.so by oracle/Makefile,
and records inputs + observed outputs as small JSON fixtures. The reference
has no tests or fixtures of its own, so these vectors are what pins
the oracle (tests/test_oracle_golden.py) and the product (tests/test_*).

Only data is committed (hex inputs, outputs, hashes); no reference source.
"""
import ctypes as C
import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import wsynth  # noqa: E402

REF = os.path.join(HERE, "..", "..", "oracle", "_ref", "libwsref.so")
SENT_U64 = 0xA5A5A5A5A5A5A5A5
SENT_INT = -7


def load_ref():
    lib = C.CDLL(os.path.abspath(REF))
    lib.websocketframeDecode.restype = C.c_int
    lib.websocketframeDecode.argtypes = [C.c_void_p, C.c_ulonglong, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_ulonglong), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.websocketframeComputeSecAccept.restype = C.c_void_p
    lib.websocketframeComputeSecAccept.argtypes = [C.c_char_p, C.c_uint, C.c_char_p]
    lib.websocketframeDecodeHandshakeRequest.restype = C.c_int
    lib.websocketframeDecodeHandshakeRequest.argtypes = [C.c_void_p, C.c_uint, C.POINTER(C.c_void_p),
                                                         C.POINTER(C.c_uint), C.POINTER(C.c_void_p),
                                                         C.POINTER(C.c_uint)]
    lib.websocketframeEncodeHandshakeResponse.restype = C.c_void_p
    lib.websocketframeEncodeHandshakeResponse.argtypes = [C.c_char_p, C.c_uint, C.c_char_p]
    lib.websocketframeEncodeHandshakeResponseWithProtocol.restype = C.c_void_p
    lib.websocketframeEncodeHandshakeResponseWithProtocol.argtypes = [C.c_char_p, C.c_uint, C.c_char_p, C.c_uint]
    lib.websocketframeFreeString.argtypes = [C.c_void_p]
    lib.websocketframeEncodeHeadLength.restype = C.c_uint
    lib.websocketframeEncodeHeadLength.argtypes = [C.c_ulonglong]
    lib.websocketframeEncode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_ulonglong]
    return lib


def masked_wrap_ub(b, length):
    """True if the reference would unmask past the buffer (u64 wrap, websocketframe.c:149)."""
    if length < 2 or not (b[1] >> 7):
        return False
    p7 = b[1] & 0x7F
    ext = 2 if p7 == 126 else (8 if p7 == 127 else 0)
    if length < 2 + ext + 4 or len(b) < 2 + ext:
        return False
    plen = int.from_bytes(bytes(b[2:2 + ext]), "big") if ext else p7
    tot = (2 + ext + 4 + plen) & 0xFFFFFFFFFFFFFFFF
    return tot < plen and length >= tot


def ref_decode(lib, buf, length, base_addr=None):
    """Run the reference on a ctypes buffer; returns a dict of observed outputs."""
    data = C.c_void_p(SENT_U64)
    datalen = C.c_ulonglong(SENT_U64)
    fin = C.c_int(SENT_INT)
    typ = C.c_int(SENT_INT)
    r = lib.websocketframeDecode(buf, length, C.byref(data), C.byref(datalen), C.byref(fin), C.byref(typ))
    base = C.addressof(buf) if base_addr is None else base_addr
    if data.value == SENT_U64:
        doff = "untouched"
    elif data.value is None:
        doff = None
    else:
        doff = data.value - base
    return {"ret": r, "fin": fin.value, "type": typ.value, "datalen": datalen.value,
            "data_off": doff}


# ---------------------------------------------------------------- single frames

def frame(b0, plen, key=None, payload=None, ext_form=None):
    """build wire bytes; ext_form forces 7/16/64-bit length encoding"""
    if ext_form is None:
        ext_form = 7 if plen < 126 else (16 if plen <= 0xFFFF else 64)
    m = 0x80 if key is not None else 0
    if ext_form == 7:
        h = [b0, m | plen]
    elif ext_form == 16:
        h = [b0, m | 126, (plen >> 8) & 0xFF, plen & 0xFF]
    else:
        h = [b0, m | 127] + [(plen >> (56 - 8 * i)) & 0xFF for i in range(8)]
    if key is not None:
        h += list(key)
    if payload is None:
        payload = bytes((i * 7 + 3) & 0xFF for i in range(min(plen, 1 << 20)))
    body = bytes(payload)
    if key is not None:
        body = bytes(c ^ key[i % 4] for i, c in enumerate(body))
    return bytes(h) + body


def single_cases():
    cases = []

    def add(name, wire, length=None):
        cases.append((name, bytes(wire), len(wire) if length is None else length))

    K = bytes([0xAA, 0x55, 0x0F, 0xF0])
    add("empty", b"")
    add("one_byte", b"\x81")
    add("mask_truncated", bytes([0x81, 0x85, 1, 2, 3]))
    add("payload_short", bytes([0x02, 0x83, 0, 0, 0, 0, ord("a"), ord("b")]))
    add("rsv_bits_empty", bytes([0xF1, 0x00]))
    add("opcode_15_nofin", bytes([0x7F, 0x00]))
    add("reserved_opcode_3", bytes([0x83, 0x00]))
    add("unmasked_abc", bytes([0x82, 0x03]) + b"abc")
    add("masked_zero_len", bytes([0x81, 0x80, 1, 2, 3, 4]))
    add("nonminimal_16bit", bytes([0x82, 0x7E, 0x00, 0x05]) + b"hello")
    add("control_gt125", bytes([0x89, 0x7E, 0x00, 0xC8]) + bytes(range(200)))
    add("ping_masked_xy", bytes([0x89, 0x82, 0xFF, 0x00, 0xFF, 0x00, ord("x"), ord("y")]))
    add("masked_test", frame(0x81, 4, K, b"test"))
    add("len127_65536_masked", frame(0x82, 65536, K))
    w = frame(0x82, 65536, K)
    add("len127_65536_masked_short1", w, len(w) - 1)
    add("len127_msb_set", bytes([0x82, 0x7F, 0x80, 0, 0, 0, 0, 0, 0, 1]))
    # u64 wrap on the length sum (websocketframe.c:149): outputs written, ret (int)sum
    huge = (1 << 64) - 10
    add("len127_unmasked_wrap_ret0", bytes([0x82, 0x7F]) + huge.to_bytes(8, "big"))
    add("len127_unmasked_wrap_ret5", bytes([0x82, 0x7F]) + ((1 << 64) - 5).to_bytes(8, "big") + b"ABCDEFGH")
    # int truncation of the return (websocketframe.c:164); unmasked so no payload is touched
    add("len127_unmasked_2p31", bytes([0x82, 0x7F]) + (1 << 31).to_bytes(8, "big"), (1 << 31) + 10)
    add("len127_unmasked_2p32p100", bytes([0x82, 0x7F]) + ((1 << 32) + 100).to_bytes(8, "big"), (1 << 32) + 110)
    add("len127_unmasked_2p32m10", bytes([0x82, 0x7F]) + ((1 << 32) - 10).to_bytes(8, "big"), (1 << 32))
    # boundary payload lengths, masked and unmasked, every length encoding
    for pl in (0, 1, 2, 3, 4, 5, 125, 126, 127, 65535, 65536):
        add("masked_len_%d" % pl, frame(0x82, pl, K))
        add("unmasked_len_%d" % pl, frame(0x81, pl))
    for pl in (0, 5, 125):
        add("masked_len_%d_ext16" % pl, frame(0x82, pl, K, ext_form=16))
        add("masked_len_%d_ext64" % pl, frame(0x82, pl, K, ext_form=64))
    # truncations of one masked 16-bit frame at every header boundary
    w = frame(0x81, 300, K)
    for L in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 307, 308):
        add("trunc300_len_%d" % L, w, L)
    # extra trailing bytes after a complete frame
    add("masked_test_trailing", frame(0x81, 4, K, b"test") + b"\x81\x85\x00")
    # random short frames
    rng = random.Random(1234)
    for i in range(400):
        pl = rng.choice([0, 1, 2, 3, 7, 13, 64, 100, 125, 126, 200, 1000, 4096])
        form = rng.choice([None, None, None, 16, 64]) if pl <= 0xFFFF else 64
        key = bytes(rng.randrange(256) for _ in range(4)) if rng.random() < 0.8 else None
        b0 = rng.randrange(256)
        payload = bytes(rng.randrange(256) for _ in range(pl))
        w = frame(b0, pl, key, payload, ext_form=form)
        L = len(w) if rng.random() < 0.7 else rng.randrange(len(w) + 1)
        add("rand_%03d" % i, w, L)
    # random garbage
    for i in range(200):
        n = rng.randrange(0, 40)
        g = bytes(rng.randrange(256) for _ in range(n))
        add("garbage_%03d" % i, g)
    return cases


def gen_single(lib):
    out = []
    for name, wire, length in single_cases():
        b = bytearray(wire)
        if masked_wrap_ub(b, length):
            continue
        buf = (C.c_ubyte * max(1, len(b))).from_buffer_copy(bytes(b) if b else b"\0")
        res = ref_decode(lib, buf, length)
        after = bytes(buf)[: len(b)]
        rec = {"name": name, "input": wire.hex(), "len": length}
        rec.update(res)
        rec["output"] = after.hex() if len(after) <= 4096 else None
        rec["output_sha256"] = hashlib.sha256(after).hexdigest()
        out.append(rec)
    return out


# ---------------------------------------------------------------- segments (a5 loop)

def ref_loop(lib, buf, seg_off, seg_len, max_frames):
    """net_reactor.c:515-526 loop per segment, recording descriptor-equivalent outputs"""
    base = C.addressof(buf)
    segs = []
    for so, sl in zip(seg_off, seg_len):
        off, frames, status = 0, [], 0
        while off < sl:
            if len(frames) >= max_frames:
                status = 1
                break
            view = (C.c_ubyte * 1).from_address(base + so + off)
            b = bytes((C.c_ubyte * min(16, sl - off)).from_address(base + so + off))
            if masked_wrap_ub(b, sl - off):
                status = -2
                break
            r = ref_decode(lib, view, sl - off, base_addr=base)
            if r["ret"] == 0:
                break
            hdr = 2 + {126: 2, 127: 8}.get(b[1] & 0x7F, 0) + (4 if b[1] >> 7 else 0)
            frames.append({"frame_off": so + off, "ret": r["ret"], "fin": r["fin"], "type": r["type"],
                           "datalen": r["datalen"], "data_off": r["data_off"], "masked": b[1] >> 7,
                           "hdrlen": hdr})
            if r["ret"] < 0:
                status = -1
                break
            off += r["ret"] & 0xFFFFFFFF
        segs.append({"consumed": off, "n_frames": len(frames), "status": status, "frames": frames})
    return segs


def segment_cases():
    rng = random.Random(99)
    K = [bytes(rng.randrange(256) for _ in range(4)) for _ in range(64)]
    cases = []
    # several frames + incomplete tail
    s = frame(0x81, 5, K[0], b"hello") + frame(0x82, 300, K[1]) + frame(0x09, 0) + frame(0x8A, 3, K[2], b"pon")
    cases.append(("stream_mixed_tail", [s + frame(0x82, 100, K[3])[:50]], 8))
    # exact end, no tail
    cases.append(("stream_exact", [frame(0x82, 126, K[4]) + frame(0x82, 65535, K[5]) + frame(0x82, 65536, K[6])], 8))
    # max_frames stop
    cases.append(("stream_maxframes", [b"".join(frame(0x82, 10, K[i]) for i in range(6))], 4))
    # wrap-5 quirk: ret 5, the loop walks on into the header bytes
    cases.append(("stream_wrap5", [bytes([0x82, 0x7F]) + ((1 << 64) - 5).to_bytes(8, "big") + frame(0x81, 3, K[7], b"abc")], 8))
    # unaligned segments with 16-fragment messages (cfg5 shape, small)
    frag = b"".join(frame(0x02 if j == 0 else (0x80 if j == 15 else 0x00), 1024, K[j]) for j in range(16))
    cases.append(("fragmented_16x1024", [frag], 32))
    # many random segments packed back to back at odd offsets
    segs = []
    for i in range(120):
        n = rng.randrange(0, 6)
        parts = []
        for _ in range(n):
            pl = rng.choice([0, 1, 3, 17, 125, 126, 1000, 4096] + ([70000] if i % 40 == 0 else []))
            form = rng.choice([None, None, 16, 64]) if pl <= 0xFFFF else 64
            key = K[rng.randrange(64)] if rng.random() < 0.85 else None
            parts.append(frame(rng.randrange(256), pl, key, bytes(rng.randrange(256) for _ in range(pl)), ext_form=form))
        seg = b"".join(parts)
        if rng.random() < 0.4 and seg:
            seg = seg[: rng.randrange(len(seg) + 1)]
        if rng.random() < 0.1:
            seg += bytes(rng.randrange(256) for _ in range(rng.randrange(20)))
        segs.append(seg)
    cases.append(("random_segments", segs, 4))
    return cases


def gen_segments(lib):
    out = []
    for name, segs, max_frames in segment_cases():
        pad = 3  # start segments at odd offsets
        blob = bytearray()
        seg_off, seg_len = [], []
        for sg in segs:
            blob += bytes(pad)
            seg_off.append(len(blob))
            seg_len.append(len(sg))
            blob += sg
        blob += bytes(16)
        buf = (C.c_ubyte * len(blob)).from_buffer_copy(bytes(blob))
        res = ref_loop(lib, buf, seg_off, seg_len, max_frames)
        after = bytes(buf)
        out.append({"name": name, "input": bytes(blob).hex(), "seg_off": seg_off, "seg_len": seg_len,
                    "max_frames": max_frames, "segments": res,
                    "output_sha256": hashlib.sha256(after).hexdigest(),
                    "output": after.hex() if len(after) <= 8192 else None})
    return out


# ---------------------------------------------------------------- seeded batch hashes

def desc_bytes(segs):
    """canonical descriptor encoding: same packing as WebsocketFrameDesc_t"""
    dt = np.dtype([("frame_off", "<u8"), ("data_off", "<u8"), ("datalen", "<u8"), ("ret", "<i4"),
                   ("is_fin", "u1"), ("type", "u1"), ("masked", "u1"), ("hdrlen", "u1")])
    rows = []
    for sg in segs:
        for fr in sg["frames"]:
            doff = 0xFFFFFFFFFFFFFFFF if fr["data_off"] is None else fr["data_off"]
            rows.append((fr["frame_off"], doff, fr["datalen"], fr["ret"], fr["fin"], fr["type"],
                         fr["masked"], fr["hdrlen"]))
    return np.array(rows, dtype=dt).tobytes()


BATCHES = [
    # name, nframes, plen_kind, fixed_len, b0_kind, seed, frames per segment
    ("cfg1_16x125_text", 16, wsynth.PLEN_FIXED, 125, wsynth.B0_TEXT, 1, 16),
    ("cfg2_small_256x4096", 256, wsynth.PLEN_FIXED, 4096, wsynth.B0_BINARY, 2, 16),
    ("cfg3_small_48_mix3", 48, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 3, 16),
    ("cfg5_small_4x16x1024", 64, wsynth.PLEN_FIXED, 1024, wsynth.B0_FRAG16, 5, 16),
]


def gen_batches(lib):
    out = []
    for name, n, pk, fl, bk, seed, fps in BATCHES:
        wire, off, pl, plain = wsynth.make_batch(n, pk, fl, bk, seed)
        seg_off = [int(off[i]) for i in range(0, n, fps)]
        ends = [int(off[i + fps]) if i + fps < n else len(wire) for i in range(0, n, fps)]
        seg_len = [e - s for s, e in zip(seg_off, ends)]
        buf = (C.c_ubyte * len(wire)).from_buffer_copy(wire.tobytes())
        segs = ref_loop(lib, buf, seg_off, seg_len, fps)
        after = bytes(buf)
        assert after == plain.tobytes(), name
        rec = {"name": name, "nframes": n, "plen_kind": pk, "fixed_len": fl, "b0_kind": bk, "seed": seed,
               "frames_per_segment": fps, "wire_bytes": len(wire),
               "input_sha256": hashlib.sha256(wire.tobytes()).hexdigest(),
               "output_sha256": hashlib.sha256(after).hexdigest(),
               "desc_sha256": hashlib.sha256(desc_bytes(segs)).hexdigest(),
               "consumed": [s["consumed"] for s in segs], "n_frames": [s["n_frames"] for s in segs]}
        if n <= 16:
            rec["input"] = wire.tobytes().hex()
            rec["segments"] = segs
        out.append(rec)
    return out


# ---------------------------------------------------------------- handshake (§8f row 4)

def gen_handshake(lib):
    out = {"sec_accept": [], "decode_request": [], "encode_response": []}
    rng = random.Random(7)
    keys = [b"dGhlIHNhbXBsZSBub25jZQ==", b"", b"x", b"AQIDBAUGBwgJCgsMDQ4PEA=="]
    keys += [bytes(rng.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=")
                   for _ in range(rng.randrange(1, 80))) for _ in range(30)]
    for k in keys:
        acc = C.create_string_buffer(60)
        r = lib.websocketframeComputeSecAccept(k, len(k), acc)
        out["sec_accept"].append({"key": k.decode(), "accept": acc.value.decode() if r else None})
    reqs = [
        b"GET /chat HTTP/1.1\r\nHost: server.example.com\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
        b"Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nSec-WebSocket-Version: 13\r\n\r\n",
        b"GET / HTTP/1.1\r\nSec-WebSocket-Key:   abc\r\nSec-WebSocket-Protocol: chat, superchat\r\n\r\nTAIL",
        b"GET / HTTP/1.1\r\nSec-WebSocket-Key: abc\r\n",
        b"GET / HTTP/1.1\r\nHost: x\r\n\r\n",
        b"GET / HTTP/1.1\r\nSec-WebSocket-Key:\r\n\r\n",
        b"GET / HTTP/1.1\r\nSec-WebSocket-Protocol:   \r\nSec-WebSocket-Key: k1\r\n\r\n",
        b"GET / HTTP/1.1\r\nSec-WebSocket-Key: \t k2\r\nSec-WebSocket-Protocol:p\r\n\r\n",
    ]
    for q in reqs:
        buf = C.create_string_buffer(q, len(q))
        sk, skl, sp, spl = C.c_void_p(SENT_U64), C.c_uint(777), C.c_void_p(SENT_U64), C.c_uint(777)
        r = lib.websocketframeDecodeHandshakeRequest(buf, len(q), C.byref(sk), C.byref(skl), C.byref(sp), C.byref(spl))
        base = C.addressof(buf)

        def off(p):
            return "untouched" if p.value == SENT_U64 else (None if p.value is None else p.value - base)
        out["decode_request"].append({"request": q.decode(), "ret": r, "sec_key_off": off(sk), "sec_key_len": skl.value,
                                      "sec_protocol_off": off(sp), "sec_protocol_len": spl.value})
    for acc, proto in [(b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo=", None), (b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo=", b"chat"),
                       (b"abc", b""), (b"", b"p1")]:
        b = C.create_string_buffer(162)
        r1 = C.string_at(lib.websocketframeEncodeHandshakeResponse(acc, len(acc), b)).decode()
        p = lib.websocketframeEncodeHandshakeResponseWithProtocol(acc, len(acc), proto, len(proto) if proto else 0)
        r2 = C.string_at(p).decode()
        lib.websocketframeFreeString(p)
        out["encode_response"].append({"accept": acc.decode(), "protocol": None if proto is None else proto.decode(),
                                       "response": r1, "response_with_protocol": r2})
    enc = []
    for dl in (0, 1, 125, 126, 127, 65535, 65536, (1 << 32) + 5):
        for fin, prev in ((1, 1), (0, 1), (1, 0), (0, 0)):
            for t in (1, 2, 9):
                h = (C.c_ubyte * 10)()
                lib.websocketframeEncode(h, fin, prev, t, dl)
                n = lib.websocketframeEncodeHeadLength(dl)
                enc.append({"datalen": dl, "is_fin": fin, "prev_is_fin": prev, "type": t, "headlen": n,
                            "head": bytes(h)[:n].hex()})
    out["encode_header"] = enc
    return out


def main():
    lib = load_ref()
    fx = {
        "decode_single.json": gen_single(lib),
        "decode_segments.json": gen_segments(lib),
        "batches.json": gen_batches(lib),
        "handshake.json": gen_handshake(lib),
    }
    for fn, obj in fx.items():
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py",
                       "source": "reference build oracle/_ref/libwsref.so (hujianzhe/util websocketframe.c, memfunc.c, sha1.c, base64.c)",
                       "cases": obj}, f, indent=0, sort_keys=True)
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
