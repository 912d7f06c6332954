"""Pin the oracle (oracle/ws_oracle.c) to the reference's own outputs.

Golden vectors were produced by the reference build (tests/golden/make_golden.py
-> oracle/_ref/libwsref.so compiled from hujianzhe/util sources). CPU only.
"""
import ctypes as C
import hashlib

import numpy as np
import pytest

import wsynth
from oracle_lib import load_oracle, oracle_segments, used_descs
from util_amd.wsframe import DATA_OFF_NULL, DESC_DTYPE


def golden_desc_rows(segments):
    rows = []
    for sg in segments:
        for fr in sg["frames"]:
            rows.append((fr["frame_off"], DATA_OFF_NULL if fr["data_off"] is None else fr["data_off"], fr["datalen"],
                         fr["ret"], fr["fin"], fr["type"], fr["masked"], fr["hdrlen"]))
    return np.array(rows, dtype=DESC_DTYPE)


def run_oracle_single(lib, wire, length):
    n = max(1, len(wire))
    buf = (C.c_ubyte * n).from_buffer_copy(wire if wire else b"\0")
    sent = 0xA5A5A5A5A5A5A5A5
    data, dl, fin, typ = C.c_void_p(sent), C.c_ulonglong(sent), C.c_int(-7), C.c_int(-7)
    r = lib.ws_oracle_decode(buf, length, C.byref(data), C.byref(dl), C.byref(fin), C.byref(typ))
    doff = "untouched" if data.value == sent else (None if data.value is None else data.value - C.addressof(buf))
    return r, doff, dl.value, fin.value, typ.value, bytes(buf)[: len(wire)]


def test_single_frames(golden):
    lib = load_oracle()
    cases = golden("decode_single.json")
    assert len(cases) > 600
    for c in cases:
        wire = bytes.fromhex(c["input"])
        r, doff, dl, fin, typ, after = run_oracle_single(lib, wire, c["len"])
        assert r == c["ret"], c["name"]
        assert doff == c["data_off"], c["name"]
        assert (dl, fin, typ) == (c["datalen"], c["fin"], c["type"]), c["name"]
        assert hashlib.sha256(after).hexdigest() == c["output_sha256"], c["name"]


def test_segments(golden):
    for c in golden("decode_segments.json"):
        buf = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
        desc, res = oracle_segments(buf, c["seg_off"], c["seg_len"], c["max_frames"])
        exp = golden_desc_rows(c["segments"])
        got = used_descs(desc, res, c["max_frames"])
        assert np.array_equal(got, exp), c["name"]
        assert [int(x) for x in res["consumed"]] == [s["consumed"] for s in c["segments"]], c["name"]
        assert [int(x) for x in res["status"]] == [s["status"] for s in c["segments"]], c["name"]
        assert hashlib.sha256(buf.tobytes()).hexdigest() == c["output_sha256"], c["name"]


@pytest.mark.parametrize("idx", range(4))
def test_seeded_batches(golden, idx):
    c = golden("batches.json")[idx]
    wire, off, pl, plain = wsynth.make_batch(c["nframes"], c["plen_kind"], c["fixed_len"], c["b0_kind"], c["seed"])
    assert hashlib.sha256(wire.tobytes()).hexdigest() == c["input_sha256"]  # generator pinned too
    fps = c["frames_per_segment"]
    n = c["nframes"]
    seg_off = [int(off[i]) for i in range(0, n, fps)]
    ends = [int(off[i + fps]) if i + fps < n else len(wire) for i in range(0, n, fps)]
    seg_len = [e - s for s, e in zip(seg_off, ends)]
    buf = wire.copy()
    desc, res = oracle_segments(buf, seg_off, seg_len, fps)
    assert hashlib.sha256(buf.tobytes()).hexdigest() == c["output_sha256"]
    assert hashlib.sha256(used_descs(desc, res, fps).tobytes()).hexdigest() == c["desc_sha256"]
    assert np.array_equal(buf, plain)


def test_encode(golden):
    lib = load_oracle()
    for c in golden("handshake.json")["encode_header"]:
        h = (C.c_ubyte * 10)()
        lib.ws_oracle_encode(h, c["is_fin"], c["prev_is_fin"], c["type"], c["datalen"])
        n = lib.ws_oracle_encode_headlen(c["datalen"])
        assert n == c["headlen"]
        assert bytes(h)[:n].hex() == c["head"]


def test_sec_accept(golden):
    lib = load_oracle()
    for c in golden("handshake.json")["sec_accept"]:
        out = C.create_string_buffer(60)
        k = c["key"].encode()
        lib.ws_oracle_sec_accept(k, len(k), out)
        assert out.value.decode() == c["accept"], c["key"]
    # RFC 6455 §1.3 sample
    out = C.create_string_buffer(60)
    lib.ws_oracle_sec_accept(b"dGhlIHNhbXBsZSBub25jZQ==", 24, out)
    assert out.value == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_reference_build_agrees_if_present():
    """when the reference build exists (dev container), fuzz oracle vs reference directly"""
    import os
    ref = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libwsref.so")
    if not os.path.exists(ref):
        pytest.skip("reference build not present (GPU box): fixtures carry the pin")
    rl = C.CDLL(ref)
    rl.websocketframeDecode.restype = C.c_int
    rl.websocketframeDecode.argtypes = [C.c_void_p, C.c_ulonglong, C.POINTER(C.c_void_p), C.POINTER(C.c_ulonglong),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]
    ol = load_oracle()
    rng = np.random.default_rng(5)
    for i in range(3000):
        n = int(rng.integers(0, 300))
        b = rng.integers(0, 256, n, dtype=np.uint8)
        if n >= 2 and rng.random() < 0.7:
            b[1] = (b[1] & 0x80) | int(rng.choice([0, 1, 5, 100, 125, 126, 127]))
            if (b[1] & 0x7F) == 127 and n >= 10:
                b[2:8] = 0
        if n >= 2 and (b[1] & 0x7F) == 127 and n >= 10 and (b[1] >> 7):
            plen = int.from_bytes(bytes(b[2:10]), "big")
            if (14 + plen) % (1 << 64) < plen:
                continue  # masked wrap: reference is UB here
        outs = []
        for lib, fn in ((rl, rl.websocketframeDecode), (ol, ol.ws_oracle_decode)):
            buf = (C.c_ubyte * max(1, n)).from_buffer_copy(b.tobytes() if n else b"\0")
            d, dl, f, t = C.c_void_p(1), C.c_ulonglong(2), C.c_int(3), C.c_int(4)
            r = fn(buf, n, C.byref(d), C.byref(dl), C.byref(f), C.byref(t))
            dv = None if d.value in (None, 1) else d.value - C.addressof(buf)
            outs.append((r, dv, dl.value, f.value, t.value, bytes(buf)))
        assert outs[0] == outs[1], i


def test_oracle_encode_composition_roundtrip():
    """the encode composition used as the batch-encode checker: its masked frames decode
    (oracle a5 loop) back to the source payloads with websocketframeEncode's header fields"""
    import wsynth  # noqa: F401  (tests/ on sys.path)
    from oracle_lib import oracle_encode_frames, oracle_segments
    from util_amd.wsframe import ENC_DTYPE
    rng = np.random.default_rng(5)
    lens = [0, 1, 5, 125, 126, 127, 1000, 65535, 65536, 70000, 3]
    src = rng.integers(0, 256, sum(lens) + 7, dtype=np.uint8)
    fr = np.zeros(len(lens), ENC_DTYPE)
    o = 7
    for i, n in enumerate(lens):
        fr[i] = (o, n, int(rng.integers(0, 2**32)), i % 3, i % 2, (i + 1) % 2, 1 if i % 4 else 0)
        o += n
    wire, offs = oracle_encode_frames(src, fr)
    buf = np.frombuffer(wire, dtype=np.uint8).copy()
    desc, res = oracle_segments(buf, [0], [len(buf)], len(lens))
    assert int(res[0]["n_frames"]) == len(lens) and int(res[0]["consumed"]) == len(buf)
    for i, n in enumerate(lens):
        d = desc[i]
        assert int(d["frame_off"]) == int(offs[i]) and int(d["datalen"]) == n
        assert int(d["masked"]) == int(fr[i]["masked"]) and int(d["is_fin"]) == int(fr[i]["is_fin"])
        assert int(d["type"]) == (int(fr[i]["type"]) if fr[i]["prev_is_fin"] else 0)
        if n:
            got = buf[int(d["data_off"]):int(d["data_off"]) + n]
            assert np.array_equal(got, src[int(fr[i]["src_off"]):int(fr[i]["src_off"]) + n])


def test_oracle_reassemble_delivery_rule():
    """the reassembly checker on a hand-built connection: [A no FIN][B FIN][C FIN][D no FIN]
    -> messages A+B, C (complete) and D (pending); a carried-in open message marks the first
    message `continued`; an error frame ends delivery"""
    from oracle_lib import oracle_reassemble

    def frame(b0, body, key=b"\x01\x02\x03\x04"):
        masked = bytes(x ^ key[i % 4] for i, x in enumerate(body))
        return bytes([b0, 0x80 | len(body)]) + key + masked
    wire = frame(0x02, b"alpha") + frame(0x80, b"beta") + frame(0x81, b"gamma") + frame(0x00, b"delta")
    w = np.frombuffer(wire, dtype=np.uint8)
    desc, res, msgs, regions, op = oracle_reassemble(w, [0], [len(wire)], 8)
    assert int(res[0]["n_frames"]) == 4 and int(res[0]["consumed"]) == len(wire)
    assert [m[1:] for m in msgs[0]] == [(9, 0, 2, 1, 0), (5, 2, 1, 1, 0), (5, 3, 1, 0, 0)]
    assert bytes(regions[0][1]) == b"alphabetagammadelta" and op[0] == 1
    _, _, msgs2, _, op2 = oracle_reassemble(w, [0], [len(wire)], 8, open_in=[1])
    assert msgs2[0][0][5] == 1 and msgs2[0][1][5] == 0
