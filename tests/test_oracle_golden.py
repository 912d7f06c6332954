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
    desc, res, msgs, regions, op, _ = oracle_reassemble(w, [0], [len(wire)], 8)
    assert int(res[0]["n_frames"]) == 4 and int(res[0]["consumed"]) == len(wire)
    assert [m[1:] for m in msgs[0]] == [(9, 0, 2, 1, 0), (5, 2, 1, 1, 0), (5, 3, 1, 0, 0)]
    assert bytes(regions[0][1]) == b"alphabetagammadelta" and op[0] == 1
    _, _, msgs2, _, op2, _ = oracle_reassemble(w, [0], [len(wire)], 8, open_in=[1])
    assert msgs2[0][0][5] == 1 and msgs2[0][1][5] == 0


# ------------------------------------------------------------------ reassembly, pinned to the
# reference's own rx stack (tests/golden/reassemble.json, made by tests/golden/make_reasm_golden.py
# from NetReactor_handle -> on_read_stream -> fragment cache -> on_recv, oracle/reactor_harness.c)

def _reasm_cases(golden):
    import reasm_cases as R
    for c in golden("reassemble.json"):
        wire, limit = R.build(c["name"])
        assert R.sha256(wire) == c["wire_sha256"] and len(wire) == c["wire_len"], c["name"]  # stream pinned
        assert limit == c["readcache_max"]
        yield c, wire


def _fixture_view(c):
    return (c["msg_lens"], c["bodies_sha256"], c["consumed"], c["frames"], c["detach_error"], c["pending"], c["cached"])


def _view_digest(v):
    import reasm_cases as R
    lens, bodies, consumed, frames, det, pend, cached = v
    return (lens, R.sha256(bodies), consumed, frames, det, pend, cached)


def test_reassemble_fixture_vs_oracle(golden):
    """the reassembly checker (oracle_reassemble: decode oracle + delivery rule + cache limit) on
    each whole stream as one rx segment reproduces the reference reactor's deliveries exactly"""
    from oracle_lib import oracle_reassemble, reactor_view
    n = 0
    for c, wire in _reasm_cases(golden):
        mf = c["frames"] + 2
        _, res, msgs, regions, op, cached = oracle_reassemble(wire, [0], [len(wire)], mf,
                                                             readcache_max=c["readcache_max"])
        assert _view_digest(reactor_view(msgs, regions, res, op, cached)) == tuple(_fixture_view(c)), c["name"]
        n += 1
    assert n == 10


def oracle_reassemble_batches(wire, max_frames, limit):
    """the stream decoded batch after batch (each batch: the bytes from the previous batch's
    `consumed` on, max_frames frames at most), open state and cached bytes carried across
    batches; returns the reference-reactor view of the whole stream"""
    from oracle_lib import oracle_reassemble
    pos, frames, lens, bodies = 0, 0, [], []
    op, cached = [0], [0]
    carry = np.zeros(0, np.uint8)                     # the pending message's bytes from earlier batches
    while True:
        seg = wire[pos:]
        _, res, msgs, regions, op, cached = oracle_reassemble(seg, [0], [len(seg)], max_frames, open_in=op,
                                                             out_off=[0], readcache_max=limit, cached_in=cached)
        ob, body = regions[0]
        for (o, n, _f, _k, complete, cont) in msgs[0]:
            part = body[int(o):int(o) + int(n)]
            whole = np.concatenate([carry, part]) if cont else part
            if complete:
                lens.append(len(whole))
                bodies.append(whole)
                carry = np.zeros(0, np.uint8)
            else:
                carry = whole
        st = int(res[0]["status"])
        pos += int(res[0]["consumed"])
        frames += int(res[0]["n_frames"]) - (1 if st == -4 else 0)
        if st != 1:                                   # anything but MAX_FRAMES ends the stream
            return (lens, np.concatenate(bodies) if bodies else np.zeros(0, np.uint8), pos, frames,
                    7 if st == -4 else 0, int(op[0]), int(cached[0]))


@pytest.mark.parametrize("mf", [1, 16, 64])
def test_reassemble_fixture_batches_vs_oracle(golden, mf):
    """the same streams cut into batches of at most `mf` frames, state carried across batches
    (d_open / d_cached): deliveries identical to the reference reactor's"""
    for c, wire in _reasm_cases(golden):
        if mf == 1 and len(wire) > 3000000:
            continue
        v = oracle_reassemble_batches(wire, mf, c["readcache_max"])
        assert _view_digest(v) == tuple(_fixture_view(c)), (c["name"], mf)


def _reference_reactor():
    import ref_reactor
    if not ref_reactor.available():
        pytest.skip("reference build not present (GPU box): tests/golden/reassemble.json carries the pin")
    return ref_reactor


def test_reference_reactor_fuzz_vs_oracle():
    """dev container only: random streams with random cache limits through the reference's own
    reactor vs the reassembly checker"""
    X = _reference_reactor()
    import reasm_cases as R
    from oracle_lib import oracle_reassemble, reactor_view
    rng = np.random.default_rng(99)
    for i in range(150):
        parts = []
        for _ in range(int(rng.integers(0, 25))):
            nfr = int(rng.integers(1, 6))
            sizes = [int(rng.choice([0, 1, 50, 125, 126, 700, 3000, 20000])) for _ in range(nfr)]
            parts.append(R.message(rng, sizes, masked=rng.random() < 0.8, opcode=int(rng.integers(0, 3))))
            if rng.random() < 0.2:
                parts.append(R.frame(rng, int(rng.choice([0x89, 0x8A, 0x00, 0x02])), int(rng.integers(0, 125))))
        wire = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
        if rng.random() < 0.3 and len(wire):
            wire = wire[:int(rng.integers(0, len(wire)))]
        limit = int(rng.choice([0, 0, 100, 1000, 5000, 30000]))
        r = X.reactor_deliver(wire, int(rng.choice([3, 100, 4096, 1 << 20])), limit)
        _, res, msgs, regions, op, cached = oracle_reassemble(wire, [0], [len(wire)], r["frames"] + 2,
                                                             readcache_max=limit)
        v = reactor_view(msgs, regions, res, op, cached)
        assert v[0] == r["lens"] and np.array_equal(v[1], r["bodies"]), i
        assert v[2:] == (r["consumed"], r["frames"], r["detach_error"], r["pending"], r["cached"]), i


def test_reference_reactor_with_amd_glue(golden):
    """the drop-in at the plugin seam: the reference's reactor + stream hook with
    NetChannelExProc_t.on_decode = libwsframe_amd.so's websocketframeOnDecode (our host decode
    and glue, include/wsframe_amd_channel.h) delivers exactly what it delivers with the
    reference's own websocketframeDecode (the fixture)"""
    X = _reference_reactor()
    import reasm_cases as R
    from util_amd import load_lib
    glue = C.cast(load_lib().websocketframeOnDecode, C.c_void_p).value
    for c, wire in _reasm_cases(golden):
        r = X.reactor_deliver(wire, 1500, c["readcache_max"], on_decode=glue)
        v = (r["lens"], R.sha256(r["bodies"]), r["consumed"], r["frames"], r["detach_error"], r["pending"], r["cached"])
        assert v == tuple(_fixture_view(c)), c["name"]


def test_reference_reactor_with_batch_glue(golden, tmp_path):
    """the GPU integration at the plugin seam: a channel's inbuf decoded as a batch (here by
    the oracle, bit-identical to the GPU's batch decode) is read by the reference's own
    reactor, whose on_decode replays the batch's descriptors through libwsframe_amd.so's
    websocketframeOnDecodeBatch — the deliveries (fragment cache, limit, detach included)
    are the fixture's, i.e. the reference's own websocketframeDecode's. Streams that arrive
    in one read (the cursor covers one inbuf fill)."""
    import os
    import subprocess
    import reasm_cases as R
    from oracle_lib import oracle_segments
    from util_amd import load_lib
    X = _reference_reactor()
    lib = load_lib()
    here = os.path.dirname(os.path.abspath(__file__))
    so_path = str(tmp_path / "libtramp.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", os.path.join(os.path.dirname(here), "include"),
                    os.path.join(here, "c", "batch_glue_tramp.c"), "-o", so_path,
                    "-L", os.path.dirname(lib._name), "-lwsframe_amd", "-Wl,-rpath," + os.path.dirname(lib._name)],
                   check=True)
    tr = C.CDLL(so_path)
    tr.tramp_set.argtypes = [C.c_void_p, C.c_uint, C.c_ulonglong, C.c_int]
    glue = C.cast(tr.tramp_on_decode, C.c_void_p).value
    done = 0
    for c, wire in _reasm_cases(golden):
        if len(wire) > 64 << 10:
            continue
        dec = wire.copy()
        od, orr = oracle_segments(dec, [0], [len(dec)], 1 << 16)      # the batch decode, in place
        desc = np.ascontiguousarray(od[:max(1, int(orr[0]["n_frames"]))])
        tr.tramp_set(desc.ctypes.data, int(orr[0]["n_frames"]), int(orr[0]["consumed"]), int(orr[0]["status"]))
        r = X.reactor_deliver(dec, len(dec) + 1, c["readcache_max"], on_decode=glue)
        v = (r["lens"], R.sha256(r["bodies"]), r["consumed"], r["frames"], r["detach_error"], r["pending"], r["cached"])
        assert v == tuple(_fixture_view(c)), c["name"]
        done += 1
    assert done >= 5


def _batched_reactor_check(golden, chunk, gpu_fn=None, oracle_fn=None, max_frames=64):
    """every fixture stream as one connection of a multi-connection batched reactor (grouped by
    readcache_max_size): deliveries equal the reference reactor's own (the fixture)"""
    import ref_reactor
    from util_amd import load_lib
    replay = C.cast(load_lib().websocketframeOnDecodeBatch, C.c_void_p).value
    groups = {}
    for c, wire in _reasm_cases(golden):
        groups.setdefault(c["readcache_max"], []).append((c, wire))
    total_batches = 0
    for limit, cases in sorted(groups.items()):
        res, nb = ref_reactor.reactor_deliver_batched([w for _, w in cases], chunk, limit, max_frames, gpu_fn=gpu_fn,
                                                      oracle_fn=oracle_fn, replay_fn=replay)
        total_batches += nb
        for (c, _), r in zip(cases, res):
            v = (r["lens"], _view_digest((r["lens"], r["bodies"], 0, 0, 0, 0, 0))[1], r["consumed"], r["frames"],
                 r["detach_error"], r["pending"], r["cached"])
            assert v == tuple(_fixture_view(c)), (c["name"], chunk)
    return total_batches


@pytest.mark.parametrize("chunk,max_frames", [(7, 64), (100, 64), (1500, 64), (65536, 64), (65536, 3)])
def test_batched_reactor_binding_oracle(golden, chunk, max_frames):
    """INTEGRATION.md §2 over the reference's own reactor and stream hook: recv for every
    readable connection, ONE batch decode (here the oracle's, bit-identical to the GPU's) over
    their whole inbufs — each starting with the previous read's undecoded tail — then each
    connection's on_read loop replaying the batch through websocketframeOnDecodeBatch. The
    streams arrive in `chunk`-byte writes, so frames and headers split across reads; a small
    descriptor capacity makes the glue decode the frames past it on the host (MAX_FRAMES)."""
    _reference_reactor()
    olib = load_oracle()
    fn = C.cast(olib.ws_oracle_decode_segments, C.c_void_p).value
    assert _batched_reactor_check(golden, chunk, oracle_fn=fn, max_frames=max_frames) > 0
