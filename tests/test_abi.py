"""C-ABI checks that need no GPU: libwsframe_amd.so loads, exports every symbol
include/wsframe_amd.h declares, and its host half (the eight reference symbols)
matches the reference's golden vectors. No compute call touches a GPU here."""
import ctypes as C
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

import util_amd
from util_amd import _lib
from util_amd import wsframe as W

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


REF_INC = "/root/reference/inc"


def header_symbols(*names):
    out = set()
    for n in names or ("wsframe_amd.h", "wsframe_amd_channel.h"):
        src = open(os.path.join(REPO, "include", n)).read()
        out |= set(re.findall(r"WSFRAME_AMD_EXPORT[^;]*?\b(websocketframe\w+)\s*\(", src, re.S))
    return sorted(out)


def dynamic_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_exports_exactly_the_declared_symbols():
    """libwsframe_amd.so's dynamic symbol table is its C ABI and nothing else: the reference's
    eight symbols + the batch / glue API of include/wsframe_amd.h + wsframe_amd_channel.h (no
    kernel stubs, no bench or calibration entry points, no C++ symbols)"""
    lib = util_amd.load_lib()
    declared = header_symbols()
    assert len(declared) == 20
    assert sorted(_lib.EXPORTS) == declared
    assert dynamic_symbols(_lib.LIB_PATH) == set(declared)
    for s in declared:
        assert getattr(lib, s) is not None
    bench = header_symbols("wsframe_amd_bench.h")
    assert sorted(_lib.BENCH_EXPORTS) == bench
    assert dynamic_symbols(_lib.BENCH_LIB_PATH) == set(bench)
    _lib.load_bench_lib()


def test_reference_signature_set():
    """the eight reference symbols (websocketframe.h:42-49) are all there"""
    ref8 = {"websocketframeComputeSecAccept", "websocketframeDecodeHandshakeRequest",
            "websocketframeEncodeHandshakeResponse", "websocketframeEncodeHandshakeResponseWithProtocol",
            "websocketframeFreeString", "websocketframeDecode", "websocketframeEncodeHeadLength",
            "websocketframeEncode"}
    assert ref8 <= set(header_symbols())


def test_host_decode_single(golden):
    for c in golden("decode_single.json"):
        wire = bytes.fromhex(c["input"])
        buf = bytearray(wire if wire else b"\0")
        r, doff, dl, fin, typ = W.websocketframeDecode(buf, c["len"])
        assert r == c["ret"], c["name"]
        if c["data_off"] == "untouched":
            assert doff is None and dl is None, c["name"]
        else:
            assert (doff, dl, fin, typ) == (c["data_off"], c["datalen"], c["fin"], c["type"]), c["name"]
        assert hashlib.sha256(bytes(buf[: len(wire)])).hexdigest() == c["output_sha256"], c["name"]


def test_host_decode_loop_segments(golden):
    """the host symbol driven by the reactor loop reproduces the segment fixtures"""
    for c in golden("decode_segments.json"):
        buf = bytearray(bytes.fromhex(c["input"]))
        for so, sl, sg in zip(c["seg_off"], c["seg_len"], c["segments"]):
            off, nf, frames = 0, 0, []
            while off < sl and nf < c["max_frames"]:
                r, doff, dl, fin, typ = W.websocketframeDecode(buf, sl - off, so + off)
                if r == 0:
                    break
                frames.append((r, doff, dl, fin, typ))
                nf += 1
                if r < 0:
                    break
                off += r & 0xFFFFFFFF
            exp = [(f["ret"], f["data_off"], f["datalen"], f["fin"], f["type"]) for f in sg["frames"]]
            if sg["status"] == -2:
                continue
            assert frames == exp, c["name"]
            assert off == sg["consumed"], c["name"]
        assert hashlib.sha256(bytes(buf)).hexdigest() == c["output_sha256"], c["name"]


def test_host_encode(golden):
    for c in golden("handshake.json")["encode_header"]:
        assert W.websocketframeEncodeHeadLength(c["datalen"]) == c["headlen"]
        assert W.websocketframeEncode(c["is_fin"], c["prev_is_fin"], c["type"], c["datalen"]).hex() == c["head"]


def test_host_handshake(golden):
    hs = golden("handshake.json")
    for c in hs["sec_accept"]:
        assert W.websocketframeComputeSecAccept(c["key"].encode()) == c["accept"], c["key"]
    assert W.websocketframeComputeSecAccept(b"dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="
    for c in hs["decode_request"]:
        got = W.websocketframeDecodeHandshakeRequest(c["request"].encode())
        exp = (c["ret"], c["sec_key_off"], c["sec_key_len"], c["sec_protocol_off"], c["sec_protocol_len"])
        assert got == exp, c["request"]
    for c in hs["encode_response"]:
        assert W.websocketframeEncodeHandshakeResponse(c["accept"].encode()) == c["response"]
        proto = None if c["protocol"] is None else c["protocol"].encode()
        assert W.websocketframeEncodeHandshakeResponseWithProtocol(c["accept"].encode(), proto) == \
            c["response_with_protocol"]


def test_struct_layout():
    assert C.sizeof(_lib.WsDesc) == 32 and C.sizeof(_lib.WsSegRes) == 16
    assert W.DESC_DTYPE.itemsize == 32
    assert np.dtype(W.SEGRES_DTYPE).itemsize == 16


def test_host_decode_word_xor_matches_bytewise():
    """host unmask (8-byte words) vs a byte loop at every alignment and length"""
    rng = np.random.default_rng(1)
    for align in range(8):
        for plen in (0, 1, 7, 8, 9, 15, 16, 17, 125, 126, 300, 4096, 65536, 70001):
            key = rng.integers(0, 256, 4, dtype=np.uint8)
            pay = rng.integers(0, 256, plen, dtype=np.uint8)
            hl = 2 if plen < 126 else (4 if plen <= 0xFFFF else 10)
            h = bytearray([0x82])
            if hl == 2:
                h.append(0x80 | plen)
            elif hl == 4:
                h += bytes([0x80 | 126]) + plen.to_bytes(2, "big")
            else:
                h += bytes([0x80 | 127]) + plen.to_bytes(8, "big")
            frame = bytes(h) + key.tobytes() + (pay ^ np.resize(key, plen)).tobytes()
            buf = bytearray(align) + bytearray(frame)
            r, doff, dl, fin, typ = W.websocketframeDecode(buf, len(frame), align)
            assert r == len(frame) and dl == plen
            assert bytes(buf[align + hl + 4:]) == pay.tobytes()


def _build_run(tmp_path, src, name, extra, expect):
    util_amd.load_lib()
    exe = str(tmp_path / name)
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror"] + extra +
                   ["-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "c", src), "-L", libdir,
                    "-lwsframe_amd", "-Wl,-rpath," + libdir, "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == expect


def test_c_program_links_and_runs(tmp_path):
    """a C caller of the reference API (tests/c/drop_in.c), compiled against
    include/wsframe_amd.h and linked to libwsframe_amd.so in place of websocketframe.c"""
    _build_run(tmp_path, "drop_in.c", "drop_in", [], "drop_in ok")


def test_c_program_reference_header(tmp_path):
    """the same caller compiled against the REFERENCE's own header
    (inc/crt/protocol/websocketframe.h: enum, WEBSOCKET_MAX_ENCODE_HEADLENGTH, the two handshake
    request templates, the eight prototypes) links to libwsframe_amd.so unchanged"""
    if not os.path.isdir(REF_INC):
        pytest.skip("reference headers not present (GPU box)")
    _build_run(tmp_path, "drop_in.c", "drop_in_ref",
               ["-I", REF_INC, '-DWS_API_HEADER="crt/protocol/websocketframe.h"', "-Wno-unused-function"], "drop_in ok")


def test_channel_glue_layout(tmp_path):
    """include/wsframe_amd_channel.h against the reference's net_channel_ex.h: identical
    NetChannelInbufDecodeResult_t layout, websocketframeOnDecode assignable to
    NetChannelExProc_t.on_decode, NETPACKET_FRAGMENT value; the glue runs"""
    if not os.path.isdir(REF_INC):
        pytest.skip("reference headers not present (GPU box)")
    _build_run(tmp_path, "channel_layout.c", "channel_layout", ["-I", REF_INC, "-D_GNU_SOURCE", "-Wno-unused-function"],
               "channel_layout ok")


class _DecodeResult(C.Structure):          # NetChannelInbufDecodeResult_t (net_channel_ex.h:10-20)
    _fields_ = [("err", C.c_char), ("incomplete", C.c_char), ("fragment_eof", C.c_char), ("pktype", C.c_char),
                ("ignore", C.c_char), ("pkseq", C.c_uint), ("decodelen", C.c_uint), ("bodylen", C.c_uint),
                ("bodyptr", C.c_void_p)]


class _Cursor(C.Structure):                 # WebsocketBatchCursor_t (include/wsframe_amd_channel.h)
    _fields_ = [("desc", C.c_void_p), ("consumed", C.c_ulonglong), ("n_frames", C.c_uint), ("status", C.c_int),
                ("seg_off", C.c_ulonglong), ("inbuf", C.c_void_p), ("next", C.c_uint)]


def _reactor_loop(buf, on_decode):
    """the reactor loop over one inbuf (net_reactor.c:515-526) with an on_decode glue:
    what the stream hook sees, as (body offset, bodylen, fragment_eof, pktype, decodelen)"""
    base = buf.ctypes.data
    off, out = 0, []
    while off < len(buf):
        r = _DecodeResult()
        on_decode(base + off, len(buf) - off, C.byref(r))
        if r.err != b"\x00":
            out.append("err")
            break
        if r.incomplete != b"\x00":
            break
        out.append(((r.bodyptr or base) - base, r.bodylen, r.fragment_eof, r.pktype, r.decodelen))
        off += r.decodelen
    return out, off


@pytest.mark.parametrize("case", ["mixed", "overflow_count", "zero_len", "tail"])
def test_channel_glue_batch_replay(case):
    """websocketframeOnDecodeBatch replays a batch decode's descriptors (here the oracle's,
    bit-identical to the GPU's) to the reactor loop exactly as websocketframeOnDecode's
    per-frame decode drives it: same bodies, lengths, FIN flags, packet types and stop"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import reasm_cases as R
    from oracle_lib import oracle_segments
    lib = util_amd.load_lib()
    lib.websocketframeOnDecodeBatch.restype = None
    lib.websocketframeOnDecodeBatch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    wire, _ = R.build(case)
    single = wire.copy()
    ref, ref_off = _reactor_loop(single, lambda p, n, r: lib.websocketframeOnDecode(None, p, n, r))
    batch = wire.copy()
    od, orr = oracle_segments(batch, [0], [len(batch)], 1 << 16)     # the batch decode, in place
    desc = np.ascontiguousarray(od[:int(orr[0]["n_frames"])])
    cur = _Cursor(desc.ctypes.data, int(orr[0]["consumed"]), int(orr[0]["n_frames"]), int(orr[0]["status"]), 0,
                  batch.ctypes.data, 0)
    got, got_off = _reactor_loop(batch, lambda p, n, r: lib.websocketframeOnDecodeBatch(C.byref(cur), p, n, r))
    assert got == ref and got_off == ref_off
    assert np.array_equal(batch[:ref_off], single[:ref_off])


OPTION_CHECK = r"""
import sys
sys.path.insert(0, sys.argv[1])
from util_amd import wsframe as W
names = sys.argv[2].split(",")
VAL = {"stream_rw_cmax": 20}                              # (16..26)
bad = [n for n in names if W.load_lib().websocketframeGpuSetOption(n.encode(), VAL.get(n, 1)) != 0]
unknown_ok = W.load_lib().websocketframeGpuSetOption(b"no_such_option", 1) == 0
print("BAD", bad, "UNKNOWN_ACCEPTED", unknown_ok)
sys.exit(1 if bad or unknown_ok else 0)
"""


def test_documented_options_are_accepted():
    """every tuning knob the header documents for websocketframeGpuSetOption is accepted by the
    library and an unknown name is refused (checked in a child process: setting options is
    process-global state)"""
    hdr = open(os.path.join(_lib.REPO, "include", "wsframe_amd.h")).read()
    block = hdr[hdr.index("/* Launch tuning knobs"):hdr.index("WSFRAME_AMD_EXPORT int websocketframeGpuSetOption")]
    names = sorted(set(re.findall(r'"([a-z0-9_]+)"', block)))
    assert "piece_lds" in names and "reasm_cfg" in names and "piece_spec" not in names, names
    util_amd.load_lib()
    r = subprocess.run([os.environ.get("PYTHON", "python3"), "-c", OPTION_CHECK, _lib.REPO, ",".join(names)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
