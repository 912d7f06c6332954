"""Python mirror of the websocketframe API (inc/crt/protocol/websocketframe.h:10-49)
and of the batch API (include/wsframe_amd.h Part 2), over libwsframe_amd.so.

Host functions take a mutable ``bytearray``/numpy uint8 buffer and behave like
the C functions (same argument meaning, same return conventions: >0 bytes
consumed, 0 incomplete, <0 error). Batch functions take torch CUDA tensors and
only pass raw device pointers and the current HIP stream to the C ABI.
"""
import ctypes as C

import numpy as np

from ._lib import WsDesc, WsSegRes, check, check_bench, load_bench_lib, load_lib

WEBSOCKET_CONTINUE_FRAME = 0
WEBSOCKET_TEXT_FRAME = 1
WEBSOCKET_BINARY_FRAME = 2
WEBSOCKET_CLOSE_FRAME = 8
WEBSOCKET_PING_FRAME = 9
WEBSOCKET_PONG_FRAME = 10
WEBSOCKET_MAX_ENCODE_HEADLENGTH = 10

SEG_OK, SEG_MAX_FRAMES, SEG_ERR_DECODE, SEG_ERR_LEN_WRAP = 0, 1, -1, -2
SEG_ERR_OUT_SPACE = -3
SEG_ERR_CACHE_OVERFLOW = -4
NETPACKET_FRAGMENT = 6  # transport_ctx.h:11-18; the pktype websocketframeOnDecode reports
DATA_OFF_NULL = 0xFFFFFFFFFFFFFFFF
BATCH_PAD = 32  # WEBSOCKET_BATCH_PAD: readable device bytes required after every segment

DESC_DTYPE = np.dtype([("frame_off", "<u8"), ("data_off", "<u8"), ("datalen", "<u8"), ("ret", "<i4"),
                       ("is_fin", "u1"), ("type", "u1"), ("masked", "u1"), ("hdrlen", "u1")])
SEGRES_DTYPE = np.dtype([("consumed", "<u8"), ("n_frames", "<u4"), ("status", "<i4")])
MSG_DTYPE = np.dtype([("out_off", "<u8"), ("len", "<u8"), ("first_frame", "<u4"), ("n_frames", "<u4"),
                      ("complete", "<u4"), ("continued", "<u4")])
assert MSG_DTYPE.itemsize == 32
ENC_DTYPE = np.dtype([("src_off", "<u8"), ("len", "<u8"), ("mask_key", "<u4"), ("type", "u1"), ("is_fin", "u1"),
                      ("prev_is_fin", "u1"), ("masked", "u1")])
assert ENC_DTYPE.itemsize == 24
assert DESC_DTYPE.itemsize == C.sizeof(WsDesc) == 32
assert SEGRES_DTYPE.itemsize == C.sizeof(WsSegRes) == 16


def _addr(buf):
    """address of a writable host buffer (bytearray or numpy array)"""
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    return C.addressof((C.c_char * len(buf)).from_buffer(buf))


# ------------------------------------------------------------------ host, one frame

def websocketframeDecode(buf, length=None, offset=0):
    """websocketframe.c:112-165 on buf[offset:offset+length], in place.

    Returns (ret, data_off, datalen, is_fin, type); data_off is the payload offset
    into ``buf`` (None where the C function sets *data = NULL). Out-params the C
    function leaves untouched (ret 0) come back as None.
    """
    lib = load_lib()
    if length is None:
        length = len(buf) - offset
    sent = 0xA5A5A5A5A5A5A5A5
    data, datalen, fin, typ = C.c_void_p(sent), C.c_ulonglong(sent), C.c_int(-7), C.c_int(-7)
    base = _addr(buf) if len(buf) else 0
    r = lib.websocketframeDecode(base + offset, length, C.byref(data), C.byref(datalen), C.byref(fin), C.byref(typ))
    if data.value == sent:
        return r, None, None, None, None
    doff = None if data.value is None else data.value - base
    return r, doff, datalen.value, fin.value, typ.value


def websocketframeEncodeHeadLength(datalen):
    return load_lib().websocketframeEncodeHeadLength(datalen)


def websocketframeEncode(is_fin, prev_is_fin, type_, datalen):
    """websocketframe.c:176-202; returns the header bytes"""
    lib = load_lib()
    h = (C.c_ubyte * WEBSOCKET_MAX_ENCODE_HEADLENGTH)()
    lib.websocketframeEncode(h, is_fin, prev_is_fin, type_, datalen)
    return bytes(h)[: lib.websocketframeEncodeHeadLength(datalen)]


def websocketframeComputeSecAccept(sec_key):
    lib = load_lib()
    out = C.create_string_buffer(60)
    r = lib.websocketframeComputeSecAccept(sec_key, len(sec_key), out)
    return out.value.decode() if r else None


def websocketframeDecodeHandshakeRequest(data):
    """returns (ret, sec_key_off, sec_key_len, sec_protocol_off, sec_protocol_len); offsets
    into ``data`` or None (NULL) / "untouched" when the C function does not write them"""
    lib = load_lib()
    buf = C.create_string_buffer(bytes(data), len(data))
    sent = 0xA5A5A5A5A5A5A5A5
    sk, skl, sp, spl = C.c_void_p(sent), C.c_uint(777), C.c_void_p(sent), C.c_uint(777)
    r = lib.websocketframeDecodeHandshakeRequest(buf, len(data), C.byref(sk), C.byref(skl), C.byref(sp), C.byref(spl))
    base = C.addressof(buf)

    def off(p):
        return "untouched" if p.value == sent else (None if p.value is None else p.value - base)
    return r, off(sk), skl.value, off(sp), spl.value


def websocketframeEncodeHandshakeResponse(sec_accept):
    lib = load_lib()
    out = C.create_string_buffer(162)
    return C.string_at(lib.websocketframeEncodeHandshakeResponse(sec_accept, len(sec_accept), out)).decode()


def websocketframeEncodeHandshakeResponseWithProtocol(sec_accept, sec_protocol):
    lib = load_lib()
    p = lib.websocketframeEncodeHandshakeResponseWithProtocol(
        sec_accept, len(sec_accept), sec_protocol, len(sec_protocol) if sec_protocol else 0)
    if not p:
        return None
    s = C.string_at(p).decode()
    lib.websocketframeFreeString(p)
    return s


# ------------------------------------------------------------------ batch, device

def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def batch_decode_device(buf, seg_off, seg_len, max_frames, desc, res, desc_base=None, stream=None):
    """websocketframeBatchDecodeDevice on torch CUDA tensors (uint8 buf, int64 seg_off/
    seg_len/desc_base, desc: uint8 [>= 32*slots], res: uint8 [16*nseg]); async on `stream`."""
    nseg = seg_off.numel()
    assert buf.numel() >= BATCH_PAD, "device batch needs WEBSOCKET_BATCH_PAD bytes of slack"
    assert seg_len.numel() == nseg and res.numel() * res.element_size() >= 16 * nseg
    if desc_base is None:
        assert desc.numel() * desc.element_size() >= 32 * nseg * max_frames, "desc holds < nseg*max_frames slots"
    assert buf.is_cuda and seg_off.is_cuda and seg_len.is_cuda and desc.is_cuda and res.is_cuda
    # buflen: segments lie in [0, numel - PAD); the last PAD bytes are the readable slack
    rc = load_lib().websocketframeBatchDecodeDevice(_ptr(buf), buf.numel() - BATCH_PAD, _ptr(seg_off), _ptr(seg_len),
                                                    nseg, max_frames, _ptr(desc_base), _ptr(desc), _ptr(res),
                                                    _stream(stream))
    check(rc, "websocketframeBatchDecodeDevice")


def stream_decode_device(buf, length, max_frames, desc, res, stream=None):
    """websocketframeStreamDecodeDevice: one raw stream buf[0:length) (uint8 CUDA tensor with
    >= BATCH_PAD bytes after it), decoded in place; asynchronous on `stream` (graph-capturable;
    an eager call on a stream of >= 512 KiB reads the pass state back)."""
    assert buf.numel() >= length + BATCH_PAD
    rc = load_lib().websocketframeStreamDecodeDevice(_ptr(buf), length, max_frames, _ptr(desc), _ptr(res),
                                                     _stream(stream))
    check(rc, "websocketframeStreamDecodeDevice")


def batch_reassemble_device(buf, seg_off, seg_len, max_frames, desc, res, out, msg, nmsg, out_off=None, open_state=None,
                            stream=None, readcache_max=0, cached=None):
    """websocketframeBatchReassembleDeviceEx on torch CUDA tensors: buf (uint8, wire, read only;
    the last BATCH_PAD bytes are slack), seg_off/seg_len/out_off (int64), desc (uint8
    >= 32*nseg*max_frames), res (uint8 16*nseg), out (uint8), msg (uint8 >= 32*nseg*max_frames),
    nmsg (int32 nseg), open_state (uint8 nseg, in/out, optional), readcache_max (the channel's
    readcache_max_size, 0 = unlimited), cached (int32 nseg, in/out, optional: the pending
    message's cached bytes, u32); async on `stream`."""
    nseg = seg_off.numel()
    assert buf.numel() >= BATCH_PAD and seg_len.numel() == nseg and nmsg.numel() >= nseg
    assert desc.numel() * desc.element_size() >= 32 * nseg * max_frames
    assert msg.numel() * msg.element_size() >= 32 * nseg * max_frames
    assert res.numel() * res.element_size() >= 16 * nseg
    assert cached is None or cached.numel() * cached.element_size() >= 4 * nseg
    rc = load_lib().websocketframeBatchReassembleDeviceEx(
        _ptr(buf), buf.numel() - BATCH_PAD, _ptr(seg_off), _ptr(seg_len), nseg, max_frames, _ptr(desc), _ptr(res),
        _ptr(out), _ptr(out_off), _ptr(msg), _ptr(nmsg), _ptr(open_state), int(readcache_max), _ptr(cached),
        _stream(stream))
    check(rc, "websocketframeBatchReassembleDeviceEx")


def batch_encode_device(src, frames, dst, wire_off, capacity=None, stream=None):
    """websocketframeBatchEncodeDevice on torch CUDA tensors: src (uint8 payload bytes),
    frames (uint8 tensor holding ENC_DTYPE records), dst (uint8), wire_off (int64,
    nframes + 1); async on `stream`. capacity defaults to dst.numel()."""
    n = frames.numel() // ENC_DTYPE.itemsize
    assert wire_off.numel() >= n + 1
    cap = dst.numel() if capacity is None else capacity
    rc = load_lib().websocketframeBatchEncodeDevice(_ptr(src), _ptr(frames), n, _ptr(dst), cap, _ptr(wire_off),
                                                    _stream(stream))
    check(rc, "websocketframeBatchEncodeDevice")


def batch_decode_host(buf, seg_off, seg_len, max_frames, device=0):
    """websocketframeBatchDecodeHost: buf (numpy uint8, modified in place), seg_off/seg_len
    (numpy uint64). Returns (desc structured array [nseg*max_frames], res [nseg])."""
    nseg = len(seg_off)
    seg_off = np.ascontiguousarray(seg_off, dtype=np.uint64)
    seg_len = np.ascontiguousarray(seg_len, dtype=np.uint64)
    desc = np.zeros(max(1, nseg * max_frames), dtype=DESC_DTYPE)
    res = np.zeros(max(1, nseg), dtype=SEGRES_DTYPE)
    rc = load_lib().websocketframeBatchDecodeHost(buf.ctypes.data, buf.nbytes, seg_off.ctypes.data,
                                                  seg_len.ctypes.data, nseg, max_frames, desc.ctypes.data,
                                                  res.ctypes.data, device)
    check(rc, "websocketframeBatchDecodeHost")
    return desc, res[:nseg]


def batch_decode_host_multi(buf, seg_off, seg_len, max_frames, devices):
    """websocketframeBatchDecodeHostMulti: buf (numpy uint8, modified in place) decoded on several
    devices (a byte-balanced range each; a device may repeat). Returns (desc, res) as
    batch_decode_host does."""
    nseg = len(seg_off)
    seg_off = np.ascontiguousarray(seg_off, dtype=np.uint64)
    seg_len = np.ascontiguousarray(seg_len, dtype=np.uint64)
    desc = np.zeros(max(1, nseg * max_frames), dtype=DESC_DTYPE)
    res = np.zeros(max(1, nseg), dtype=SEGRES_DTYPE)
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    rc = load_lib().websocketframeBatchDecodeHostMulti(buf.ctypes.data, buf.nbytes, seg_off.ctypes.data,
                                                       seg_len.ctypes.data, nseg, max_frames, desc.ctypes.data,
                                                       res.ctypes.data, devs.ctypes.data, len(devs))
    check(rc, "websocketframeBatchDecodeHostMulti")
    return desc, res[:nseg]


def synth_device(buf, frame_off, nframes, plen_kind, fixed_len, b0_kind, seed, stream=None, first_frame=0):
    """websocketframeSynthDeviceRange (libwsframe_amd_bench.so): bench/test input generated in
    HBM — generator frames first_frame .. first_frame + nframes - 1 at buf + frame_off[i]"""
    rc = load_bench_lib().websocketframeSynthDeviceRange(_ptr(buf), _ptr(frame_off), first_frame, nframes, plen_kind,
                                                         fixed_len, b0_kind, seed, _stream(stream))
    check_bench(rc, "websocketframeSynthDeviceRange")


def synth_verify_device(buf, frame_off, nframes, plen_kind, fixed_len, seed, expect_plain, mismatch, stream=None,
                        first_frame=0):
    rc = load_bench_lib().websocketframeSynthVerifyDeviceRange(_ptr(buf), _ptr(frame_off), first_frame, nframes,
                                                               plen_kind, fixed_len, seed, 1 if expect_plain else 0,
                                                               _ptr(mismatch), _stream(stream))
    check_bench(rc, "websocketframeSynthVerifyDeviceRange")


def frame_hash_device(buf, desc, res, nseg, max_frames, out, stream=None):
    """websocketframeFrameHashDevice: adds the decoded batch's output hash into out (int64 CUDA
    tensor, one element, u64 wrap-around)"""
    rc = load_bench_lib().websocketframeFrameHashDevice(_ptr(buf), _ptr(desc), _ptr(res), nseg, max_frames, _ptr(out),
                                                        _stream(stream))
    check_bench(rc, "websocketframeFrameHashDevice")


def set_option(name, value):
    """websocketframeGpuSetOption (launch tuning knobs, for A/B measurement)"""
    rc = load_lib().websocketframeGpuSetOption(name.encode(), int(value))
    if rc != 0:
        raise ValueError("unknown option %r" % name)


def get_stat(name):
    """websocketframeGpuGetStat (diagnostic counters of the most recent call)"""
    v = C.c_ulonglong(0)
    if load_lib().websocketframeGpuGetStat(name.encode(), C.byref(v)) != 0:
        raise ValueError("unknown stat %r" % name)
    return int(v.value)
