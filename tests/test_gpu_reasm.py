"""GPU parity of websocketframeBatchReassembleDevice(Ex) (fused decode + message reassembly,
SURVEY §8a row a6) against the reference's own rx stack (tests/golden/reassemble.json: the
reactor + stream hook + fragment cache compiled from the reference, oracle/reactor_harness.c)
and against the oracle composition (tests/oracle_lib.py: oracle_reassemble = the pinned
decode oracle + the delivery rule + the cache limit, itself pinned to that fixture),
bit-exact: descriptors, segment results, message descriptors, gathered bodies, open state,
cached bytes; the wire must come back untouched."""
import numpy as np
import pytest

import bench
from oracle_lib import oracle_reassemble, used_descs
from test_gpu_parity import random_stream
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# reasm_path 1: fused one-workgroup-per-segment kernel (ws_reasm_seg_kernel, LDS windows),
# 2: scan + layout + gather kernels; 0 (auto) picks by batch shape
@pytest.fixture(params=[1, 2], ids=["fused", "three_kernel"], autouse=True)
def reasm_path(request):
    W.set_option("reasm_path", request.param)
    yield request.param
    W.set_option("reasm_path", 0)


def gpu_reassemble(dev, wire, so, sl, max_frames, open_in=None, out_off=None, out_size=None, readcache_max=0,
                   cached_in=None):
    n = len(wire)
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    if n:
        d[:n] = torch.from_numpy(wire).to(dev)
    nseg = len(so)
    T = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=dev)  # noqa: E731
    out = torch.full(((out_size or n) + 64,), 0xEE, dtype=torch.uint8, device=dev)
    desc = torch.full((max(1, nseg * max_frames) * 32,), 0xEE, dtype=torch.uint8, device=dev)
    msg = torch.full((max(1, nseg * max_frames) * 32,), 0xEE, dtype=torch.uint8, device=dev)
    res = torch.zeros(max(1, nseg) * 16, dtype=torch.uint8, device=dev)
    nmsg = torch.zeros(max(1, nseg), dtype=torch.int32, device=dev)
    op = None if open_in is None else torch.tensor(np.asarray(open_in, dtype=np.uint8), device=dev)
    ca = None if cached_in is None else torch.tensor(np.asarray(cached_in, dtype=np.uint32).view(np.int32), device=dev)
    W.batch_reassemble_device(d, T(so), T(sl), max_frames, desc, res, out, msg, nmsg,
                              out_off=None if out_off is None else T(out_off), open_state=op,
                              readcache_max=readcache_max, cached=ca)
    torch.cuda.synchronize()
    assert np.array_equal(d[:n].cpu().numpy(), wire), "wire buffer modified"
    return (out.cpu().numpy(), desc.cpu().numpy().view(W.DESC_DTYPE), res.cpu().numpy().view(W.SEGRES_DTYPE)[:nseg],
            msg.cpu().numpy().view(W.MSG_DTYPE), nmsg.cpu().numpy()[:nseg],
            None if op is None else op.cpu().numpy(), None if ca is None else ca.cpu().numpy().view(np.uint32))


def check(dev, wire, so, sl, mf, open_in=None, out_off=None, out_size=None, tag="", readcache_max=0, cached_in=None):
    out, gd, gr, gm, gn, gop, gca = gpu_reassemble(dev, wire, so, sl, mf, open_in, out_off, out_size, readcache_max,
                                                   cached_in)
    od, orr, oms, oreg, oop, oca = oracle_reassemble(wire, so, sl, mf, open_in, out_off, readcache_max, cached_in)
    assert np.array_equal(gr, orr), tag
    assert np.array_equal(used_descs(gd, gr, mf), used_descs(od, orr, mf)), tag
    for s in range(len(so)):
        assert int(gn[s]) == len(oms[s]), (tag, s)
        for i, m in enumerate(oms[s]):
            g = gm[s * mf + i]
            assert tuple(int(g[f]) for f in W.MSG_DTYPE.names) == m, (tag, s, i)
        ob, body = oreg[s]
        assert np.array_equal(out[ob:ob + len(body)], body), (tag, s)
    if open_in is not None:
        assert np.array_equal(gop, oop), tag
    if cached_in is not None:
        assert np.array_equal(gca, oca), tag
    return out, oms, oop


@pytest.mark.parametrize("seed,mf", [(1, 16), (2, 4), (3, 1), (4, 64)])
def test_reassemble_random_vs_oracle(dev, seed, mf):
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 1500)
    out, _, _ = check(dev, wire, so, sl, mf, tag="seed %d" % seed)
    # bytes between the gathered bodies of different segments stay untouched
    covered = np.zeros(len(wire) + 64, bool)
    _, _, _, oreg, _, _ = oracle_reassemble(wire, so, sl, mf)
    for ob, body in oreg:
        covered[ob:ob + len(body)] = True
    assert (out[~covered] == 0xEE).all()


@pytest.mark.parametrize("cfg", [1, 2])
def test_reassemble_fused_geometries(dev, reasm_path, cfg):
    """the fused kernel's other geometries (reasm_cfg 1: the compiler's occupancy, 2: 19 KiB
    windows; default 0 = 8 waves/SIMD) give the same results, cache limit included"""
    if reasm_path != 1:
        pytest.skip("fused kernel option")
    W.set_option("reasm_cfg", cfg)
    try:
        rng = np.random.default_rng(40 + cfg)
        wire, so, sl = random_stream(rng, 1200)
        check(dev, wire, so, sl, 16, tag="reasm_cfg %d" % cfg)
        check(dev, wire, so, sl, 16, tag="reasm_cfg %d limit" % cfg, readcache_max=3000)
    finally:
        W.set_option("reasm_cfg", 0)


def test_reassemble_carry_open_state(dev):
    """two batches per connection: the open state out of batch 1 is the state into batch 2"""
    rng = np.random.default_rng(21)
    wire, so, sl = random_stream(rng, 800)
    open0 = rng.integers(0, 2, len(so)).astype(np.uint8)
    check(dev, wire, so, sl, 16, open_in=open0, tag="carry-in")


def test_reassemble_out_regions_elsewhere(dev):
    """explicit output offsets (regions in a separate, larger buffer, in reverse order)"""
    rng = np.random.default_rng(22)
    wire, so, sl = random_stream(rng, 500)
    caps = np.asarray(sl, dtype=np.int64)
    out_off = np.zeros(len(so), np.int64)
    o = 5
    for s in reversed(range(len(so))):
        out_off[s] = o
        o += int(caps[s]) + 3
    check(dev, wire, so, sl, 16, out_off=out_off, out_size=o + 16, tag="out_off")


def test_reassemble_cfg5_shape(dev):
    """cfg5's layout (16 x 1 KiB fragments per message, one message per rx segment) at
    reduced size: every message complete, 16 KiB contiguous, equal to the oracle's"""
    wl = bench.Workload.make("cfg5", dev, nframes=16 * 4096)
    wire = wl.buf[:wl.wire_bytes].cpu().numpy().copy()
    out, oms, _ = check(dev, wire, wl.seg_off_h, wl.seg_len_h, 16, tag="cfg5")
    assert all(len(m) == 1 and m[0][4] == 1 and m[0][1] == 16 * 1024 for m in oms)


@pytest.mark.parametrize("swin", [-1, 0, 1, 2])
def test_reassemble_segment_windows(dev, reasm_path, swin):
    """the fused kernel's segment windows (seg_win: 2^k windows streamed side by side, -1 the
    default 8) over 2,101 cfg5-shaped segments — the last window's spare blocks store nothing"""
    if reasm_path != 1:
        pytest.skip("fused kernel option")
    W.set_option("seg_win", swin)
    try:
        wl = bench.Workload.make("cfg5", dev, nframes=16 * 2101)
        wire = wl.buf[:wl.wire_bytes].cpu().numpy().copy()
        check(dev, wire, wl.seg_off_h, wl.seg_len_h, 16, tag="seg_win %d" % swin)
    finally:
        W.set_option("seg_win", -1)


def _frame(rng, plen, masked=True, b0=0x82, form=None):
    key = rng.integers(0, 256, 4, dtype=np.uint8) if masked else None
    form = form or (7 if plen < 126 else (16 if plen <= 0xFFFF else 64))
    h = bytearray([b0])
    m = 0x80 if masked else 0
    if form == 7:
        h.append(m | plen)
    elif form == 16:
        h += bytes([m | 126]) + plen.to_bytes(2, "big")
    else:
        h += bytes([m | 127]) + plen.to_bytes(8, "big")
    if masked:
        h += key.tobytes()
    return bytes(h) + rng.integers(0, 256, plen, dtype=np.uint8).tobytes()


def _segments(parts_list, rng, gaps=True):
    blob, so, sl = bytearray(), [], []
    for parts in parts_list:
        if gaps:
            blob += bytes(int(rng.integers(0, 20)))
        so.append(len(blob))
        seg = b"".join(parts)
        blob += seg
        sl.append(len(seg))
    return np.frombuffer(bytes(blob), dtype=np.uint8).copy(), so, sl


def test_reassemble_frames_across_windows(dev):
    """frames much longer than the fused kernel's 20 KiB LDS window, headers straddling
    window edges, fragments with FIN only at the end, at every alignment"""
    rng = np.random.default_rng(31)
    segs = []
    for i in range(64):
        n = int(rng.integers(1, 8))
        parts = []
        for k in range(n):
            plen = int(rng.choice([20475, 20470, 20480, 40960 + 3, 65536, 70000, 100, 0, 1]))
            b0 = (0x80 if k == n - 1 else 0) | (2 if k == 0 else 0)
            parts.append(_frame(rng, plen, masked=rng.random() < 0.9, b0=b0))
        segs.append(parts)
    wire, so, sl = _segments(segs, rng)
    check(dev, wire, so, sl, 16, tag="windows")


def test_reassemble_tiny_frames_max64(dev):
    """many 0-3 byte bodies per segment (64 frames per walk round), max_frames 64"""
    rng = np.random.default_rng(32)
    segs = [[_frame(rng, int(rng.integers(0, 4)), masked=rng.random() < 0.8,
                    b0=0x80 if rng.random() < 0.3 else 0) for _ in range(int(rng.integers(0, 90)))]
            for _ in range(300)]
    wire, so, sl = _segments(segs, rng)
    check(dev, wire, so, sl, 64, tag="tiny")


def test_reassemble_length_quirks(dev):
    """u64 length wrap of an unmasked frame (websocketframe.c:149: consumed, body larger
    than the segment -> WEBSOCKET_SEG_ERR_OUT_SPACE), masked wrap (fence), non-minimal
    length forms, a ret < 0 frame is impossible below 2 GiB, so decode errors come only
    from the fence"""
    rng = np.random.default_rng(33)
    # 10 + len wraps to 4: the reactor consumes 4 bytes and walks on inside the header
    wrap = bytes([0x82, 127]) + ((1 << 64) - 6).to_bytes(8, "big") + bytes(range(14))
    mwrap = bytes([0x82, 0xFF]) + ((1 << 64) - 14 + 5).to_bytes(8, "big") + bytes(range(14))
    segs = []
    for i in range(200):
        parts = []
        for _ in range(int(rng.integers(0, 5))):
            plen = int(rng.integers(0, 300))
            forms = [7, 16, 64] if plen < 126 else [16, 64]
            parts.append(_frame(rng, plen, form=int(rng.choice(forms)) if i % 3 else None))
        if i % 4 == 1:
            parts.insert(int(rng.integers(0, len(parts) + 1)), wrap)
        if i % 4 == 2:
            parts.insert(int(rng.integers(0, len(parts) + 1)), mwrap)
        segs.append(parts)
    wire, so, sl = _segments(segs, rng)
    _, orr, _, _, _, _ = oracle_reassemble(wire, so, sl, 16)
    assert (orr["status"] == -3).any() and (orr["status"] == -2).any()
    check(dev, wire, so, sl, 16, tag="quirks")


@pytest.mark.parametrize("total", [(1 << 31) + 6, 1 << 32])
def test_reassemble_int_truncation_real_size(dev, total):
    """a frame whose length sum reaches 2^31 (negative (int) return: descriptor, decode error,
    no body) or exactly 2^32 (return 0: not consumed) at its real size, vs the oracle"""
    plen = total - 14
    n = total + 100
    block = np.random.default_rng(8).integers(0, 256, (1 << 20) + 7, dtype=np.uint8)
    wire = np.empty(n, dtype=np.uint8)
    for a in range(0, n, len(block)):
        wire[a:a + len(block)] = block[:n - a]
    wire[:14] = np.frombuffer(bytes([0x02, 0x80 | 127]) + plen.to_bytes(8, "big") + bytes([1, 2, 3, 4]), dtype=np.uint8)
    _, oms, _ = check(dev, wire, [0], [n], 4, out_size=1 << 20, tag="int truncation")
    assert oms == [[]]


# ------------------------------------------------------------------ the reference's own deliveries

def _gpu_reactor_view(dev, wire, max_frames, limit):
    """the stream decoded on the GPU batch after batch (each batch = the bytes from the previous
    batch's `consumed` on, at most max_frames frames), d_open / d_cached carried across batches:
    the reference reactor's view (complete messages, consumed, frames, detach error, pending,
    cached) of the whole stream"""
    pos, frames, lens, bodies = 0, 0, [], []
    op, ca = [0], [0]
    carry = np.zeros(0, np.uint8)
    while True:
        seg = wire[pos:]
        out, gd, gr, gm, gn, op, ca = gpu_reassemble(dev, seg, [0], [len(seg)], max_frames, open_in=op,
                                                     readcache_max=limit, cached_in=ca)
        for i in range(int(gn[0])):
            m = gm[i]
            part = out[int(m["out_off"]):int(m["out_off"]) + int(m["len"])]
            whole = np.concatenate([carry, part]) if int(m["continued"]) else part
            if int(m["complete"]):
                lens.append(len(whole))
                bodies.append(whole)
                carry = np.zeros(0, np.uint8)
            else:
                carry = whole
        st = int(gr[0]["status"])
        pos += int(gr[0]["consumed"])
        frames += int(gr[0]["n_frames"]) - (1 if st == -4 else 0)
        if st != 1:
            return (lens, np.concatenate(bodies) if bodies else np.zeros(0, np.uint8), pos, frames,
                    7 if st == -4 else 0, int(op[0]), int(ca[0]))


@pytest.mark.parametrize("mf", [16, 64, 0], ids=["mf16", "mf64", "whole"])
def test_reassemble_reference_reactor_fixture(dev, golden, reasm_path, mf):
    """every stream of tests/golden/reassemble.json (cfg5 shape, mixed messages with pings inside
    fragmented ones, open at the end, incomplete tail, fragment-cache overflow at the limit and
    past it, FIN frames that skip the check, empty fragments): the GPU delivers exactly what the
    reference's own reactor delivered — message lengths, body bytes (SHA-256), bytes and frames
    consumed, the detach, the cache state at the end. mf 0 = the whole stream as one segment
    (three-kernel path only: the fused kernel holds <= 64 frames per segment)."""
    import reasm_cases as R
    if mf == 0 and reasm_path == 1:
        pytest.skip("fused path: max_frames <= 64")
    for c in golden("reassemble.json"):
        wire, limit = R.build(c["name"])
        assert R.sha256(wire) == c["wire_sha256"]
        lens, bodies, consumed, frames, det, pend, cached = _gpu_reactor_view(dev, wire, mf or c["frames"] + 2, limit)
        assert lens == c["msg_lens"], c["name"]
        assert R.sha256(bodies) == c["bodies_sha256"], c["name"]
        assert (consumed, frames, det, pend, cached) == (c["consumed"], c["frames"], c["detach_error"], c["pending"],
                                                         c["cached"]), c["name"]


@pytest.mark.parametrize("limit", [1, 700, 4096, 65536])
def test_reassemble_cache_limit_random_vs_oracle(dev, limit):
    """many connections per batch, random fragmented streams, open/cached state carried in,
    every readcache_max_size regime: bit-exact vs the oracle (pinned to the reference reactor)"""
    rng = np.random.default_rng(40 + limit)
    wire, so, sl = random_stream(rng, 1200)
    open0 = rng.integers(0, 2, len(so)).astype(np.uint8)
    cached0 = np.where(open0 == 1, rng.integers(0, 2 * limit, len(so)), 0).astype(np.uint32)
    od, orr, _, _, _, _ = oracle_reassemble(wire, so, sl, 16, open0, None, limit, cached0)
    assert (orr["status"] == -4).any(), "the limit never triggered: the case tests nothing"
    check(dev, wire, so, sl, 16, open_in=open0, readcache_max=limit, cached_in=cached0, tag="limit %d" % limit)


@pytest.mark.parametrize("limit,overflow", [(16 * 1024, False), (16 * 1024 - 1, True)], ids=["fits", "one_byte_short"])
def test_reassemble_cfg5_cache_limit_full_size(dev, limit, overflow):
    """cfg5 at full size (262,144 messages of 16 x 1 KiB) under a fragment-cache limit: a
    16 KiB limit holds every message (the FIN fragment brings the cache to exactly the limit:
    no overflow); one byte less refuses every segment's 16th fragment
    (WEBSOCKET_SEG_ERR_CACHE_OVERFLOW, 15 frames consumed; the open message is reported
    incomplete, never delivered); a reduced size is compared with the oracle frame for frame"""
    wl = bench.Workload.make("cfg5", dev)
    n, nseg = wl.wire_bytes, wl.nseg
    out = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    desc = torch.empty(nseg * 16 * 32, dtype=torch.uint8, device=dev)
    msg = torch.empty(nseg * 16 * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(nseg * 16, dtype=torch.uint8, device=dev)
    nmsg = torch.zeros(nseg, dtype=torch.int32, device=dev)
    op = torch.zeros(nseg, dtype=torch.uint8, device=dev)
    ca = torch.zeros(nseg, dtype=torch.int32, device=dev)
    W.batch_reassemble_device(wl.buf, wl.seg_off, wl.seg_len, 16, desc, res, out, msg, nmsg, open_state=op,
                              readcache_max=limit, cached=ca)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(W.SEGRES_DTYPE)
    nm = nmsg.cpu().numpy()
    cached = ca.cpu().numpy().view(np.uint32)
    fw = 1024 + 8                                                   # a 1 KiB fragment on the wire
    if overflow:
        assert (r["status"] == W.SEG_ERR_CACHE_OVERFLOW).all() and (r["n_frames"] == 16).all()
        assert (r["consumed"] == 15 * fw).all() and (nm == 1).all()
        m = msg.cpu().numpy().view(W.MSG_DTYPE).reshape(nseg, 16)[:, 0]
        assert (m["complete"] == 0).all() and (m["len"] == 15 * 1024).all()
    else:
        assert (r["status"] == W.SEG_OK).all() and (r["n_frames"] == 16).all() and (nm == 1).all()
        assert (r["consumed"] == 16 * fw).all() and (cached == 0).all() and (op.cpu().numpy() == 0).all()
        m = msg.cpu().numpy().view(W.MSG_DTYPE).reshape(nseg, 16)[:, 0]
        assert (m["len"] == 16 * 1024).all() and (m["complete"] == 1).all()
    # frame for frame against the oracle on the first 512 segments
    k = 512
    wire = wl.buf[:int(wl.seg_off_h[k])].cpu().numpy().copy()
    check(dev, wire, wl.seg_off_h[:k], wl.seg_len_h[:k], 16, tag="cfg5 limit", readcache_max=limit,
          cached_in=[0] * k)
