"""GPU parity of the speculative piece path (util_amd/csrc/ws_spec.hip): the unmask kernel
predicts every segment's frame grid from its first header (no scan kernel in front), verifies
the headers it streams, and a repair kernel undoes and walks exactly every segment whose
prediction failed. Every case here is a prediction that fails somewhere (or a batch the
path must refuse), bit-exact against the oracle (oracle/ws_oracle.c, pinned to the
reference's websocketframe.c:112-165 under the reactor loop net_reactor.c:515-526):
payload bytes, descriptors of every decoded frame, segment results."""
import numpy as np
import pytest

import test_gpu_parity as P
from oracle_lib import oracle_segments, used_descs
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def forced_spec():
    """path 3, speculative whenever the batch fits (the repair handles every misprediction)"""
    W.set_option("path", 3)
    W.set_option("piece_spec", 2)
    yield
    W.set_option("path", -1)
    W.set_option("piece_spec", 0)
    W.set_option("spec_spins", 2048)
    W.set_option("spec_g", 0)


def frame(rng, plen, masked=True, form=None, b0=0x82):
    """one wire frame: websocketframeEncode's header forms (websocketframe.c:176-202), or a
    forced (non-minimal) form, MASK + key when masked"""
    form = form or (7 if plen < 126 else (16 if plen <= 0xFFFF else 64))
    m = 0x80 if masked else 0
    if form == 7:
        h = bytes([b0, m | plen])
    elif form == 16:
        h = bytes([b0, m | 126]) + plen.to_bytes(2, "big")
    else:
        h = bytes([b0, m | 127]) + plen.to_bytes(8, "big")
    if masked:
        h += rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
    return h + rng.integers(0, 256, plen, dtype=np.uint8).tobytes()


def batch(segments, rng, gap=True):
    """segments (lists of byte strings) back to back, with odd gaps between them"""
    blob, so, sl = bytearray(), [], []
    for parts in segments:
        if gap:
            blob += bytes(int(rng.integers(0, 9)))
        so.append(len(blob))
        seg = b"".join(parts)
        sl.append(len(seg))
        blob += seg
    return np.frombuffer(bytes(blob), dtype=np.uint8).copy(), so, sl


def spec_calls():
    return W.get_stat("piece_spec_calls")


def wirelen(plen, masked=True):
    return plen + (2 if plen < 126 else (4 if plen <= 0xFFFF else 10)) + (4 if masked else 0)


def check(dev, wire, so, sl, max_frames, tag, g, expect_spec=True, desc_base=None):
    """decode speculatively predicting frames of wire length g (the host's hint), vs the oracle"""
    W.set_option("spec_g", g)
    n0 = spec_calls()
    out = P.assert_same(dev, wire, so, sl, max_frames, desc_base=desc_base, tag=tag)
    if expect_spec:
        assert spec_calls() == n0 + 1, tag + ": the speculative path did not run"
    return out


ANOMALIES = ["longer", "shorter", "unmasked_same_wire", "form16_same_wire", "form64_same_wire", "unmasked_other",
             "garbage_header", "zero_payload"]


def anomalous(rng, kind, plen):
    if kind == "longer":
        return frame(rng, plen + 3)
    if kind == "shorter":
        return frame(rng, plen - 5)
    if kind == "unmasked_same_wire":               # same wire length: still on the grid, no XOR
        return frame(rng, plen + 4, masked=False)
    if kind == "form16_same_wire":                 # 2 more header bytes, 2 fewer payload bytes
        return frame(rng, plen - 2, form=16) if plen < 126 else frame(rng, plen - 6, form=64)
    if kind == "form64_same_wire":
        return frame(rng, plen - 8, form=64) if plen < 126 else frame(rng, plen - 6, form=64)
    if kind == "unmasked_other":
        return frame(rng, plen, masked=False)
    if kind == "garbage_header":
        return rng.integers(0, 256, plen + 8, dtype=np.uint8).tobytes()
    return frame(rng, 0)


@pytest.mark.parametrize("gap", [True, False], ids=["gaps", "contiguous"])
@pytest.mark.parametrize("kind", ANOMALIES)
@pytest.mark.parametrize("plen", [1000, 100, 4096, 2500, 70000])
def test_misprediction_at_every_frame_index(dev, kind, plen, gap):
    """16-frame segments of equal frames, segment j broken at frame 1 + j % 15 (every index
    1..15, several times), next to unbroken segments: every broken segment is repaired.
    Frames of >= 2 KiB take S1's fast path (its frames in scalar registers), across a
    segment boundary too when the segments are contiguous; 70000 B: the 64-bit length form"""
    rng = np.random.default_rng(ANOMALIES.index(kind) * 10007 + plen + gap)
    segs = []
    for j in range(96 if plen < 10000 else 30):
        parts = [frame(rng, plen) for _ in range(16)]
        if j % 3 != 2:
            parts[1 + j % 15] = anomalous(rng, kind, plen)
        segs.append(parts)
    wire, so, sl = batch(segs, rng, gap=gap)
    check(dev, wire, so, sl, 16, "%s plen %d" % (kind, plen), wirelen(plen))
    check(dev, wire, so, sl, 20, "%s plen %d max 20" % (kind, plen), wirelen(plen))


@pytest.mark.parametrize("plen", [700, 4096])
@pytest.mark.parametrize("tail", ["exact", "hdr1", "hdr5", "payload_short", "shorter_complete", "garbage",
                                  "longer_incomplete", "zero_frame"])
def test_segment_tails(dev, tail, plen):
    """what follows the last predicted frame: nothing, an incomplete header or payload (the
    reference stops, consumed excludes it), a complete shorter frame (misprediction), garbage;
    segments back to back (4096: S1's fast path reaches the tails' ranges)"""
    rng = np.random.default_rng(5 + plen)
    segs = []
    for j in range(80):
        n = 1 + j % 16
        parts = [frame(rng, plen) for _ in range(n)]
        extra = {"exact": b"", "hdr1": b"\x82", "hdr5": frame(rng, plen)[:5],
                 "payload_short": frame(rng, plen)[:plen - 200], "shorter_complete": frame(rng, 10),
                 "garbage": rng.integers(0, 256, 300, dtype=np.uint8).tobytes(),
                 "longer_incomplete": frame(rng, plen * 7)[:plen - 50], "zero_frame": frame(rng, 0)}[tail]
        segs.append(parts + [extra])
    wire, so, sl = batch(segs, rng, gap=plen == 700)
    check(dev, wire, so, sl, 17, tail, wirelen(plen))


@pytest.mark.parametrize("plen", [300, 3000])
@pytest.mark.parametrize("max_frames", [1, 2, 7, 16, 64])
def test_max_frames(dev, max_frames, plen):
    """segments of 16 equal frames (+ a partial one) under every descriptor capacity:
    MAX_FRAMES predicted exactly when frames remain (3000: the fast path, contiguous segments)"""
    rng = np.random.default_rng(max_frames + plen)
    segs = [[frame(rng, plen) for _ in range(16)] + ([frame(rng, plen)[:100]] if j % 2 else []) for j in range(64)]
    wire, so, sl = batch(segs, rng, gap=plen == 300)
    check(dev, wire, so, sl, max_frames, "max_frames %d" % max_frames, wirelen(plen))


def test_first_frame_quirks(dev):
    """first frames the speculation refuses (walked exactly): (int) return <= 0 cannot be built
    at test size, but wrap-fenced masked lengths, unmasked 64-bit lengths that wrap, and
    empty / 1-byte / header-only segments can"""
    rng = np.random.default_rng(8)
    wrap = bytes([0x82, 0x80 | 127]) + (2**64 - 4).to_bytes(8, "big") + bytes(4) + bytes(40)
    wrap_unmasked = bytes([0x82, 127]) + (2**64 - 8).to_bytes(8, "big") + frame(rng, 20) + frame(rng, 20)
    segs = [[wrap], [wrap_unmasked], [b""], [b"\x82"], [frame(rng, 50)[:6]], [frame(rng, 70) * 3],
            [frame(rng, 0) for _ in range(10)], [frame(rng, 1) for _ in range(40)]]
    wire, so, sl = batch(segs * 20, rng)
    for g in (wirelen(20), wirelen(0), wirelen(1), 2, 10):
        check(dev, wire, so, sl, 64, "quirks g %d" % g, g)


def test_garbage_and_random_streams(dev):
    """random bytes cut into segments, and the parity suite's random streams (mixed lengths,
    truncations, garbage tails): most segments mispredict"""
    rng = np.random.default_rng(21)
    n = 1 << 20
    wire = rng.integers(0, 256, n, dtype=np.uint8)
    cuts = np.sort(rng.choice(n, 3000, replace=False))
    check(dev, wire, [int(x) for x in cuts[:-1]], [int(b - a) for a, b in zip(cuts[:-1], cuts[1:])], 32, "garbage",
          100)
    wire, so, sl = P.random_stream(np.random.default_rng(22), 2000)
    for g in (6, 131, 1006, 4104):
        check(dev, wire, so, sl, 16, "random g %d" % g, g)


def test_unordered_and_out_of_range(dev):
    """the table checkers find an unordered table (or a segment past the declared length):
    nothing is stored by the speculation and the repair kernel walks every segment"""
    rng = np.random.default_rng(23)
    segs = [[frame(rng, 900) for _ in range(16)] for _ in range(200)]
    wire, so, sl = batch(segs, rng)
    perm = rng.permutation(len(so))
    check(dev, wire, [so[i] for i in perm], [sl[i] for i in perm], 16, "unordered", wirelen(900))
    so2, sl2 = list(so), list(sl)
    so2[50], so2[51] = so2[51], so2[50]
    sl2[50], sl2[51] = sl2[51], sl2[50]
    check(dev, wire, so2, sl2, 16, "one swap", wirelen(900))
    W.set_option("spec_g", wirelen(900))
    n = len(wire)
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    d[:n] = torch.from_numpy(wire).to(dev)
    so_t = torch.tensor(np.asarray(so, dtype=np.int64), device=dev)
    sl_t = torch.tensor(np.asarray(sl, dtype=np.int64), device=dev)
    desc = torch.zeros(len(so) * 16 * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(len(so) * 16, dtype=torch.uint8, device=dev)
    lib = W.load_lib()
    rc = lib.websocketframeBatchDecodeDevice(d.data_ptr(), so[-1] + sl[-1] - 10, so_t.data_ptr(), sl_t.data_ptr(),
                                             len(so), 16, None, desc.data_ptr(), res.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, 16)
    assert np.array_equal(res.cpu().numpy().view(W.SEGRES_DTYPE), orr)
    assert np.array_equal(d[:n].cpu().numpy(), ob)


def test_wrong_frame_length_hint(dev):
    """a hint that matches no segment (the previous call's frames were another size): every
    segment mispredicts at its first frame and is repaired"""
    rng = np.random.default_rng(70)
    wire, so, sl = batch([[frame(rng, 1000) for _ in range(16)] for _ in range(200)], rng)
    for g in (wirelen(4096), wirelen(999), wirelen(1001), 2, wirelen(1000) * 2):
        check(dev, wire, so, sl, 16, "hint %d" % g, g)


@pytest.mark.parametrize("spins", [0, 1])
def test_checker_give_up_path(dev, spins):
    """waves that stop waiting for the table checkers store nothing and tag their 4 KiB range;
    the repair undoes the speculative XOR only where it was stored, then walks exactly
    (spec_spins 0: most of the first waves give up)"""
    W.set_option("spec_spins", spins)
    rng = np.random.default_rng(30 + spins)
    segs = [[frame(rng, 4096) for _ in range(16)] for _ in range(300)]
    for j in range(0, 300, 7):
        segs[j][3 + j % 12] = frame(rng, 4000)
    wire, so, sl = batch(segs, rng)
    check(dev, wire, so, sl, 16, "spins %d" % spins, wirelen(4096))
    wire, so, sl = P.random_stream(np.random.default_rng(31), 1500)
    check(dev, wire, so, sl, 16, "spins %d random" % spins, 1006)


def test_desc_base_and_empty_segments(dev):
    rng = np.random.default_rng(40)
    segs = [[frame(rng, 333) for _ in range(1 + j % 9)] if j % 5 else [] for j in range(300)]
    for j in range(1, 300, 11):
        if segs[j]:
            segs[j][-1] = frame(rng, 30)
    wire, so, sl = batch(segs, rng, gap=False)
    base = (np.arange(len(so), dtype=np.int64)[::-1] * 10).copy()
    check(dev, wire, so, sl, 10, "desc_base", wirelen(333), desc_base=base)


def test_state_across_calls_and_shapes(dev):
    """the path's resting state (heads, mismatch flags) across calls on one stream whose segment
    count grows and shrinks, most segments mispredicting: a flag left set from an earlier shape
    would skip a repair; decoding twice restores the wire"""
    rng = np.random.default_rng(50)
    shapes = [200, 40, 400, 400, 100, 800]
    for i, nseg in enumerate(shapes):
        segs = [[frame(rng, 200) for _ in range(8)] for _ in range(nseg)]
        for j in range(nseg):
            if (j + i) % 2:
                segs[j][j % 7 + 1] = frame(rng, 150)
        wire, so, sl = batch(segs, rng)
        gb, gd, gr = check(dev, wire, so, sl, 8, "shape %d (%d)" % (i, nseg), wirelen(200))
        gb2, _, _ = P.gpu_decode(dev, gb.copy(), so, sl, 8)
        assert np.array_equal(gb2, wire), "decode twice"


def test_adaptive_choice(dev):
    """piece_spec 1 (adaptive; the default is 0): the first call on a stream takes the scan kernel, which
    advises the speculative path for a batch of equal frames of >= 48 KiB; a batch of mixed
    lengths makes the repair kernel advise the scan kernel again; equal frames below 48 KiB
    stay on the scan kernel (profiles/r03_spec_sweep.log). Every call bit-exact."""
    W.set_option("piece_spec", 1)
    W.set_option("spec_g", 0)
    rng = np.random.default_rng(60)
    stream = torch.cuda.Stream(dev)
    uni = batch([[frame(rng, 50000) for _ in range(4)] for _ in range(40)], rng)
    small = batch([[frame(rng, 2000) for _ in range(16)] for _ in range(200)], rng)
    mixed = P.random_stream(np.random.default_rng(61), 600)
    seq = [(uni, False), (uni, True), (uni, True), (mixed, True), (mixed, False), (mixed, False), (uni, False),
           (uni, True), (small, True), (small, False), (small, False), (uni, False), (uni, True)]
    with torch.cuda.stream(stream):
        for k, ((wire, so, sl), want_spec) in enumerate(seq):
            n0 = spec_calls()
            P.assert_same(dev, wire, so, sl, 16, tag="call %d" % k)
            torch.cuda.synchronize()
            assert (spec_calls() == n0 + 1) == want_spec, "call %d: speculative=%s" % (k, not want_spec)
