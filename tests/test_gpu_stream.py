"""GPU parity of websocketframeStreamDecodeDevice (one raw stream, grid-wide speculative
frame-boundary discovery + the piece path's unmask) against the oracle's reactor loop
over the single segment [0, len): bit-exact buffer, descriptors and result."""
import numpy as np
import pytest

import wsynth
from oracle_lib import oracle_segments
from test_gpu_parity import random_stream
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def run(dev, wire, max_frames, shift=0):
    n = len(wire)
    d = torch.zeros(n + shift + 64, dtype=torch.uint8, device=dev)
    d[shift:shift + n] = torch.from_numpy(wire).to(dev)
    desc = torch.full((max(1, max_frames) * 32,), 0xEE, dtype=torch.uint8, device=dev)
    res = torch.zeros(16, dtype=torch.uint8, device=dev)
    W.stream_decode_device(d[shift:], n, max_frames, desc, res)
    torch.cuda.synchronize()
    gb = d[shift:shift + n].cpu().numpy()
    gr = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
    gd = desc.cpu().numpy().view(W.DESC_DTYPE)[:int(gr["n_frames"])]
    ob = wire.copy()
    od, orr = oracle_segments(ob, [0], [n], max_frames)
    assert tuple(gr) == tuple(orr[0])
    assert np.array_equal(gd, od[:int(orr[0]["n_frames"])])
    if not np.array_equal(gb, ob):
        bad = np.nonzero(gb != ob)[0]
        raise AssertionError("%d bytes differ, first at %d" % (len(bad), bad[0]))
    return gr


@pytest.mark.parametrize("shift", [0, 5])
def test_stream_uniform(dev, shift):
    wire, off, pl, plain = wsynth.make_batch(20000, 0, 4096, 0, 3)
    r = run(dev, wire, 1 << 15, shift)
    assert int(r["n_frames"]) == 20000 and int(r["consumed"]) == len(wire)


def test_stream_runs_of_lengths(dev):
    """runs of equal lengths: one pass per change"""
    parts = []
    for i, (n, fl) in enumerate([(3000, 125), (700, 1500), (40, 65536), (1, 7), (5000, 0), (900, 300)]):
        w, *_ = wsynth.make_batch(n, 0, fl, 0, 10 + i)
        parts.append(w)
    wire = np.concatenate(parts)
    r = run(dev, wire, 1 << 14)
    assert int(r["n_frames"]) == 3000 + 700 + 40 + 1 + 5000 + 900


def test_stream_random_and_truncated(dev):
    """lengths changing every frame (the single-wavefront walk), garbage, truncated tail"""
    for seed in (1, 2, 3):
        rng = np.random.default_rng(seed)
        wire, so, sl = random_stream(rng, 300)
        run(dev, wire, 4096)


def test_stream_max_frames(dev):
    wire, *_ = wsynth.make_batch(5000, 0, 1000, 0, 4)
    r = run(dev, wire, 1234)
    assert int(r["n_frames"]) == 1234 and int(r["status"]) == W.SEG_MAX_FRAMES


# --- long streams whose lengths change every frame: the chunk-parallel walk ------------------
# (ws_stream.hip R1-R3; streams of >= 16 MiB after the grid passes stop paying)

def long_stream(rng, nbytes, pick, masked=0.999, b0=None, payload=None):
    """frames back to back until about nbytes: pick(rng) -> payload length; b0 None = a
    client opcode (text/binary/continuation, FIN random); payload(rng, n) -> bytes"""
    parts, total = [], 0
    while total < nbytes:
        plen = int(pick(rng))
        key = rng.integers(0, 256, 4, dtype=np.uint8) if rng.random() < masked else None
        first = b0 if b0 is not None else int(rng.choice([0x00, 0x01, 0x02, 0x80, 0x81, 0x82, 0x89, 0x8A]))
        m = 0x80 if key is not None else 0
        if plen < 126:
            h = bytes([first, m | plen])
        elif plen <= 0xFFFF:
            h = bytes([first, m | 126]) + plen.to_bytes(2, "big")
        else:
            h = bytes([first, m | 127]) + plen.to_bytes(8, "big")
        if key is not None:
            h += key.tobytes()
        body = payload(rng, plen) if payload else rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        parts.append(h + body)
        total += len(h) + plen
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy()


def mix3(rng):
    return rng.choice([125, 1500, 65536])


@pytest.fixture
def serial_walk():
    """the same stream through the one-wavefront walk, for a before/after check"""
    W.set_option("stream_rw", 0)
    yield
    W.set_option("stream_rw", 1)


@pytest.mark.parametrize("shift", [0, 3])
def test_long_stream_cfg3_mix(dev, shift):
    """the cfg3 length mix as one 48 MiB client stream (16 MiB chunks)"""
    wire = long_stream(np.random.default_rng(21), 48 << 20, mix3, masked=1.0)
    W.set_option("stream_rw", 2)                  # the host follows the records: its counters
    try:
        r = run(dev, wire, 1 << 16, shift)
    finally:
        W.set_option("stream_rw", 1)
    assert int(r["consumed"]) == len(wire) and int(r["status"]) == W.SEG_OK
    # every chunk from the speculative records (no one-wavefront chunk walks; an unmasked
    # frame in a client stream would end its chunk's speculation)
    assert W.get_stat("stream_rw_chunks") >= 3 and W.get_stat("stream_rw_chunk_walks") == 0


def test_long_stream_small_frames(dev):
    """0..300 B frames: chunks shrink to keep about a thousand frames each"""
    wire = long_stream(np.random.default_rng(22), 20 << 20, lambda g: g.integers(0, 301))
    r = run(dev, wire, 1 << 18)
    assert int(r["consumed"]) == len(wire)


def test_long_stream_frames_longer_than_window(dev):
    """frames of 100 KiB - 1 MiB: chunk entries outside the candidate window, chunk walks"""
    wire = long_stream(np.random.default_rng(23), 40 << 20, lambda g: g.integers(100 << 10, 1 << 20))
    r = run(dev, wire, 1 << 12)
    assert int(r["consumed"]) == len(wire)


def test_long_stream_rare_long_frames(dev):
    """small frames with a rare 200-400 KiB one: the sample (first 256 KiB) rarely sees one, so
    the chunk windows (from the sample's mean and longest frame) are far shorter than the frames
    that cover some of them: those chunks are walked by one wavefront; eager and captured"""
    def pick(g):
        return int(g.integers(200 << 10, 400 << 10)) if g.random() < 0.004 else int(g.integers(0, 301))
    wire = long_stream(np.random.default_rng(27), 24 << 20, pick)
    r = run(dev, wire, 1 << 18)
    assert int(r["consumed"]) == len(wire)
    n = len(wire)
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    desc = torch.zeros((1 << 18) * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(16, dtype=torch.uint8, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        W.stream_decode_device(d, n, 1 << 18, desc, res)
    ob = wire.copy()
    od, orr = oracle_segments(ob, [0], [n], 1 << 18)
    for rnd in range(2):
        d[:n].copy_(torch.from_numpy(wire).to(dev))
        g.replay()
        torch.cuda.synchronize()
        gr = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
        assert tuple(gr) == tuple(orr[0]), rnd
        assert np.array_equal(desc.cpu().numpy().view(W.DESC_DTYPE)[:int(gr["n_frames"])],
                              od[:int(orr[0]["n_frames"])]), rnd
        assert np.array_equal(d[:n].cpu().numpy(), ob), rnd


def test_long_stream_unmasked_and_mixed(dev):
    """server frames (no MASK) and a stream that mixes both"""
    run(dev, long_stream(np.random.default_rng(24), 24 << 20, mix3, masked=0.0), 1 << 14)
    run(dev, long_stream(np.random.default_rng(25), 24 << 20, mix3, masked=0.7), 1 << 14)


@pytest.mark.parametrize("kind", ["server_zeros", "client_0x80", "partly_dense"])
def test_long_stream_dense_candidates(dev, kind):
    """payloads whose every position reads as a plausible header (zero bytes in a server
    stream, 0x80 bytes in a client one): R1's waves with more candidates than they stage
    (RW_WCAP) and chunk lists with more survivors than slots"""
    pick = lambda g: g.integers(2000, 40000)
    if kind == "server_zeros":
        wire = long_stream(np.random.default_rng(31), 20 << 20, pick, masked=0.0, payload=lambda g, n: bytes(n))
    elif kind == "client_0x80":
        wire = long_stream(np.random.default_rng(32), 20 << 20, pick, masked=1.0, payload=lambda g, n: b"\x80" * n)
    else:
        def some(g, n):
            return b"\x80" * n if g.random() < 0.3 else g.integers(0, 256, n, dtype=np.uint8).tobytes()
        wire = long_stream(np.random.default_rng(33), 20 << 20, pick, masked=1.0, payload=some)
    r = run(dev, wire, 1 << 14)
    assert int(r["consumed"]) == len(wire)


def test_long_stream_nested_frames(dev):
    """payloads made of valid client frames: speculative walks that look like the chain
    (slot overflow, merged walks) must not change the result"""
    def inner(rng, n):
        out = bytearray()
        while len(out) < n:
            k = int(rng.integers(0, 120))
            out += bytes([0x82, 0x80 | k]) + rng.integers(0, 256, 4 + k, dtype=np.uint8).tobytes()
        return bytes(out[:n])
    wire = long_stream(np.random.default_rng(26), 24 << 20, lambda g: g.integers(2000, 40000), payload=inner)
    r = run(dev, wire, 1 << 14)
    assert int(r["consumed"]) == len(wire)


@pytest.mark.parametrize("cut", ["max_frames", "truncated", "garbage", "error"])
def test_long_stream_endings(dev, cut):
    """the walk ending inside the parallel part: MAX_FRAMES, an incomplete last frame,
    random bytes inserted mid-stream, a LEN_WRAP / decode-error header mid-stream"""
    rng = np.random.default_rng(27)
    wire = long_stream(rng, 32 << 20, mix3)
    max_frames = 1 << 16
    if cut == "max_frames":
        max_frames = 1200
    elif cut == "truncated":
        wire = wire[:len(wire) - 1000].copy()
    elif cut == "garbage":
        at = 20 << 20
        wire = np.concatenate([wire[:at], rng.integers(0, 256, 37, dtype=np.uint8), wire[at:]])
    else:
        # a 64-bit length with the top bit set at the first frame start after 25 MiB
        od, orr = oracle_segments(wire.copy(), [0], [len(wire)], 1 << 16)
        fo = od["frame_off"][:int(orr[0]["n_frames"])]
        at = int(fo[np.searchsorted(fo, 25 << 20)])
        bad = bytes([0x82, 0xFF]) + (0xFFFFFFFFFFFFFFF0).to_bytes(8, "big") + bytes(4)
        wire = np.concatenate([wire[:at], np.frombuffer(bad, dtype=np.uint8), wire[at:]])
    run(dev, wire, max_frames)


def _cut_stream(cut, rng, wire, keep_len=False):
    """the stream `wire` ended inside the parallel walk by `cut` (max_frames is the caller's);
    keep_len: the same length (a captured call's length is fixed)"""
    if cut == "truncated" and not keep_len:
        return wire[:len(wire) - 1000].copy()
    w = wire.copy()
    if cut == "garbage":
        at = 20 << 20
        if keep_len:
            w[at:at + 37] = rng.integers(0, 256, 37, dtype=np.uint8)
        else:
            w = np.concatenate([wire[:at], rng.integers(0, 256, 37, dtype=np.uint8), wire[at:]])
    elif cut == "wrap":
        # a masked 64-bit length that wraps the u64 sum (LEN_WRAP) at the first frame start after 25 MiB
        od, orr = oracle_segments(wire.copy(), [0], [len(wire)], 1 << 16)
        fo = od["frame_off"][:int(orr[0]["n_frames"])]
        at = int(fo[np.searchsorted(fo, 25 << 20)])
        bad = np.frombuffer(bytes([0x82, 0xFF]) + (0xFFFFFFFFFFFFFFF0).to_bytes(8, "big") + bytes(4), dtype=np.uint8)
        if keep_len:
            w[at:at + len(bad)] = bad
        else:
            w = np.concatenate([wire[:at], bad, wire[at:]])
    return w


@pytest.mark.parametrize("cut", ["max_frames", "truncated", "garbage", "wrap"])
def test_skip_path_stream_endings(dev, cut):
    """the eager skip path (no pass rounds: the plan kernel starts the walk at 0 and
    does the first round's chores) on purpose, not by test order — a mixed-length call sets the
    walk hint, then the cut stream is decoded: the call must skip the rounds and be bit-exact"""
    rng = np.random.default_rng(81)
    wire = long_stream(rng, 32 << 20, mix3)
    W.set_option("stream_rw", 1)
    run(dev, wire, 1 << 16)                                   # sets the hint (or keeps it set)
    n0 = W.get_stat("stream_skips")
    run(dev, wire, 1 << 16)
    assert W.get_stat("stream_skips") == n0 + 1               # the hint is set now
    cw = _cut_stream(cut, rng, wire)
    n0 = W.get_stat("stream_skips")
    run(dev, cw, 1200 if cut == "max_frames" else 1 << 16)
    assert W.get_stat("stream_skips") == n0 + 1, cut


@pytest.mark.parametrize("cut", ["max_frames", "garbage", "wrap"])
def test_skip_path_stream_endings_captured(dev, cut):
    """the same cuts in a captured raw-stream decode: replays of mixed bytes set the device hint,
    so the replay of the cut bytes skips its rounds on the device; every replay bit-exact"""
    rng = np.random.default_rng(82)
    wire = long_stream(rng, 32 << 20, mix3)
    cw = _cut_stream(cut, rng, wire, keep_len=True)
    n = len(wire)
    mf = 1200 if cut == "max_frames" else 1 << 16
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    desc = torch.zeros(mf * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(16, dtype=torch.uint8, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        W.stream_decode_device(d, n, mf, desc, res)
    for w in (wire, wire, cw, wire, cw):
        ob = w.copy()
        od, orr = oracle_segments(ob, [0], [n], mf)
        d[:n].copy_(torch.from_numpy(w).to(dev))
        desc.zero_()
        res.zero_()
        g.replay()
        torch.cuda.synchronize()
        gr = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
        assert tuple(gr) == tuple(orr[0]), (cut, gr, orr[0])
        assert np.array_equal(desc.cpu().numpy().view(W.DESC_DTYPE)[:int(gr["n_frames"])],
                              od[:int(orr[0]["n_frames"])])
        assert np.array_equal(d[:n].cpu().numpy(), ob)


def test_long_stream_same_as_serial(dev, serial_walk):
    """the one-wavefront walk on a chunk-parallel-sized stream (the option's other side)"""
    wire = long_stream(np.random.default_rng(28), 17 << 20, mix3)
    run(dev, wire, 1 << 14)


def test_long_stream_length_shift(dev):
    """the sample sees 64 KiB frames, the rest are ~1 KiB: chunks sized for big frames
    hold far more frames than their staging lists (the emit walks the excess)"""
    rng = np.random.default_rng(29)
    big = long_stream(rng, 2 << 20, lambda g: 65536, masked=1.0)
    small = long_stream(rng, 38 << 20, lambda g: g.integers(500, 1500), masked=1.0)
    wire = np.concatenate([big, small])
    r = run(dev, wire, 1 << 16)
    assert int(r["consumed"]) == len(wire) and int(r["n_frames"]) > 30000


def test_stream_tiny_frames_medium(dev):
    """2 MiB of 2..40 B frames (about 80 K frames): the chunk-parallel walk from 512 KiB on"""
    wire = long_stream(np.random.default_rng(30), 2 << 20, lambda g: g.integers(0, 27), masked=1.0)
    r = run(dev, wire, 1 << 17)
    assert int(r["consumed"]) == len(wire)


@pytest.mark.parametrize("alphabet", [(125, 1500, 65536), (7, 300), (0, 126, 65535, 70000)])
def test_stream_walk_alphabets(dev, alphabet):
    """the one-wavefront group walk's length speculation (two lengths: a 6-deep tree, three: 4
    deep, a fourth length replacing one round-robin): short streams of lengths drawn from an
    alphabet, cut by max_frames at every depth of a step, truncated mid-frame and with a bad
    header mid-stream"""
    rng = np.random.default_rng(sum(alphabet))
    pick = lambda g: g.choice(alphabet)
    wire = long_stream(rng, 300 << 10, pick, masked=1.0)
    r = run(dev, wire, 1 << 14)
    n = int(r["n_frames"])
    assert int(r["consumed"]) == len(wire)
    for mf in (1, 2, 3, 4, 5, 6, 7, 11, 13, n // 2, n - 1):
        r = run(dev, wire, max(1, mf))
        assert int(r["n_frames"]) == min(mf, n)
    run(dev, wire[:len(wire) - 3], 1 << 14)                                 # the last frame incomplete
    bad = wire.copy()
    bad[len(bad) // 2:len(bad) // 2 + 64] = 0x70                            # RSV bits: a decode error or garbage
    run(dev, bad, 1 << 14)


def test_stream_state_survives_mixed_calls(dev):
    """the pass loop's state rests in the stream's auxiliary workspace between calls: long
    changing streams (the chunk-parallel walk grows that workspace), short ones (the walk in
    the last resolve), batch decodes and reassembly on the same stream in between"""
    from test_gpu_parity import random_stream as rs
    long_w = long_stream(np.random.default_rng(31), 3 << 20, mix3)
    uni, *_ = wsynth.make_batch(3000, 0, 2000, 0, 32)
    short_w, so, sl = rs(np.random.default_rng(33), 200)
    for wire, mf in ((uni, 4096), (long_w, 1 << 14), (short_w, 4096), (uni, 4096), (long_w, 1 << 14)):
        run(dev, wire, mf)
        # a batch decode on the same (default) stream between stream decodes
        bw, boff, *_ = wsynth.make_batch(64, 0, 3000, 0, 34)
        n = len(bw)
        d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        d[:n] = torch.from_numpy(bw).to(dev)
        so_t = torch.tensor([0], dtype=torch.int64, device=dev)
        sl_t = torch.tensor([n], dtype=torch.int64, device=dev)
        desc = torch.zeros(64 * 32, dtype=torch.uint8, device=dev)
        res = torch.zeros(16, dtype=torch.uint8, device=dev)
        W.batch_decode_device(d, so_t, sl_t, 64, desc, res)
        torch.cuda.synchronize()
        assert int(res.cpu().numpy().view(W.SEGRES_DTYPE)[0]["n_frames"]) == 64


def test_stream_skips_rounds_while_lengths_keep_changing(dev):
    """eager calls on one stream: after a chunk walk whose sample saw lengths that keep changing,
    the next call skips the pass rounds (its walk starts at 0); a uniform stream then seen by
    that walk sends the call after it back to the rounds. Every call bit-exact vs the oracle."""
    mixed, *_ = wsynth.make_batch(1500, wsynth.PLEN_MIX3, 0, 0, 46)
    mixed2, *_ = wsynth.make_batch(1400, wsynth.PLEN_MIX3, 0, 0, 47)
    uni, *_ = wsynth.make_batch(20000, 0, 4096, 0, 3)
    W.set_option("stream_rw", 1)
    # (stream, skips the rounds); the first call may follow another test's call on this stream
    seq = [(mixed, None), (mixed, True), (mixed2[:len(mixed2) - 777], True), (uni, True), (uni, False),
           (mixed, False), (mixed2, True), (mixed2, True)]
    for i, (w, want) in enumerate(seq):
        n0 = W.get_stat("stream_skips")
        run(dev, w, 1 << 14, shift=5 if i == 6 else 0)
        skipped = W.get_stat("stream_skips") == n0 + 1
        if want is not None:
            assert skipped == want, (i, skipped)


def test_two_raw_streams_in_parallel_threads(dev):
    """two host threads, each decoding its own raw stream on its own HIP stream, four calls each:
    every HIP stream has its own workspace, pass state and walk hint (one thread's changing
    stream must not make the other's uniform stream skip its rounds, or the reverse); every call
    bit-exact vs the oracle"""
    import threading
    mixed, *_ = wsynth.make_batch(1500, wsynth.PLEN_MIX3, 0, 0, 71)
    uni, *_ = wsynth.make_batch(9000, 0, 4096, 0, 72)
    mixed2, *_ = wsynth.make_batch(1400, wsynth.PLEN_MIX3, 0, 0, 73)
    plans = {0: [mixed, mixed, uni, mixed2], 1: [uni, uni, mixed2, uni]}
    want = {}
    for w in (mixed, uni, mixed2):
        ob = w.copy()
        od, orr = oracle_segments(ob, [0], [len(w)], 1 << 15)
        want[id(w)] = (ob, od[:int(orr[0]["n_frames"])], tuple(orr[0]))
    errors = []

    def worker(k):
        try:
            st = torch.cuda.Stream(dev)
            cap = max(len(w) for w in plans[k]) + 64
            d = torch.zeros(cap, dtype=torch.uint8, device=dev)
            desc = torch.zeros((1 << 15) * 32, dtype=torch.uint8, device=dev)
            res = torch.zeros(16, dtype=torch.uint8, device=dev)
            for i, w in enumerate(plans[k]):
                with torch.cuda.stream(st):
                    d[:len(w)].copy_(torch.from_numpy(w).to(dev, non_blocking=False))
                    W.stream_decode_device(d, len(w), 1 << 15, desc, res, stream=st)
                st.synchronize()
                ob, od, orr = want[id(w)]
                gr = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
                assert tuple(gr) == orr, (k, i)
                assert np.array_equal(desc.cpu().numpy().view(W.DESC_DTYPE)[:len(od)], od), (k, i)
                assert np.array_equal(d[:len(w)].cpu().numpy(), ob), (k, i)
        except BaseException as e:  # noqa: BLE001 - reported by the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a decode thread hung"
    assert not errors, errors


# --- round 6: the split walk (option "stream_split"): K2 as two launches, the walk of the stream
# past the first launch's pieces on a side stream beside it (ws_stream.hip RwSplit) -------------

@pytest.fixture
def split_opts():
    """restores the split options after a test that changes them"""
    yield
    W.set_option("stream_split", 8)
    W.set_option("stream_split2", 48)
    W.set_option("stream_split_wait", 0)
    W.set_option("stream_c0", 3)
    W.set_option("stream_c1", 2)
    W.set_option("stream_split_capture", 1)
    W.set_option("stream_rw", 1)


def _frames_before(wire, nbytes, mf=1 << 17):
    od, orr = oracle_segments(wire.copy(), [0], [len(wire)], mf)
    fo = od["frame_off"][:int(orr[0]["n_frames"])]
    return int(np.searchsorted(fo, nbytes))


@pytest.mark.parametrize("split,split2,wait,c0,c1", [(1, 0, 0, 2, 1), (16, 0, 0, 2, 1), (16, 0, 1, 0, 1),
                                                    (16, 0, 2, 6, 1), (40, 0, 0, 3, 1), (128, 0, 0, 2, 1),
                                                    (255, 0, 2, 2, 1), (8, 32, 0, 3, 1), (2, 5, 1, 6, 0),
                                                    (24, 200, 2, 2, 3), (100, 101, 0, 0, 6)])
def test_stream_split_boundaries(dev, split_opts, split, split2, wait, c0, c1):
    """the split points (piece p0 = npieces * split / 256, and with split2 a second cut: three parts)
    fall inside frames; each part (its own chunk size) hands the chain over to the next mid-frame;
    streams ending (max_frames, truncation, garbage, a decode error) inside part 0, at the hand-off
    and inside the later parts; two buffer phases. Every call bit-exact vs the oracle and the split
    taken (stat stream_splits)"""
    W.set_option("stream_split", split)
    W.set_option("stream_split2", split2)
    W.set_option("stream_split_wait", wait)
    W.set_option("stream_c0", c0)
    W.set_option("stream_c1", c1)
    rng = np.random.default_rng(600 + split + split2)
    wire = long_stream(rng, 40 << 20, mix3)
    x = len(wire) * split // 256
    n0 = W.get_stat("stream_splits")
    run(dev, wire, 1 << 16)
    run(dev, wire, 1 << 16, shift=7)
    assert W.get_stat("stream_splits") >= n0 + 2
    # max_frames inside part 0, just past the split point and inside the later part(s)
    x2 = len(wire) * split2 // 256 if split2 > split else len(wire)
    for at in sorted({x // 2, x + 70000, (x + x2) // 2, x2 + 70000, (x2 + len(wire)) // 2}):
        if at >= len(wire):
            continue
        mf = max(1, _frames_before(wire, at))
        r = run(dev, wire, mf)
        assert int(r["n_frames"]) <= mf
    # garbage around the split points
    for at in (max(0, x - 5000), x + 3, min(len(wire) - 64, x + (20 << 20) // 3), min(len(wire) - 64, x2 + 11)):
        g = wire.copy()
        g[at:at + 37] = rng.integers(0, 256, 37, dtype=np.uint8)
        run(dev, g, 1 << 16)
    run(dev, wire[:x + 1000].copy(), 1 << 16)                                     # truncated after the split
    run(dev, wire[:len(wire) - 999].copy(), 1 << 16)


def test_stream_split_long_frames_and_host_path(dev, split_opts):
    """frames longer than part 0's small chunks (its owner walks cross them; entries outside the
    windows: the serial linker of a part) and the eager host-linked path (stream_rw 2: no split)"""
    W.set_option("stream_split", 64)
    W.set_option("stream_c0", 6)
    wire = long_stream(np.random.default_rng(611), 40 << 20, lambda g: g.integers(100 << 10, 1 << 20))
    run(dev, wire, 1 << 12)
    wire2 = long_stream(np.random.default_rng(612), 24 << 20, mix3)
    W.set_option("stream_rw", 2)
    run(dev, wire2, 1 << 16)


@pytest.mark.parametrize("cap", [0, 1])
def test_stream_split_captured(dev, split_opts, cap):
    """a captured raw-stream decode with the split option set: with stream_split_capture (the
    default) the side stream becomes a graph branch, without it the captured call takes one
    launch. Replays of changing bytes and a max_frames stop where part 0 would end
    are bit-exact each time"""
    W.set_option("stream_split", 32)
    W.set_option("stream_split_capture", cap)
    rng = np.random.default_rng(621)
    wire = long_stream(rng, 32 << 20, mix3)
    cw = _cut_stream("garbage", rng, wire, keep_len=True)
    n = len(wire)
    for mf in (1 << 16, max(1, _frames_before(wire, n * 32 // 256 // 2))):
        d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        desc = torch.zeros(mf * 32, dtype=torch.uint8, device=dev)
        res = torch.zeros(16, dtype=torch.uint8, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            W.stream_decode_device(d, n, mf, desc, res)
        for w in (wire, cw, wire, wire):
            ob = w.copy()
            od, orr = oracle_segments(ob, [0], [n], mf)
            d[:n].copy_(torch.from_numpy(w).to(dev))
            desc.zero_()
            res.zero_()
            g.replay()
            torch.cuda.synchronize()
            gr = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
            assert tuple(gr) == tuple(orr[0]), (mf, gr, orr[0])
            assert np.array_equal(desc.cpu().numpy().view(W.DESC_DTYPE)[:int(gr["n_frames"])],
                                  od[:int(orr[0]["n_frames"])])
            assert np.array_equal(d[:n].cpu().numpy(), ob)
        del g
