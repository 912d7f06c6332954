"""GPU parity of decode path 5 (ws_spec.hip: the reactor loop's chain predicted per segment,
checked by the unmask blocks on their own pieces, mispredicted segments undone and walked
exactly) against the oracle (oracle/ws_oracle.c, pinned to the reference's golden vectors),
bit-exact: payload bytes, descriptors, segment results. The cases aim at every way a
prediction can be wrong and at the repair path's undo."""
import numpy as np
import pytest

from oracle_lib import oracle_segments, used_descs
from test_gpu_parity import assert_same, gpu_decode
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def spec_path():
    W.set_option("path", 5)
    yield
    W.set_option("path", -1)


def frame(rng, plen, b0=0x82, masked=True, form=None):
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
        h += rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
    return bytes(h) + rng.integers(0, 256, plen, dtype=np.uint8).tobytes()


def batch(segs, rng, gaps=True):
    blob, so, sl = bytearray(), [], []
    for seg in segs:
        if gaps:
            blob += bytes(int(rng.integers(0, 40)))
        so.append(len(blob))
        blob += seg
        sl.append(len(seg))
    return np.frombuffer(bytes(blob), dtype=np.uint8).copy(), so, sl


def regular(rng, n, plen, **kw):
    return b"".join(frame(rng, plen, **kw) for _ in range(n))


def test_spec_regular(dev):
    """equal frames in every segment (the predicted case), every 16-B phase of the segment starts"""
    rng = np.random.default_rng(1)
    segs = [regular(rng, 16, 4096) for _ in range(300)]
    wire, so, sl = batch(segs, rng)
    assert_same(dev, wire, so, sl, 16, tag="regular")


def test_spec_mispredicted_lengths(dev):
    """a frame of another length at every position of the chain, in every 3rd segment: the
    blocks after it applied the prediction; the repair undoes it and walks exactly"""
    rng = np.random.default_rng(2)
    segs = []
    for i in range(400):
        plens = [3000] * 20
        if i % 3 == 0:
            plens[i % 20] = int(rng.choice([2999, 3001, 100, 9000, 0, 70000]))
        segs.append(b"".join(frame(rng, p) for p in plens))
    wire, so, sl = batch(segs, rng)
    assert_same(dev, wire, so, sl, 32, tag="mispredicted")


def test_spec_same_total_other_layout(dev):
    """frames of the same wire length g with another header layout (non-minimal 64-bit length,
    unmasked frames, any FIN/opcode): the prediction holds, each frame keeps its own header"""
    rng = np.random.default_rng(3)
    segs = []
    for i in range(300):
        parts = []
        for k in range(12):
            r = rng.random()
            if r < 0.2:
                parts.append(frame(rng, 4104 - 14, b0=int(rng.integers(0, 256)), form=64))   # 14-B header
            elif r < 0.35:
                parts.append(frame(rng, 4104 - 4, masked=False))                           # unmasked, 4-B header
            else:
                parts.append(frame(rng, 4096, b0=int(rng.integers(0, 256))))
        segs.append(b"".join(parts))
    wire, so, sl = batch(segs, rng)
    assert_same(dev, wire, so, sl, 16, tag="layouts")


@pytest.mark.parametrize("mf", [1, 5, 16, 17])
def test_spec_tails_and_max_frames(dev, mf):
    """incomplete tails (a frame prefix: the stop check holds), complete short frames after the
    predicted ones (the stop check fails), and max_frames below / at / above the frame count"""
    rng = np.random.default_rng(4 + mf)
    segs = []
    for i in range(400):
        seg = regular(rng, 16, 2000)
        t = i % 5
        if t == 1:
            seg += frame(rng, 2000)[:int(rng.integers(1, 2008))]          # incomplete tail
        elif t == 2:
            seg += frame(rng, int(rng.integers(0, 1500)))                 # a complete shorter frame
        elif t == 3:
            seg += frame(rng, 2000)[:1]                                   # 1 byte left
        elif t == 4:
            seg += frame(rng, 3000)                                       # a longer complete frame
        segs.append(seg)
    wire, so, sl = batch(segs, rng)
    assert_same(dev, wire, so, sl, mf, tag="tails mf %d" % mf)


def test_spec_mixed_segment_kinds(dev):
    """predicted segments next to unpredictable ones (small frames g < 128, a first frame that is
    incomplete, empty segments, garbage) and long frames spanning many pieces"""
    rng = np.random.default_rng(6)
    segs = []
    for i in range(500):
        k = i % 6
        if k == 0:
            segs.append(regular(rng, 8, 100))                             # g < 128: walked by the repair
        elif k == 1:
            segs.append(frame(rng, 5000)[:3000])                          # first frame incomplete
        elif k == 2:
            segs.append(b"")
        elif k == 3:
            segs.append(rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes())
        elif k == 4:
            segs.append(regular(rng, 3, 70000))                           # 64-bit lengths, many pieces
        else:
            segs.append(regular(rng, 30, 700))
    wire, so, sl = batch(segs, rng)
    assert_same(dev, wire, so, sl, 32, tag="mixed kinds")


def test_spec_tiny_segments_many_per_piece(dev):
    """hundreds of short predicted segments inside one 16 KiB piece (one or two 130-B frames each)"""
    rng = np.random.default_rng(7)
    segs = [regular(rng, int(rng.integers(1, 3)), 124) for _ in range(3000)]
    wire, so, sl = batch(segs, rng, gaps=False)
    assert_same(dev, wire, so, sl, 4, tag="tiny segments")


def test_spec_unordered_and_out_of_range(dev):
    """segments out of buffer order: nothing is stored by the unmask blocks, every segment is walked"""
    rng = np.random.default_rng(8)
    segs = [regular(rng, 10, int(rng.choice([600, 4096]))) for _ in range(400)]
    wire, so, sl = batch(segs, rng)
    perm = rng.permutation(len(so))
    assert_same(dev, wire, [so[i] for i in perm], [sl[i] for i in perm], 16, tag="unordered")


def test_spec_repeated_calls_and_graph_replay(dev):
    """the repair list is never reset (a growing counter, per-call tags): eager calls and replays
    of one captured call alternate between batches that need repairs and batches that need none"""
    rng = np.random.default_rng(9)
    good = batch([regular(rng, 16, 4096) for _ in range(200)], rng)
    bad_segs = [regular(rng, 16, 4096) for _ in range(200)]
    for i in range(0, 200, 4):
        bad_segs[i] = regular(rng, 7, 4096) + frame(rng, 555) + regular(rng, 8, 4096)
    bad = batch(bad_segs, rng)
    for rnd in range(3):
        for w, so, sl in (good, bad, good):
            assert_same(dev, w, so, sl, 16, tag="eager %d" % rnd)
    # one captured call, replayed on a buffer whose contents change between replays
    n = max(len(good[0]), len(bad[0]))
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    so_t = torch.zeros(200, dtype=torch.int64, device=dev)
    sl_t = torch.zeros(200, dtype=torch.int64, device=dev)
    desc = torch.zeros(200 * 16 * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(200 * 16, dtype=torch.uint8, device=dev)

    def load(b):
        w, so, sl = b
        d.zero_()
        d[:len(w)] = torch.from_numpy(w).to(dev)
        so_t.copy_(torch.tensor(so, dtype=torch.int64))
        sl_t.copy_(torch.tensor(sl, dtype=torch.int64))
    load(good)
    W.batch_decode_device(d, so_t, sl_t, 16, desc, res)              # sizes the workspace before capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        W.batch_decode_device(d, so_t, sl_t, 16, desc, res)
    for b in (bad, good, bad, bad, good):
        load(b)
        g.replay()
        torch.cuda.synchronize()
        w, so, sl = b
        ob = w.copy()
        od, orr = oracle_segments(ob, so, sl, 16)
        gr = res.cpu().numpy().view(W.SEGRES_DTYPE)
        gd = desc.cpu().numpy().view(W.DESC_DTYPE)
        assert np.array_equal(gr, orr)
        assert np.array_equal(used_descs(gd, gr, 16), used_descs(od, orr, 16))
        assert np.array_equal(d[:len(w)].cpu().numpy(), ob)


def test_spec_full_size_cfg2_with_breaks(dev):
    """BASELINE cfg2 at full size (1 M x 4 KiB, 65,536 segments) with one frame of another length
    in every 64th segment: decode -> the generator's plaintext outside the broken segments, and
    the broken segments equal the oracle's walk"""
    import bench
    wl = bench.Workload.make("cfg2", dev)
    try:
        # shorten frame 5 of every 64th segment to 4000 B payload: the rest of its segment is garbage
        # to the reference loop (walks into payload bytes); compare those segments with the oracle
        segs = list(range(0, wl.nseg, 64))
        host = {}
        for s in segs:
            o = int(wl.off_h[s * 16 + 5])
            hb = wl.buf[o:o + 4].cpu().numpy().copy()
            hb[2:4] = np.frombuffer((4000).to_bytes(2, "big"), dtype=np.uint8)
            wl.buf[o:o + 4] = torch.from_numpy(hb).to(dev)
            a, b = int(wl.seg_off_h[s]), int(wl.seg_off_h[s] + wl.seg_len_h[s])
            host[s] = wl.buf[a:b].cpu().numpy().copy()
        wl.decode()
        torch.cuda.synchronize()
        res = wl.res.cpu().numpy().view(W.SEGRES_DTYPE)
        desc = wl.desc.cpu().numpy().view(W.DESC_DTYPE)
        for s in segs[:64]:
            ob = host[s].copy()
            od, orr = oracle_segments(ob, [0], [len(ob)], 16)
            a = int(wl.seg_off_h[s])
            assert np.array_equal(wl.buf[a:a + len(ob)].cpu().numpy(), ob), s
            assert (int(res[s]["consumed"]), int(res[s]["n_frames"]), int(res[s]["status"])) == \
                (int(orr[0]["consumed"]), int(orr[0]["n_frames"]), int(orr[0]["status"])), s
            gd = desc[s * 16:s * 16 + int(orr[0]["n_frames"])].copy()
            gd["frame_off"] -= a
            gd["data_off"] = np.where(gd["data_off"] == W.DATA_OFF_NULL, gd["data_off"], gd["data_off"] - a)
            assert np.array_equal(gd, used_descs(od, orr, 16)), s
        ok = np.ones(wl.nseg, bool)
        ok[segs] = False
        assert (res["status"][ok] == 0).all() and (res["n_frames"][ok] == 16).all()
    finally:
        wl.free()


def test_spec_first_call_on_a_fresh_stream(dev):
    """the first call on a new HIP stream gets a freshly zeroed workspace: its repairs (tags,
    disorder word) must not be mistaken for an earlier call's"""
    rng = np.random.default_rng(10)
    segs = [regular(rng, 16, 4096) for _ in range(64)]
    for i in range(0, 64, 3):
        segs[i] = regular(rng, 3, 4096) + frame(rng, 333) + regular(rng, 9, 4096)
    wire, so, sl = batch(segs, rng)
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, 16)
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, 16)
    assert np.array_equal(gr, orr)
    assert np.array_equal(used_descs(gd, gr, 16), used_descs(od, orr, 16))
    assert np.array_equal(gb, ob)
