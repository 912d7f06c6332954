"""GPU parity: websocketframeBatchDecodeDevice (gfx950 kernels, through the C ABI)
against the oracle (oracle/ws_oracle.c, pinned to the reference) and the
reference's golden vectors. Bit-exact: buffer bytes, descriptors, segment results.
Full-size configs are checked by size-independent properties (decode restores
the generator's plaintext; decoding twice restores the wire bytes)."""
import hashlib
import os

import numpy as np
import pytest

import wsynth
from oracle_lib import oracle_segments, used_descs
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# decode variants: -1 auto (the default: 4 for many small segments, else 3), 3 the piece path
# (scan kernel + one-shot 16 KiB piece unmask), 4 one workgroup per segment (segfuse)
@pytest.fixture(params=[-1, 3, 4], ids=["auto", "piece", "segfuse"], autouse=True)
def decode_path(request):
    W.set_option("path", request.param)
    yield request.param
    W.set_option("path", -1)


def gpu_decode(dev, host_buf, seg_off, seg_len, max_frames, desc_base=None, pad=64):
    """copy to device (with slack), decode, copy back. Returns (buf, desc, res)."""
    n = len(host_buf)
    d = torch.zeros(n + pad, dtype=torch.uint8, device=dev)
    if n:
        d[:n] = torch.from_numpy(host_buf).to(dev)
    so = torch.tensor(np.asarray(seg_off, dtype=np.int64), device=dev)
    sl = torch.tensor(np.asarray(seg_len, dtype=np.int64), device=dev)
    nseg = len(seg_off)
    nslots = int(max(desc_base) + max_frames) if desc_base is not None and nseg else nseg * max_frames
    desc = torch.full((max(1, nslots) * 32,), 0xEE, dtype=torch.uint8, device=dev)
    res = torch.full((max(1, nseg) * 16,), 0xEE, dtype=torch.uint8, device=dev)
    db = None if desc_base is None else torch.tensor(np.asarray(desc_base, dtype=np.int64), device=dev)
    W.batch_decode_device(d, so, sl, max_frames, desc, res, desc_base=db)
    torch.cuda.synchronize()
    out = d.cpu().numpy()
    assert not out[n:].any(), "kernel wrote past the batch"
    return out[:n], desc.cpu().numpy().view(W.DESC_DTYPE), res.cpu().numpy().view(W.SEGRES_DTYPE)[:nseg]


def assert_same(dev, wire, seg_off, seg_len, max_frames, desc_base=None, tag=""):
    gb, gd, gr = gpu_decode(dev, wire.copy(), seg_off, seg_len, max_frames, desc_base)
    ob = wire.copy()
    od, orr = oracle_segments(ob, seg_off, seg_len, max_frames, desc_base)
    assert np.array_equal(gr, orr), tag
    assert np.array_equal(used_descs(gd, gr, max_frames, desc_base), used_descs(od, orr, max_frames, desc_base)), tag
    if not np.array_equal(gb, ob):
        bad = np.nonzero(gb != ob)[0]
        raise AssertionError("%s: %d bytes differ, first at %d" % (tag, len(bad), bad[0]))
    return gb, gd, gr


def test_golden_segments(dev, golden):
    for c in golden("decode_segments.json"):
        wire = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
        gb, gd, gr = gpu_decode(dev, wire, c["seg_off"], c["seg_len"], c["max_frames"])
        assert hashlib.sha256(gb.tobytes()).hexdigest() == c["output_sha256"], c["name"]
        assert [int(x) for x in gr["consumed"]] == [s["consumed"] for s in c["segments"]], c["name"]
        assert [int(x) for x in gr["status"]] == [s["status"] for s in c["segments"]], c["name"]
        assert_same(dev, wire, c["seg_off"], c["seg_len"], c["max_frames"], tag=c["name"])


def test_golden_single_frames_as_segments(dev, golden):
    """every single-frame fixture whose buffer is real (len <= bytes) as one segment"""
    cases = [c for c in golden("decode_single.json") if c["len"] <= len(c["input"]) // 2]
    blob, so, sl = bytearray(), [], []
    for c in cases:
        blob += bytes((len(blob) * 7 + 5) % 13 + 1)  # odd gaps -> every alignment
        so.append(len(blob))
        sl.append(c["len"])
        blob += bytes.fromhex(c["input"])
    wire = np.frombuffer(bytes(blob), dtype=np.uint8).copy()
    gb, gd, gr = gpu_decode(dev, wire, so, sl, 1)
    for i, c in enumerate(cases):
        seg = gb[so[i]:so[i] + len(c["input"]) // 2]
        assert hashlib.sha256(seg.tobytes()).hexdigest() == c["output_sha256"], c["name"]
        if c["ret"] != 0:
            d = gd[i]
            assert int(gr[i]["n_frames"]) == 1, c["name"]
            assert int(d["ret"]) == c["ret"] and int(d["datalen"]) == c["datalen"], c["name"]
            assert (int(d["is_fin"]), int(d["type"])) == (c["fin"], c["type"]), c["name"]
            exp_off = W.DATA_OFF_NULL if c["data_off"] is None else so[i] + c["data_off"]
            assert int(d["data_off"]) == exp_off, c["name"]
        else:
            assert int(gr[i]["n_frames"]) == 0 and int(gr[i]["consumed"]) == 0, c["name"]


@pytest.mark.parametrize("idx", range(4))
def test_golden_seeded_batches(dev, golden, idx):
    c = golden("batches.json")[idx]
    wire, off, pl, plain = wsynth.make_batch(c["nframes"], c["plen_kind"], c["fixed_len"], c["b0_kind"], c["seed"])
    fps, n = c["frames_per_segment"], c["nframes"]
    seg_off = [int(off[i]) for i in range(0, n, fps)]
    ends = [int(off[i + fps]) if i + fps < n else len(wire) for i in range(0, n, fps)]
    seg_len = [e - s for s, e in zip(seg_off, ends)]
    gb, gd, gr = gpu_decode(dev, wire.copy(), seg_off, seg_len, fps)
    assert hashlib.sha256(gb.tobytes()).hexdigest() == c["output_sha256"]
    assert hashlib.sha256(used_descs(gd, gr, fps).tobytes()).hexdigest() == c["desc_sha256"]


def random_stream(rng, nseg, max_frame=5000):
    blob, so, sl = bytearray(), [], []
    for _ in range(nseg):
        blob += bytes(int(rng.integers(0, 20)))
        so.append(len(blob))
        parts = []
        for _ in range(int(rng.integers(0, 12))):
            plen = int(rng.choice([0, 1, 2, 3, 5, 15, 16, 17, 31, 33, 125, 126, 127, 1000, 1023, 4096,
                                   int(rng.integers(0, max_frame))]))
            key = rng.integers(0, 256, 4, dtype=np.uint8) if rng.random() < 0.85 else None
            form = 7 if plen < 126 else (16 if plen <= 0xFFFF else 64)
            if plen < 126 and rng.random() < 0.1:
                form = 16
            if plen <= 0xFFFF and rng.random() < 0.05:
                form = 64
            h = bytearray([int(rng.integers(0, 256))])
            m = 0x80 if key is not None else 0
            if form == 7:
                h.append(m | plen)
            elif form == 16:
                h += bytes([m | 126]) + plen.to_bytes(2, "big")
            else:
                h += bytes([m | 127]) + plen.to_bytes(8, "big")
            if key is not None:
                h += key.tobytes()
            parts.append(bytes(h) + rng.integers(0, 256, plen, dtype=np.uint8).tobytes())
        seg = b"".join(parts)
        r = rng.random()
        if r < 0.3 and seg:
            seg = seg[: int(rng.integers(0, len(seg) + 1))]
        elif r < 0.4:
            seg += rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        blob += seg
        sl.append(len(seg))
    return np.frombuffer(bytes(blob), dtype=np.uint8).copy(), so, sl


@pytest.mark.parametrize("seed,max_frames", [(1, 16), (2, 3), (3, 1), (4, 64)])
def test_random_streams_vs_oracle(dev, seed, max_frames):
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 3000)
    assert_same(dev, wire, so, sl, max_frames, tag="seed%d" % seed)


def test_desc_base_and_empty_segments(dev):
    rng = np.random.default_rng(11)
    wire, so, sl = random_stream(rng, 500)
    sl = [0 if i % 7 == 0 else x for i, x in enumerate(sl)]
    base = np.cumsum([0] + [8] * (len(so) - 1)).astype(np.int64)[::-1].copy()  # reversed slots
    assert_same(dev, wire, so, sl, 8, desc_base=base, tag="desc_base")


def test_garbage_streams(dev):
    rng = np.random.default_rng(12)
    n = 1 << 20
    wire = rng.integers(0, 256, n, dtype=np.uint8)
    cuts = np.sort(rng.choice(n, 4000, replace=False))
    so = [int(x) for x in cuts[:-1]]
    sl = [int(b - a) for a, b in zip(cuts[:-1], cuts[1:])]
    assert_same(dev, wire, so, sl, 32, tag="garbage")


def test_large_frames_unaligned(dev):
    """64 KiB+ payloads at every 16-B phase, and a few MiB-sized frames"""
    blob, so, sl = bytearray(), [], []
    rng = np.random.default_rng(3)
    for phase in range(16):
        for plen in (65535, 65536, 65537, 3 << 20):
            blob += bytes(phase + 1)
            key = rng.integers(0, 256, 4, dtype=np.uint8)
            if plen <= 0xFFFF:
                h = bytes([0x82, 0x80 | 126]) + plen.to_bytes(2, "big")
            else:
                h = bytes([0x82, 0x80 | 127]) + plen.to_bytes(8, "big")
            f = h + key.tobytes() + rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
            so.append(len(blob))
            sl.append(len(f))
            blob += f
    wire = np.frombuffer(bytes(blob), dtype=np.uint8).copy()
    assert_same(dev, wire, so, sl, 2, tag="large")


def test_synth_matches_numpy_generator(dev):
    for (n, pk, fl, bk, seed) in [(40, wsynth.PLEN_FIXED, 4096, wsynth.B0_BINARY, 9),
                                  (30, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 10),
                                  (32, wsynth.PLEN_FIXED, 1024, wsynth.B0_FRAG16, 11),
                                  (16, wsynth.PLEN_FIXED, 125, wsynth.B0_TEXT, 1)]:
        wire, off, pl, plain = wsynth.make_batch(n, pk, fl, bk, seed)
        d = torch.zeros(len(wire), dtype=torch.uint8, device=dev)
        offs = torch.tensor(off.astype(np.int64), device=dev)
        W.synth_device(d, offs, n, pk, fl, bk, seed)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), wire)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4", "cfg5"])
def test_full_size_properties(dev, cfg):
    """BASELINE configs at full size (cfg4: one GPU's share of the 8-GPU batch, 1 M x 64 KiB =
    68.7 GB of wire in 16-frame rx segments): decode -> generator plaintext; decode again ->
    wire bytes; descriptors/segment results consistent with the generator's lengths"""
    import bench
    wl = bench.Workload.make(cfg, dev)
    try:
        wl.decode()
        torch.cuda.synchronize()
        assert wl.verify(expect_plain=True) == 0
        res = wl.res.view(torch.int64).view(-1, 2)
        assert int(res[:, 0].sum()) == wl.wire_bytes
        nf = (res[:, 1] & 0xFFFFFFFF)
        st = (res[:, 1] >> 32)
        assert int(nf.sum()) == wl.nframes and int((st != 0).sum()) == 0
        wl.check_descs()
        wl.decode()
        torch.cuda.synchronize()
        assert wl.verify(expect_plain=False) == 0
    finally:
        wl.free()


def _host_vs_oracle(wire, so, sl, max_frames, tag):
    hb = wire.copy()
    gd, gr = W.batch_decode_host(hb, np.asarray(so, np.uint64), np.asarray(sl, np.uint64), max_frames)
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, max_frames)
    assert np.array_equal(gr, orr), tag
    assert np.array_equal(used_descs(gd, gr, max_frames), used_descs(od, orr, max_frames)), tag
    assert np.array_equal(hb, ob), tag
    # slots past n_frames come back zeroed
    for s in range(len(so)):
        assert not gd[s * max_frames + int(gr[s]["n_frames"]):(s + 1) * max_frames].view(np.uint8).any(), tag


@pytest.mark.parametrize("chunk_mb", [64, 1])
def test_host_path_pipelined(dev, chunk_mb):
    """websocketframeBatchDecodeHost: ascending segments split into many ~1 MiB groups
    (3-stream H2D / decode / D2H pipeline) and the single-group case, vs the oracle"""
    rng = np.random.default_rng(11)
    wire, so, sl = random_stream(rng, 3000, max_frame=20000)
    W.set_option("host_chunk_mb", chunk_mb)
    try:
        _host_vs_oracle(wire, so, sl, 16, "chunk %d MiB" % chunk_mb)
    finally:
        W.set_option("host_chunk_mb", 64)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0] * 7])
def test_host_path_multi_device(dev, devices):
    """websocketframeBatchDecodeHostMulti on one box: the ascending segments cut into byte-balanced
    ranges, one per listed device (here the one GPU, repeated: its ranges run one after the other
    through the same pipeline), odd segment counts and mixed segment sizes so the cuts fall
    between unequal neighbours; bit-exact vs the oracle, slots past n_frames zeroed; unordered
    segments fall back to the one-device call"""
    rng = np.random.default_rng(13 + len(devices))
    wire, so, sl = random_stream(rng, 2001, max_frame=30000)
    W.set_option("host_chunk_mb", 1)
    try:
        perm = rng.permutation(len(so))
        for tag, s_, l_ in (("ordered", so, sl), ("unordered", [so[i] for i in perm], [sl[i] for i in perm])):
            hb = wire.copy()
            gd, gr = W.batch_decode_host_multi(hb, s_, l_, 16, devices)
            ob = wire.copy()
            od, orr = oracle_segments(ob, s_, l_, 16)
            assert np.array_equal(gr, orr), tag
            assert np.array_equal(used_descs(gd, gr, 16), used_descs(od, orr, 16)), tag
            assert np.array_equal(hb, ob), tag
            for k in range(len(s_)):
                assert not gd[k * 16 + int(gr[k]["n_frames"]):(k + 1) * 16].view(np.uint8).any(), tag
    finally:
        W.set_option("host_chunk_mb", 64)


def test_host_path_unordered_segments(dev):
    """segments out of buffer order: decoded as one group spanning all of them"""
    rng = np.random.default_rng(12)
    wire, so, sl = random_stream(rng, 800)
    perm = rng.permutation(len(so))
    so2, sl2 = [so[i] for i in perm], [sl[i] for i in perm]
    W.set_option("host_chunk_mb", 1)
    try:
        _host_vs_oracle(wire, so2, sl2, 8, "unordered")
    finally:
        W.set_option("host_chunk_mb", 64)


def test_device_unordered_and_out_of_range(dev):
    """segments out of buffer order, and a batch whose declared length is short of the last
    segment: decoded correctly either way (the piece path hands such batches to the walker)"""
    rng = np.random.default_rng(13)
    wire, so, sl = random_stream(rng, 600)
    perm = rng.permutation(len(so))
    assert_same(dev, wire, [so[i] for i in perm], [sl[i] for i in perm], 8, tag="unordered")
    n = len(wire)
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    d[:n] = torch.from_numpy(wire).to(dev)
    so_t = torch.tensor(np.asarray(so, dtype=np.int64), device=dev)
    sl_t = torch.tensor(np.asarray(sl, dtype=np.int64), device=dev)
    desc = torch.zeros(len(so) * 8 * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(len(so) * 16, dtype=torch.uint8, device=dev)
    lib = W.load_lib()
    rc = lib.websocketframeBatchDecodeDevice(d.data_ptr(), max(0, n - 100), so_t.data_ptr(), sl_t.data_ptr(), len(so), 8,
                                             None, desc.data_ptr(), res.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, 8)
    assert np.array_equal(res.cpu().numpy().view(W.SEGRES_DTYPE), orr)
    assert np.array_equal(d[:n].cpu().numpy(), ob)


@pytest.mark.parametrize("total", [(1 << 31) + 6, 1 << 32])
def test_int_truncation_real_size(dev, decode_path, total):
    """frames whose length sum reaches 2^31 (the (int) return goes negative: unmasked, then
    an error, websocketframe.c:164 + net_reactor.c:518-520) and exactly 2^32 (the return
    truncates to 0: unmasked, not consumed), at their real sizes, vs the oracle"""
    if decode_path == -1:
        pytest.skip("auto == piece for one segment")
    plen = total - 14
    n = total + 100
    block = np.random.default_rng(7).integers(0, 256, (1 << 20) + 7, dtype=np.uint8)
    host = np.empty(n, dtype=np.uint8)
    for a in range(0, n, len(block)):                     # tiled random bytes: cheap at 4 GB
        host[a:a + len(block)] = block[:n - a]
    host[:14] = np.frombuffer(bytes([0x82, 0x80 | 127]) + plen.to_bytes(8, "big") + bytes([0x11, 0x22, 0x33, 0x44]),
                              dtype=np.uint8)
    gb, gd, gr = gpu_decode(dev, host.copy(), [0], [n], 4)
    ob = host.copy()
    od, orr = oracle_segments(ob, [0], [n], 4)
    assert np.array_equal(gr, orr)
    assert np.array_equal(used_descs(gd, gr, 4), used_descs(od, orr, 4))
    assert np.array_equal(gb, ob)
    if total < (1 << 32):
        assert int(gr[0]["status"]) == -1 and int(gr[0]["n_frames"]) == 1 and int(gd[0]["ret"]) < 0
    else:
        assert int(gr[0]["n_frames"]) == 0 and int(gr[0]["consumed"]) == 0
    del gb, ob, host


@pytest.mark.parametrize("opt,val", [("piece_win", 0), ("piece_win", 2), ("piece_win", 3), ("seg_win", 0),
                                     ("seg_win", 1), ("seg_win", 3), ("piece_lds", 1), ("piece_lds", 56000)])
def test_window_mappings(dev, decode_path, opt, val):
    """K2's piece windows (piece_win = log2 W; the grid rounds up to W * ceil(P / W), spare
    blocks store nothing), the segment kernels' 1 / 2 / 8-window orders (seg_win; the default is
    4 / 8; 2101 segments: the last window's spare blocks) and K2's
    blocks-per-CU cap (piece_lds: 8 and 2 blocks instead of the default 5) at every setting,
    on a batch large enough for every window to be used: bit-exact vs the oracle"""
    W.set_option(opt, val)
    try:
        wire, off, pl, plain = wsynth.make_batch(2100, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 77)
        wire = np.concatenate([wire, wire[:1000]])                   # + an incomplete tail
        so = [int(off[i]) for i in range(0, 2100, 16)]
        ends = so[1:] + [len(wire)]
        assert_same(dev, wire, so, [e - s for s, e in zip(so, ends)], 16, tag="%s=%d" % (opt, val))
        wire, off, pl, plain = wsynth.make_batch(16 * 2101, 0, 1024, 2, 78)   # cfg5 shape (segfuse)
        so = [int(off[i]) for i in range(0, 16 * 2101, 16)]
        ends = so[1:] + [len(wire)]
        assert_same(dev, wire, so, [e - s for s, e in zip(so, ends)], 16, tag="%s=%d cfg5" % (opt, val))
    finally:
        W.set_option("piece_win", -1)
        W.set_option("seg_win", -1)
        W.set_option("piece_lds", 0)


def test_window_rule_automatic_four_windows(dev, decode_path):
    """the automatic rule (piece_win -1) on a >= 16 GiB batch of one frame length: a
    call on a stream whose previous call advised mixed lengths takes two windows, the next one
    (advised: frames of one length) four (stat k2_windows); 4 M x 4 KiB frames (17.2 GB): after the
    first call every payload is the generator's plaintext, after the second the wire is back,
    descriptors equal websocketframeDecode's for every frame both times"""
    import bench
    if decode_path != -1:
        pytest.skip("the rule is the auto path's (run once)")
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        # a mixed-length batch first: the stream's advice is then "not one length" (as for a first call)
        mixed = bench.Workload.make("cfg3", dev, nframes=4096)
        mixed.decode(stream=st)
        st.synchronize()
        mixed.free()
        wl = bench.Workload.make("cfg2", dev, nframes=4 << 20)
        torch.cuda.synchronize()
        assert wl.wire_bytes >= 16 << 30
        wins = []
        for k in range(2):
            wl.decode(stream=st)
            st.synchronize()
            wins.append(W.get_stat("k2_windows"))
            assert wl.verify(expect_plain=(k == 0)) == 0, k
            wl.check_descs()
    assert wins == [2, 4], wins
    wl.free()


def test_cfg4_shape_vs_oracle(dev, decode_path):
    """cfg4's layout (64 KiB masked frames, 16-frame rx segments, 64-bit length form) at reduced
    size, bit-exact vs the oracle: generator frames taken from the middle of the global batch
    (a rank's shard)"""
    if decode_path == 4:
        pytest.skip("segfuse is chosen only for segments <= 17 KiB")
    wire, off, pl, plain = wsynth.make_batch(64, wsynth.PLEN_FIXED, 65536, wsynth.B0_BINARY, 4, first=5 << 20)
    so = [int(off[i]) for i in range(0, 64, 16)]
    ends = so[1:] + [len(wire)]
    gb, gd, gr = assert_same(dev, wire, so, [e - a for a, e in zip(so, ends)], 16, tag="cfg4 shape")
    assert np.array_equal(gb, plain)


def test_output_hash_matches_numpy(dev, decode_path):
    """websocketframeFrameHashDevice (the multi-GPU output hash) equals its numpy statement
    util_amd/dist.py:batch_hash on a random batch (every length form, empty and unmasked frames)"""
    from util_amd import dist as D
    if decode_path != -1:
        pytest.skip("one decode path is enough")
    rng = np.random.default_rng(17)
    wire, so, sl = random_stream(rng, 400)
    gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, 16)
    h_np = D.batch_hash(gb, gd, gr, 16)
    n = len(wire)
    d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    d[:n] = torch.from_numpy(gb).to(dev)
    desc = torch.from_numpy(gd.view(np.uint8).copy()).to(dev)
    res = torch.from_numpy(gr.view(np.uint8).copy()).to(dev)
    h = torch.zeros(1, dtype=torch.int64, device=dev)
    W.frame_hash_device(d, desc, res, len(so), 16, h)
    torch.cuda.synchronize()
    assert (int(h.item()) & 0xFFFFFFFFFFFFFFFF) == h_np and h_np != 0


def test_strong_scaling_hash_independent_of_rounds(decode_path):
    """bench.py --config cfg4 (one global batch sharded over ranks, rounds per rank): the
    output hash, frame count and verification do not depend on the round size (reduced batch:
    65,536 x 64 KiB frames = 4.3 GB, one round vs four)"""
    import json
    import subprocess
    import sys
    if decode_path != -1:
        pytest.skip("runs the default path in a subprocess")
    outs = []
    for rf in (65536, 16384):
        p = subprocess.run([sys.executable, "bench.py", "--config", "cfg4", "--global-frames", "65536",
                            "--round-frames", str(rf), "--steps", "2", "--warmup", "1"],
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        outs.append(json.loads(p.stdout.strip().splitlines()[-1]))
    assert all(o["verified"] for o in outs)
    assert outs[0]["output_hash"] == outs[1]["output_hash"]
    assert outs[0]["allreduced"]["frames"] == outs[1]["allreduced"]["frames"] == 65536
    assert outs[1]["config"]["rounds_per_rank"] == 4


def test_host_path_never_writes_between_segments(dev, decode_path):
    """websocketframeBatchDecodeHost writes back only segment bytes: a read-only page between
    two segments (another connection's inbuf) stays untouched (a write would fault)"""
    import ctypes
    import mmap
    if decode_path != -1:
        pytest.skip("host path: one decode path is enough")
    page = mmap.PAGESIZE
    mm = mmap.mmap(-1, 3 * page, prot=mmap.PROT_READ | mmap.PROT_WRITE)
    buf = np.frombuffer(mm, dtype=np.uint8)
    wire, off, pl, plain = wsynth.make_batch(4, wsynth.PLEN_FIXED, 1000, wsynth.B0_BINARY, 61)
    a = int(off[2])
    buf[:a] = wire[:a]                                     # segment 0: frames 0-1, page 0
    buf[2 * page:2 * page + len(wire) - a] = wire[a:]      # segment 1: frames 2-3, page 2
    buf[page:2 * page] = 0xA5                              # the gap: page 1, made read-only
    libc = ctypes.CDLL(None)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(mm)) + page
    assert libc.mprotect(ctypes.c_void_p(addr), ctypes.c_size_t(page), 1) == 0      # PROT_READ
    try:
        so = np.array([0, 2 * page], np.uint64)
        sl = np.array([a, len(wire) - a], np.uint64)
        gd, gr = W.batch_decode_host(buf, so, sl, 4)
    finally:
        libc.mprotect(ctypes.c_void_p(addr), ctypes.c_size_t(page), 3)                 # PROT_READ|WRITE
    assert int(gr["n_frames"].sum()) == 4
    assert np.array_equal(buf[:a], plain[:a]) and np.array_equal(buf[2 * page:2 * page + len(wire) - a], plain[a:])
    assert (buf[page:2 * page] == 0xA5).all()
    del buf


def _segments_of(off, n, fps, total):
    so = [int(off[i]) for i in range(0, n, fps)]
    ends = so[1:] + [total]
    return so, [e - s for s, e in zip(so, ends)]


def test_stride_hint_never_changes_results(dev, decode_path):
    """K1's first step guesses the stride from the previous call's first frame length (the
    device's hint, eager calls on one stream). Every batch below follows a uniform batch of
    another frame length, or of the same first length with other lengths after it, or with
    bytes at the guessed stride that parse as frames of the guessed length: each decode is
    bit-exact vs the oracle whatever the hint was"""
    if decode_path != 3:
        pytest.skip("the hint is the piece path's")
    primer = {}
    for plen in (4096, 1000, 125):
        wire, off, pl, plain = wsynth.make_batch(64, wsynth.PLEN_FIXED, plen, wsynth.B0_BINARY, 90 + plen)
        primer[plen] = (wire, *_segments_of(off, 64, 16, len(wire)))
    # a 4104-B first frame, then 1008-B frames whose payload holds fake 4104-B headers at every
    # multiple of 4104 from the segment start (the positions the guessed stride parses)
    fake = wsynth.header(0x82, 4096, 0x01020304)
    segs = []
    for s in range(8):
        frames = [wsynth.header(0x82, 4096, 0xA0B0C0D0 + s), np.full(4096, s, np.uint8)]
        body = np.random.default_rng(s).integers(0, 256, 20 * 1000, dtype=np.uint8)
        pos = 4104
        for k in range(20):
            frames.append(wsynth.header(0x82, 1000, 0x11223344 * (k + 1) & 0xFFFFFFFF))
            frames.append(body[1000 * k:1000 * (k + 1)].copy())
        seg = np.concatenate(frames)
        for m in range(2, len(seg) // 4104):
            p = m * 4104
            if p + len(fake) <= len(seg):
                seg[p:p + len(fake)] = fake
        segs.append(seg)
    crafted = np.concatenate(segs)
    so = list(np.cumsum([0] + [len(x) for x in segs[:-1]]))
    crafted_case = (crafted, [int(x) for x in so], [len(x) for x in segs])
    mixed, off, pl, plain = wsynth.make_batch(96, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 5)
    mixed_case = (mixed, *_segments_of(off, 96, 16, len(mixed)))
    for first, then in [(4096, primer[1000]), (1000, primer[4096]), (4096, crafted_case), (125, crafted_case),
                        (4096, mixed_case), (125, primer[4096])]:
        pw, pso, psl = primer[first]
        gpu_decode(dev, pw.copy(), pso, psl, 64)          # sets the hint for the next call on the stream
        wire, so2, sl2 = then
        assert_same(dev, wire, so2, sl2, 64, tag="hint %d" % first)
