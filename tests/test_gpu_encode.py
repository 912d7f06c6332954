"""GPU parity of websocketframeBatchEncodeDevice (gfx950 kernels, through the C ABI)
against the oracle composition (websocketframeEncode's header from the oracle,
pinned to the reference's golden vectors, + RFC 6455 client masking), bit-exact,
plus the encode -> decode round trip through the device decode path."""
import numpy as np
import pytest

from oracle_lib import oracle_encode_frames, oracle_segments
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True, params=[1, 0], ids=["front", "hipcub"])
def front(request, dev):
    """every test runs on both fronts: F1-F3 (tile scan + per-frame offsets, piece pointers
    and edge chunks before E3) and hipcub scan + E2, E3, E4"""
    W.set_option("enc_front", request.param)
    yield request.param
    W.set_option("enc_front", 1)


def random_frames(rng, n, edge=True, max_len=20000):
    choices = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 125, 126, 127, 1023, 4096, 65535, 65536, 70001]
    lens = [int(rng.choice(choices)) if edge and rng.random() < 0.5 else int(rng.integers(0, max_len))
            for _ in range(n)]
    gap = [int(rng.integers(0, 9)) for _ in range(n)]
    total = sum(lens) + sum(gap) + 16
    src = rng.integers(0, 256, total, dtype=np.uint8)
    fr = np.zeros(n, W.ENC_DTYPE)
    o = 0
    for i in range(n):
        o += gap[i]
        fr[i] = (o, lens[i], int(rng.integers(0, 2**32)), int(rng.integers(0, 16)), int(rng.integers(0, 2)),
                 int(rng.integers(0, 2)), 1 if rng.random() < 0.8 else 0)
        o += lens[i]
    return src, fr


def gpu_encode(dev, src, fr, dst_shift=0, capacity=None):
    s = torch.from_numpy(src).to(dev)
    f = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
    cap = int(fr["len"].sum()) + 14 * len(fr) if capacity is None else capacity
    dst_all = torch.full((cap + dst_shift + 64,), 0xA5, dtype=torch.uint8, device=dev)
    dst = dst_all[dst_shift:dst_shift + cap]
    off = torch.zeros(len(fr) + 1, dtype=torch.int64, device=dev)
    W.batch_encode_device(s, f, dst, off, capacity=cap)
    torch.cuda.synchronize()
    return dst_all.cpu().numpy(), off.cpu().numpy().astype(np.uint64)


@pytest.mark.parametrize("seed,shift", [(1, 0), (2, 3), (3, 13), (4, 8)])
def test_encode_vs_oracle(dev, seed, shift):
    rng = np.random.default_rng(seed)
    src, fr = random_frames(rng, 400)
    want, woff = oracle_encode_frames(src, fr)
    out, off = gpu_encode(dev, src, fr, dst_shift=shift)
    assert np.array_equal(off, woff)
    got = out[shift:shift + len(want)]
    if not np.array_equal(got, np.frombuffer(want, dtype=np.uint8)):
        bad = np.nonzero(got != np.frombuffer(want, dtype=np.uint8))[0]
        raise AssertionError("%d bytes differ, first at %d" % (len(bad), bad[0]))
    assert (out[:shift] == 0xA5).all() and (out[shift + len(want):] == 0xA5).all(), "wrote outside the wire"


def test_encode_small_frames_dense(dev):
    """many tiny frames per 16 KiB piece (header-only and 1-20 B payloads)"""
    rng = np.random.default_rng(7)
    src, fr = random_frames(rng, 5000, edge=False, max_len=21)
    want, woff = oracle_encode_frames(src, fr)
    out, off = gpu_encode(dev, src, fr)
    assert np.array_equal(off, woff)
    assert np.array_equal(out[:len(want)], np.frombuffer(want, dtype=np.uint8))


def test_encode_capacity_is_respected(dev):
    rng = np.random.default_rng(9)
    src, fr = random_frames(rng, 50)
    want, woff = oracle_encode_frames(src, fr)
    cap = len(want) // 2
    out, off = gpu_encode(dev, src, fr, capacity=cap)
    assert np.array_equal(off, woff)
    assert np.array_equal(out[:cap], np.frombuffer(want[:cap], dtype=np.uint8))
    assert (out[cap:] == 0xA5).all()


def test_encode_then_device_decode_roundtrip(dev):
    """masked client frames encoded on the GPU decode (device path) to the source payloads"""
    rng = np.random.default_rng(11)
    src, fr = random_frames(rng, 3000)
    fr["masked"] = 1
    out, off = gpu_encode(dev, src, fr)
    total = int(off[-1])
    wire = out[:total].copy()
    d = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    d[:total] = torch.from_numpy(wire).to(dev)
    # rx segments of ~8 frames each
    cuts = list(range(0, len(fr), 8))
    so = torch.tensor([int(off[c]) for c in cuts], dtype=torch.int64, device=dev)
    ends = [int(off[c + 8]) if c + 8 < len(fr) else total for c in cuts]
    sl = torch.tensor([e - int(off[c]) for c, e in zip(cuts, ends)], dtype=torch.int64, device=dev)
    desc = torch.zeros(len(cuts) * 8 * 32, dtype=torch.uint8, device=dev)
    res = torch.zeros(len(cuts) * 16, dtype=torch.uint8, device=dev)
    W.batch_decode_device(d, so, sl, 8, desc, res)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(W.SEGRES_DTYPE)
    assert (r["status"] == 0).all() and int(r["n_frames"].sum()) == len(fr)
    dd = desc.cpu().numpy().view(W.DESC_DTYPE)
    plain = d.cpu().numpy()
    for i in range(len(fr)):
        rec = dd[(i // 8) * 8 + i % 8]
        n = int(fr[i]["len"])
        assert int(rec["datalen"]) == n and int(rec["frame_off"]) == int(off[i])
        if n:
            a = int(rec["data_off"])
            assert np.array_equal(plain[a:a + n], src[int(fr[i]["src_off"]):int(fr[i]["src_off"]) + n]), i
    # and the oracle agrees on the decode of the GPU-encoded wire
    ob = wire.copy()
    _, orr = oracle_segments(ob, [int(off[c]) for c in cuts], [e - int(off[c]) for c, e in zip(cuts, ends)], 8)
    assert np.array_equal(r, orr)


def test_encode_many_tiles(dev):
    """300 K frames: 1172 tiles of 256 frames, so the one-block tile scan sums two tiles per
    thread; short payloads mix the shift path (>= 32 B) with the byte path"""
    rng = np.random.default_rng(13)
    n = 300000
    lens = rng.integers(0, 300, n)
    lens[rng.random(n) < 0.001] = 70000                                  # some 64-bit length headers
    src = rng.integers(0, 256, int(lens.max()) + 64, dtype=np.uint8)
    fr = np.zeros(n, W.ENC_DTYPE)
    fr["src_off"] = rng.integers(0, 64, n)
    fr["len"] = lens
    fr["mask_key"] = rng.integers(0, 2**32, n, dtype=np.uint64)
    fr["type"] = rng.integers(0, 16, n)
    fr["is_fin"] = rng.integers(0, 2, n)
    fr["prev_is_fin"] = rng.integers(0, 2, n)
    fr["masked"] = rng.random(n) < 0.8
    want, woff = oracle_encode_frames(src, fr)
    for shift in (0, 5):
        out, off = gpu_encode(dev, src, fr, dst_shift=shift)
        assert np.array_equal(off, woff)
        got = out[shift:shift + len(want)]
        assert np.array_equal(got, np.frombuffer(want, dtype=np.uint8))
        assert (out[:shift] == 0xA5).all() and (out[shift + len(want):] == 0xA5).all()

