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
