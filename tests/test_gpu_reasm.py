"""GPU parity of websocketframeBatchReassembleDevice (fused decode + message reassembly,
SURVEY §8a row a6) against the oracle composition (tests/oracle_lib.py:
oracle_reassemble = the pinned decode oracle + the FIN delivery rule), bit-exact:
descriptors, segment results, message descriptors, gathered bodies, open state; the
wire must come back untouched."""
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


def gpu_reassemble(dev, wire, so, sl, max_frames, open_in=None, out_off=None, out_size=None):
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
    W.batch_reassemble_device(d, T(so), T(sl), max_frames, desc, res, out, msg, nmsg,
                              out_off=None if out_off is None else T(out_off), open_state=op)
    torch.cuda.synchronize()
    assert np.array_equal(d[:n].cpu().numpy(), wire), "wire buffer modified"
    return (out.cpu().numpy(), desc.cpu().numpy().view(W.DESC_DTYPE), res.cpu().numpy().view(W.SEGRES_DTYPE)[:nseg],
            msg.cpu().numpy().view(W.MSG_DTYPE), nmsg.cpu().numpy()[:nseg],
            None if op is None else op.cpu().numpy())


def check(dev, wire, so, sl, mf, open_in=None, out_off=None, out_size=None, tag=""):
    out, gd, gr, gm, gn, gop = gpu_reassemble(dev, wire, so, sl, mf, open_in, out_off, out_size)
    od, orr, oms, oreg, oop = oracle_reassemble(wire, so, sl, mf, open_in, out_off)
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
    return out, oms, oop


@pytest.mark.parametrize("seed,mf", [(1, 16), (2, 4), (3, 1), (4, 64)])
def test_reassemble_random_vs_oracle(dev, seed, mf):
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 1500)
    out, _, _ = check(dev, wire, so, sl, mf, tag="seed %d" % seed)
    # bytes between the gathered bodies of different segments stay untouched
    covered = np.zeros(len(wire) + 64, bool)
    _, _, _, oreg, _ = oracle_reassemble(wire, so, sl, mf)
    for ob, body in oreg:
        covered[ob:ob + len(body)] = True
    assert (out[~covered] == 0xEE).all()


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
