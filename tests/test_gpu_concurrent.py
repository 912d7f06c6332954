"""Several batch decodes in flight together: one HIP stream per batch (the C ABI keeps one
workspace per stream), calls issued back to back with no host synchronisation between
them, and from two host threads at once. Every batch vs the oracle, bit-exact; then more
streams than the per-device workspace table holds (the least recently used slot is
taken after a device synchronize)."""
import threading

import numpy as np
import pytest

import wsynth
from oracle_lib import oracle_segments, used_descs
from test_gpu_parity import random_stream
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _batch(i):
    """batch i: random mixed streams (piece path) or the cfg5 shape (segfuse), sizes differ"""
    if i % 3 == 2:
        wire, off, pl, plain = wsynth.make_batch(16 * (512 + 64 * i), 0, 1024, 2, 100 + i)
        so = [int(off[j]) for j in range(0, len(off), 16)]
        ends = so[1:] + [len(wire)]
        return wire, so, [e - s for s, e in zip(so, ends)], 16
    rng = np.random.default_rng(500 + i)
    wire, so, sl = random_stream(rng, 200 + 150 * i)
    return wire, so, sl, 16


class _Job:
    def __init__(self, dev, i):
        self.wire, self.so, self.sl, self.mf = _batch(i)
        n = len(self.wire)
        self.d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        self.d[:n] = torch.from_numpy(self.wire).to(dev)
        self.so_t = torch.tensor(self.so, dtype=torch.int64, device=dev)
        self.sl_t = torch.tensor(self.sl, dtype=torch.int64, device=dev)
        self.desc = torch.zeros(len(self.so) * self.mf * 32, dtype=torch.uint8, device=dev)
        self.res = torch.zeros(len(self.so) * 16, dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.Stream(dev)

    def launch(self):
        W.batch_decode_device(self.d, self.so_t, self.sl_t, self.mf, self.desc, self.res, stream=self.stream)

    def check(self, tag):
        n = len(self.wire)
        ob = self.wire.copy()
        od, orr = oracle_segments(ob, self.so, self.sl, self.mf)
        gr = self.res.cpu().numpy().view(W.SEGRES_DTYPE)
        gd = self.desc.cpu().numpy().view(W.DESC_DTYPE)
        assert np.array_equal(gr, orr), tag
        assert np.array_equal(used_descs(gd, gr, self.mf), used_descs(od, orr, self.mf)), tag
        out = self.d.cpu().numpy()
        assert np.array_equal(out[:n], ob), tag
        assert not out[n:].any(), tag


@pytest.mark.parametrize("path", [-1, 3, 4], ids=["auto", "piece", "segfuse"])
def test_streams_in_flight(dev, path):
    W.set_option("path", path)
    try:
        jobs = [_Job(dev, i) for i in range(6)]
        torch.cuda.synchronize()
        for j in jobs:
            j.launch()
        torch.cuda.synchronize()
        for i, j in enumerate(jobs):
            j.check("stream %d" % i)
    finally:
        W.set_option("path", -1)


def test_two_host_threads(dev):
    jobs = [_Job(dev, i) for i in range(8)]
    torch.cuda.synchronize()
    errs = []

    def run(part):
        try:
            torch.cuda.set_device(dev)
            for j in part:
                j.launch()
        except Exception as e:                     # noqa: BLE001 (reported below)
            errs.append(e)

    ts = [threading.Thread(target=run, args=(jobs[k::2],)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for i, j in enumerate(jobs):
        j.check("thread job %d" % i)


def test_more_streams_than_slots(dev):
    """20 streams > the 16 workspace slots of a device: twice round, all results exact"""
    jobs = [_Job(dev, i % 5) for i in range(20)]
    torch.cuda.synchronize()
    for rnd in range(2):
        for j in jobs:
            j.launch()
        torch.cuda.synchronize()
        for i, j in enumerate(jobs):
            if rnd == 0:
                j.check("slot job %d" % i)
            else:                                  # decoded twice: the wire is back
                assert np.array_equal(j.d[:len(j.wire)].cpu().numpy(), j.wire), i


def test_stream_decodes_from_two_threads(dev):
    """websocketframeStreamDecodeDevice from two host threads on two HIP streams at once:
    each (stream) has its own workspace, pass-loop state and walk scratch (round 1 shared
    one scratch per device)"""
    from test_gpu_stream import long_stream, mix3
    from util_amd import wsframe as W2
    wires = [long_stream(np.random.default_rng(700 + i), (1 << 20) + (i << 18), mix3) for i in range(2)]
    wires.append(wsynth.make_batch(4000, 0, 1500, 0, 710)[0])
    wires.append(wsynth.make_batch(4000, 0, 1500, 0, 711)[0])
    jobs = []
    for w in wires:
        n = len(w)
        d = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        src = torch.from_numpy(w).to(dev)
        desc = torch.zeros((1 << 15) * 32, dtype=torch.uint8, device=dev)
        res = torch.zeros(16, dtype=torch.uint8, device=dev)
        ob = w.copy()
        od, orr = oracle_segments(ob, [0], [n], 1 << 15)
        jobs.append(dict(n=n, d=d, src=src, desc=desc, res=res, ob=ob, orr=orr))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    errors = []

    def worker(t):
        try:
            with torch.cuda.stream(streams[t]):
                for rep in range(3):
                    for j in jobs[t::2]:
                        j["d"][:j["n"]].copy_(j["src"])
                        W2.stream_decode_device(j["d"], j["n"], 1 << 15, j["desc"], j["res"], stream=streams[t])
                        streams[t].synchronize()
                        gr = j["res"].cpu().numpy().view(W2.SEGRES_DTYPE)[0]
                        assert tuple(gr) == tuple(j["orr"][0]), (t, rep)
                        assert np.array_equal(j["d"][:j["n"]].cpu().numpy(), j["ob"]), (t, rep)
        except Exception as e:              # surfaced below
            errors.append(e)
    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[0]
