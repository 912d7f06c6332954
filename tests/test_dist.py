"""Multi-process path on CPU: world_size-2 gloo ranks each decode their byte-balanced
shard of one batch (with the oracle: this tests the sharding/aggregation harness,
util_amd/dist.py) and the all-reduced totals equal a single-process decode."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import wsynth
from oracle_lib import oracle_segments
from util_amd import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    wire, off, pl, plain = wsynth.make_batch(96, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 21)
    fps = 4
    so = [int(off[i]) for i in range(0, 96, fps)]
    ends = [int(off[i + fps]) if i + fps < 96 else len(wire) for i in range(0, 96, fps)]
    return wire, so, [e - s for s, e in zip(so, ends)], fps, plain


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wire, so, sl, fps, plain = _batch()
    cuts = D.byte_balanced_cuts(sl, world)
    lo, hi = cuts[rank], cuts[rank + 1]
    buf = wire.copy()
    desc, res = oracle_segments(buf, so[lo:hi], sl[lo:hi], fps)
    mism = 0
    for s in range(lo, hi):
        mism += int((buf[so[s]:so[s] + sl[s]] != plain[so[s]:so[s] + sl[s]]).sum())
    tot = D.allreduce([int(res["n_frames"].sum()), int(res["consumed"].sum()), mism])
    tmax = D.allreduce([float(rank + 1)], op="max")
    q.put((rank, tot, tmax, hi - lo))
    dist.destroy_process_group()


def test_byte_balanced_cuts():
    sl = [10, 10, 10, 1000, 10, 10]
    c = D.byte_balanced_cuts(sl, 2)
    assert c[0] == 0 and c[-1] == 6 and 0 < c[1] < 6
    assert D.byte_balanced_cuts([], 3) == [0, 0, 0, 0]
    assert [D.frame_shard(10, 3, r) for r in range(3)] == [(0, 4), (4, 3), (7, 3)]


@pytest.mark.timeout(180)
def test_gloo_world2_matches_single_process():
    wire, so, sl, fps, plain = _batch()
    buf = wire.copy()
    desc, res = oracle_segments(buf, so, sl, fps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps)
    for rank, tot, tmax, nseg in out:
        assert tot == [float(res["n_frames"].sum()), float(res["consumed"].sum()), 0.0]
        assert tmax == [2.0]
    assert sum(o[3] for o in out) == len(so)


def _scatter_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wire = torch.from_numpy(_batch()[0])
    n = wire.numel() - 5                                       # a prefix: only nbytes travel
    recv = None if rank == 0 else torch.zeros(wire.numel(), dtype=torch.uint8)
    dt = D.scatter_from_root(wire if rank == 0 else None, recv, n)
    ok = True if rank == 0 else bool(torch.equal(recv[:n], wire[:n]) and int(recv[n:].sum()) == 0)
    q.put((rank, ok, dt))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_gloo_world3_scatter_from_root():
    """bench --scatter's exchange (rank 0's rx batch to every other rank) on gloo"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_scatter_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    out = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps)
    assert all(ok and dt >= 0 for _, ok, dt in out)
