"""Multi-GPU plumbing for the batch decode (one process per GPU, torch.distributed).

Frames are independent, so a batch shards into contiguous segment
ranges with no data-path collective. The only cross-rank traffic is a handful of
scalars: the max step time (bench contract) and verification counts — plus, as an
optional model of a NIC-attached rx buffer on one GPU, `scatter_from_root` (reported
separately from the decode, never inside its timed region).
"""
import numpy as np


def byte_balanced_cuts(seg_len, world):
    """Split segments [0, n) into `world` contiguous ranges of ~equal bytes (cut on
    segment boundaries; SURVEY §8e: balance by bytes, not frame count). Returns
    world+1 cut indices."""
    seg_len = np.asarray(seg_len, dtype=np.float64)
    n = len(seg_len)
    if n == 0:
        return [0] * (world + 1)
    csum = np.concatenate([[0.0], np.cumsum(seg_len)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(csum, total * r / world, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):      # monotone
        cuts[i] = max(cuts[i], cuts[i - 1])
    return cuts


def frame_shard(nframes_total, world, rank):
    """contiguous, balanced frame range [first, first+count) of `rank`"""
    base, extra = divmod(nframes_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def allreduce(values, op="sum", device=None):
    """all-reduce a list of numbers across ranks (no-op when not initialised)"""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return list(values)
    if dist.get_backend() == "gloo":
        device = None                                  # gloo reduces host tensors
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t.tolist()


def scatter_from_root(send, recv, nbytes, root=0):
    """Root sends the first `nbytes` of `send` to every other rank's `recv` (point-to-point
    sends posted together: with RCCL each goes over its own xGMI link; gloo on CPU for the
    tests). Returns this rank's wall seconds for the exchange (synchronized)."""
    import time
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 0.0
    rank, world = dist.get_rank(), dist.get_world_size()
    cuda = send.is_cuda if rank == root else recv.is_cuda
    if cuda and dist.get_backend() == "gloo":                 # multi-rank rehearsal on one GPU: host copies
        out = None if rank == root else torch.empty(nbytes, dtype=torch.uint8)
        dt = scatter_from_root(send[:nbytes].cpu() if rank == root else None, out, nbytes, root)
        if rank != root:
            recv[:nbytes].copy_(out)
        return dt
    dist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if rank == root:
        ops = [dist.P2POp(dist.isend, send[:nbytes], r) for r in range(world) if r != root]
    else:
        ops = [dist.P2POp(dist.irecv, recv[:nbytes], root)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    return dt
