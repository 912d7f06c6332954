"""Multi-GPU plumbing for the batch decode (one process per GPU, torch.distributed).

Frames are independent, so a batch shards into contiguous segment
ranges with no data-path collective. The only cross-rank traffic is a handful of
scalars: the max step time (bench contract) and verification counts.
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
