"""Multi-GPU plumbing for the batch decode (one process per GPU, torch.distributed).

Frames are independent, so a batch shards into contiguous segment
ranges with no data-path collective. The only cross-rank traffic is a handful of
scalars: the max step time (bench contract), verification counts and the output hash
({frames, payload bytes, errors, output hash}) — plus, as an optional model
of a NIC-attached rx buffer on one GPU, `scatter_from_root` (reported separately from the
decode, never inside its timed region).

Strong scaling over one global batch (`run_shard`): rank r decodes segments
[first, first + count) of ONE seeded batch (generated where it is decoded, by global frame
index), in rounds when its share exceeds the HBM budget; the per-frame output hash is
summed mod 2^64, so the all-reduced hash is the same for every world size and round size.
"""
import numpy as np

from .synth import mix64

U64 = np.uint64
HASH_C = U64(0x9E3779B97F4A7C15)


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
        # the segment boundary nearest to the r-th equal share: every rank's bytes then lie within
        # one segment of total / world
        t = total * r / world
        i = int(np.searchsorted(csum, t, side="left"))
        if 0 < i <= n and t - csum[i - 1] < csum[i] - t:
            i -= 1
        cuts.append(min(i, n))
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


def shard_cuts(nseg_total, world, seg_bytes=None):
    """world+1 segment cut indices of one global batch: byte-balanced when the segments' wire
    bytes are given (balance by bytes, not frame count — a mixed-length batch), else
    equal segment counts"""
    if seg_bytes is None:
        return [frame_shard(nseg_total, world, r)[0] for r in range(world)] + [nseg_total]
    assert len(seg_bytes) == nseg_total
    return byte_balanced_cuts(seg_bytes, world)


def shard_rounds(first, count, max_per_round, seg_bytes=None, max_bytes=None):
    """[(first_segment, nseg), ...] covering [first, first + count) in rounds of at most
    max_per_round segments and, when the segments' bytes are given, at most max_bytes wire
    bytes (the shard's HBM budget; a segment larger than that is a round of its own)"""
    out, s = [], first
    csum = None
    if seg_bytes is not None and max_bytes:
        csum = np.concatenate([[0], np.cumsum(np.asarray(seg_bytes[first:first + count], dtype=np.int64))])
    while s < first + count:
        n = min(max_per_round, first + count - s)
        if csum is not None:
            base = csum[s - first]
            fit = int(np.searchsorted(csum, base + max_bytes, side="right")) - 1 - (s - first)
            n = max(1, min(n, fit))
        out.append((s, n))
        s += n
    return out


def frame_hash(payload, datalen, is_fin, type_):
    """the output hash of one decoded frame (numpy statement of ws_hash_kernel,
    util_amd/csrc/ws_bench.hip): mix64(sum_j mix64(w_j + C*(j+1)) ^ datalen ^ fin<<56 ^
    type<<48) over the payload's little-endian 8-byte words (zero-padded)"""
    n = int(datalen)
    b = np.zeros((n + 7) // 8 * 8, np.uint8)
    b[:n] = np.asarray(payload, dtype=np.uint8)[:n]
    w = b.view("<u8").astype(np.uint64)
    j = np.arange(len(w), dtype=np.uint64)
    with np.errstate(over="ignore"):
        s = mix64(w + HASH_C * (j + U64(1))).sum(dtype=np.uint64) if len(w) else U64(0)
        return int(mix64(U64(s) ^ U64(n) ^ (U64(int(is_fin)) << U64(56)) ^ (U64(int(type_)) << U64(48))))


def batch_hash(buf, desc, res, max_frames):
    """sum (mod 2^64) of frame_hash over the used descriptors of a decoded batch"""
    h = 0
    for s in range(len(res)):
        for k in range(int(res[s]["n_frames"])):
            d = desc[s * max_frames + k]
            n = int(d["datalen"])
            a = int(d["data_off"]) if n else 0
            h = (h + frame_hash(buf[a:a + n], n, d["is_fin"], d["type"])) & 0xFFFFFFFFFFFFFFFF
    return h


def allreduce_u64(values, device=None):
    """exact all-reduce SUM of unsigned 64-bit values mod 2^64 (split into 16-bit limbs so
    that no limb overflows an int64 sum for any world size)"""
    import torch
    import torch.distributed as dist
    vals = [int(v) & 0xFFFFFFFFFFFFFFFF for v in values]
    if not (dist.is_available() and dist.is_initialized()):
        return vals
    if dist.get_backend() == "gloo":
        device = None
    limbs = [(v >> (16 * i)) & 0xFFFF for v in vals for i in range(4)]
    t = torch.tensor(limbs, dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t = t.tolist()
    return [sum(int(t[4 * k + i]) << (16 * i) for i in range(4)) & 0xFFFFFFFFFFFFFFFF for k in range(len(vals))]


def run_shard(nseg_total, world, rank, max_seg_per_round, decode_round, device=None, seg_bytes=None,
              max_bytes_per_round=None):
    """Decode this rank's share of one global batch of nseg_total segments, round by round.
    decode_round(first_segment, nseg) -> dict(frames, payload, wire, errors, hash, seconds)
    decodes segments [first, first + nseg) (global indices; it generates them where it
    decodes them) and returns its counts, its output hash and its timed decode seconds.
    seg_bytes (optional, every segment's wire bytes): the shards are byte-balanced and the rounds
    hold at most max_bytes_per_round bytes. Returns (local totals, global totals: sums over
    ranks, seconds = max over ranks; global["rank_wire"]: every rank's wire bytes)."""
    cuts = shard_cuts(nseg_total, world, seg_bytes)
    first, count = cuts[rank], cuts[rank + 1] - cuts[rank]
    loc = dict(frames=0, payload=0, wire=0, errors=0, hash=0, seconds=0.0, rounds=0, segments=count,
               first_segment=first)
    for s, n in shard_rounds(first, count, max_seg_per_round, seg_bytes, max_bytes_per_round):
        r = decode_round(s, n)
        for k in ("frames", "payload", "wire", "errors"):
            loc[k] += int(r[k])
        loc["hash"] = (loc["hash"] + int(r["hash"])) & 0xFFFFFFFFFFFFFFFF
        loc["seconds"] += float(r["seconds"])
        loc["rounds"] += 1
    frames, payload, wire, errors, h = allreduce_u64([loc["frames"], loc["payload"], loc["wire"], loc["errors"],
                                                      loc["hash"]], device=device)
    secs = allreduce([loc["seconds"]], op="max", device=device)[0]
    onehot = [0] * world
    onehot[rank] = loc["wire"]
    rank_wire = allreduce_u64(onehot, device=device)
    glob = dict(frames=frames, payload=payload, wire=wire, errors=errors, hash=h, seconds=secs, rank_wire=rank_wire)
    return loc, glob
