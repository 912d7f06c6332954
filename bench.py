"""bench.py — device-resident WebSocket unmask throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU, RCCL)

A step = one websocketframeBatchDecodeDevice call over the whole synthetic batch
(BASELINE.json configs[1]: 1,048,576 masked binary frames x 4 KiB payload, split
into rx segments of 16 frames = 65,536 connections), in place, inputs resident
in HBM. value = payload GiB/s over all ranks (weak scaling: rank r decodes frames
[r*n, (r+1)*n) of one seeded stream; frames are independent, no collective in the data
path — RCCL only carries the max-over-ranks time, counts and the output hash).
roofline.frac is the step's (the contract's timed region: walk + unmask); the unmask
kernel alone is reported as roofline.kernel_frac.

--config cfg4: BASELINE configs[3] as STRONG scaling — ONE global batch of 8 M x 64 KiB
frames (549.9 GB of wire) sharded over the ranks by segment ranges, each rank generating
its share where it decodes it, in rounds that fit its HBM; a step = one pass over the whole
batch; the output hash (util_amd/dist.py:run_shard) is the same for every N.
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes as C
import json
import os
import re
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
# kernel that dominates the step, per websocketframeGpuSetOption("path") value
KERNELS = {1: "ws_walker_kernel", 3: "ws_piece_unmask_kernel", 4: "ws_segfuse_kernel"}
STEP_KERNELS = {3: "ws_piece_scan_kernel<16> + ws_piece_unmask_kernel (which decodes unordered batches itself, "
                   "one wave per segment)",
                4: "ws_segfuse_kernel (one launch: walk + unmask, one workgroup per rx segment)"}
DEFAULT_PATH = -1  # auto: 4 (segfuse) for >= 1024 segments of <= 17 KiB - 64 B average, max_frames <= 64; else 3


def decode_path(path, wl):
    """the decode variant websocketframeBatchDecodeDevice takes for this batch (ws_api.hip: decode_path)"""
    opt = dict(kv.split("=") for kv in filter(None, os.environ.get("WSFRAME_AMD_OPTIONS", "").split(",")))
    if "path" in opt:
        path = int(opt["path"])
    if path == 4:
        return 4 if wl.fps <= 64 else 3
    if path >= 0:
        return path
    return 4 if wl.fps <= 64 and wl.nseg >= 1024 and wl.wire_bytes <= wl.nseg * ((17 << 10) - 64) else 3


_RESULT_OUT = None


def emit(obj):
    """The bench line: the only thing this process writes to its real stdout (libraries'
    stdout — e.g. gloo's connection messages — goes to stderr, see main)"""
    out = _RESULT_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def timed_region(step, steps, world):
    """The bench contract's timed region: barrier + synchronize, exactly `steps` calls of
    `step` back to back on the current stream, synchronize + barrier. HIP events are
    recorded on that stream only at the region's two ends (an event between calls would
    put its own gap into the stream), so the per-call device time is their difference /
    steps. Returns (wall seconds of this rank, device ms per call)."""
    import torch
    import torch.distributed as dist
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0, e0.elapsed_time(e1) / steps


def pmc_traffic(kernel, algo_bytes, metric, graph=None):
    """HBM bytes per launch from the newest committed rocprofv3 PMC summary of this kernel,
    workload and bench metric (profiles/<tag>_pmc.json, tools/prof_summary.py), else None.
    The metric keeps one op's profile from standing in for another op's that runs the same
    kernel over the same bytes (cfg3 batch decode and cfg3 stream decode both end in K2)."""
    import glob
    best = None
    for f in glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")):
        try:
            rec = json.load(open(f))
        except ValueError:
            continue
        g = rec.get("bench_hip_graph")
        if g is None:                        # summaries before round 6: the tag says it
            g = "_graph" in os.path.basename(f)
        if kernel in rec.get("kernel", "") and rec.get("algo_bytes_per_launch") == algo_bytes \
                and rec.get("bench_metric") == metric and rec.get("traffic_bytes_per_launch") \
                and (graph is None or bool(g) == bool(graph)):
            # newest = the highest round in the file name (r06_…), then the latest in-file time:
            # file mtimes are the checkout's, not the profile's
            m = re.match(r"r(\d+)_", os.path.basename(f))
            key = (int(m.group(1)) if m else -1, str(rec.get("created") or ""), os.path.basename(f))
            if best is None or key > best[2]:
                best = (f, rec, key)
    return best[:2] if best else None


class Workload:
    """A synthetic batch laid out in HBM exactly as a reactor would hand it over:
    frames back to back in one buffer, rx segments of `fps` frames each."""

    CONFIGS = {
        # name: nframes, plen_kind, fixed_len, b0_kind, seed, frames per segment
        "cfg1": (16, 0, 125, 1, 1, 16),
        "cfg2": (1 << 20, 0, 4096, 0, 2, 16),
        "cfg3": (1 << 20, 1, 0, 0, 3, 16),
        "cfg4": (1 << 20, 0, 65536, 0, 4, 16),   # per GPU: 8M x 64 KiB over 8 GPUs
        "cfg5": (1 << 22, 0, 1024, 2, 5, 16),    # 256K messages x 16 fragments
        # not a BASELINE config: cfg5 with 1000-B fragments (bodies off the 16-B grid)
        "cfg5u": (1 << 22, 0, 1000, 2, 6, 16),
        # cfg3's length mix as ONE global batch sharded over the ranks (strong scaling, STRONG)
        "cfg3s": (1 << 20, 1, 0, 0, 3, 16),
    }
    DESCRIPTION = {
        "cfg1": "16 masked text frames x 125 B",
        "cfg2": "1M masked binary frames x 4 KiB, 16-frame rx segments",
        "cfg3": "1M frames, payload uniform from {125 B, 1500 B, 64 KiB}, 16-frame rx segments",
        "cfg4": "1M masked binary frames x 64 KiB per GPU (8M over 8 GPUs)",
        "cfg5": "256K messages x 16 continuation frames x 1 KiB (16-frame segments = messages)",
        "cfg5u": "256K messages x 16 continuation frames x 1000 B (bodies off the 16-B grid)",
        "cfg3s": "cfg3's length mix as one global batch, byte-balanced shards",
    }

    @classmethod
    def make(cls, name, dev, nframes=None, fps=None, plen=None, first_frame=0, seed_offset=0):
        """generator frames first_frame .. first_frame + nframes - 1 of the config's seeded
        stream (rank r of a weak-scaling run: first_frame = r * nframes)"""
        from util_amd import synth
        n, pk, fl, bk, seed, fps0 = cls.CONFIGS[name]
        fps = fps or fps0
        fl = plen or fl
        if nframes is not None:
            n = nframes
        return cls(name, dev, n, pk, fl, bk, seed + seed_offset, fps, synth, first_frame)

    def __init__(self, name, dev, n, pk, fl, bk, seed, fps, gen, first_frame=0):
        import torch
        from util_amd import wsframe as W
        self.torch, self.W = torch, W
        self.name, self.dev, self.nframes, self.plen_kind, self.fixed_len = name, dev, n, pk, fl
        self.b0_kind, self.seed, self.fps, self.first_frame = bk, seed, fps, first_frame
        plen = gen.plens(pk, fl, seed, n, first_frame)
        wl = gen.wirelens(plen)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(wl[:-1], dtype=np.uint64)
        self.plen_h, self.wirelen_h, self.off_h = plen, wl, off
        self.wire_bytes = int(wl.sum())
        self.payload_bytes = int(plen.sum())
        self.nseg = (n + fps - 1) // fps
        seg_off = off[::fps]
        seg_end = np.append(seg_off[1:], np.uint64(self.wire_bytes))
        self.seg_off_h, self.seg_len_h = seg_off, seg_end - seg_off
        t = torch
        self.buf = t.empty(self.wire_bytes + 256, dtype=t.uint8, device=dev)
        self.frame_off = t.from_numpy(off.astype(np.int64)).to(dev)
        self.seg_off = t.from_numpy(seg_off.astype(np.int64)).to(dev)
        self.seg_len = t.from_numpy(self.seg_len_h.astype(np.int64)).to(dev)
        self.desc = t.empty(self.nseg * fps * 32, dtype=t.uint8, device=dev)
        self.res = t.empty(self.nseg * 16, dtype=t.uint8, device=dev)
        self.buf[self.wire_bytes:].zero_()
        W.synth_device(self.buf, self.frame_off, n, pk, fl, bk, seed, first_frame=first_frame)
        self.decodes = 0

    # algorithmic HBM bytes of one decode: read every wire byte, write every payload byte
    @property
    def algo_bytes(self):
        return self.wire_bytes + self.payload_bytes

    def decode(self, stream=None):
        self.W.batch_decode_device(self.buf, self.seg_off, self.seg_len, self.fps, self.desc, self.res, stream=stream)
        self.decodes += 1

    def verify(self, expect_plain):
        t = self.torch
        mm = t.zeros(1, dtype=t.int64, device=self.dev)
        self.W.synth_verify_device(self.buf, self.frame_off, self.nframes, self.plen_kind, self.fixed_len, self.seed,
                                   expect_plain, mm, first_frame=self.first_frame)
        t.cuda.synchronize()
        return int(mm.item())

    def output_hash(self):
        """util_amd/dist.py:frame_hash summed over the batch's decoded frames (the buffer as it
        is now: hash it after an odd number of decodes)"""
        t = self.torch
        h = t.zeros(1, dtype=t.int64, device=self.dev)
        self.W.frame_hash_device(self.buf, self.desc, self.res, self.nseg, self.fps, h)
        t.cuda.synchronize()
        return int(h.item()) & 0xFFFFFFFFFFFFFFFF

    def check_descs(self):
        """descriptors of every frame equal what websocketframeDecode returns for the generator's frames"""
        t = self.torch
        d = self.desc.view(t.int64).view(-1, 4)
        fo, do, dl, rest = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
        plen = t.from_numpy(self.plen_h.astype(np.int64)).to(self.dev)
        wl = t.from_numpy(self.wirelen_h.astype(np.int64)).to(self.dev)
        hl = wl - plen
        n = self.nframes
        assert t.equal(fo[:n], self.frame_off)
        assert t.equal(do[:n], self.frame_off + hl)
        assert t.equal(dl[:n], plen)
        ret = rest[:n] & 0xFFFFFFFF
        assert t.equal(ret, wl)
        flags = (rest[:n] >> 32) & 0xFFFFFFFF
        f = t.arange(self.first_frame, self.first_frame + n, device=self.dev)
        if self.b0_kind == 2:
            j = f & 15
            fin = (j == 15).long()
            typ = t.where(j == 0, 2, 0)
        else:
            fin = t.ones_like(f)
            typ = t.full_like(f, 1 if self.b0_kind == 1 else 2)
        exp = fin | (typ << 8) | (1 << 16) | (hl << 24)
        assert t.equal(flags, exp)

    def host_sample(self, nframes):
        """copy the first `nframes` frames' wire bytes (as currently in HBM) to host memory"""
        nseg = max(1, nframes // self.fps)
        end = int(self.seg_off_h[nseg]) if nseg < self.nseg else self.wire_bytes
        return (self.buf[:end].cpu().numpy().copy(), self.seg_off_h[:nseg].copy(), self.seg_len_h[:nseg].copy(),
                int(self.plen_h[: nseg * self.fps].sum()))

    def free(self):
        del self.buf, self.desc, self.res
        self.torch.cuda.empty_cache()


class EncodeWorkload:
    """Client-side encode of the same frames: plaintext payloads resident
    in HBM -> masked wire frames (websocketframeEncode headers + MASK + key + XOR)."""

    def __init__(self, name, dev, seed_offset=0):
        import torch
        from util_amd import wsframe as W
        n, pk, fl, bk, seed, fps = Workload.CONFIGS[name]
        assert pk == 0, "encode bench: fixed-size configs only"
        self.torch, self.W, self.dev, self.name, self.fps = torch, W, dev, name, fps
        self.nframes, self.plen = n, fl
        g = torch.Generator(device=dev)
        g.manual_seed(seed + seed_offset)
        self.src = torch.randint(0, 256, (n * fl,), dtype=torch.uint8, device=dev, generator=g)
        fr = np.zeros(n, W.ENC_DTYPE)
        fr["src_off"] = np.arange(n, dtype=np.uint64) * fl
        fr["len"] = fl
        fr["mask_key"] = np.random.default_rng(seed).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        fr["type"], fr["is_fin"], fr["prev_is_fin"], fr["masked"] = 2, 1, 1, 1
        self.frames = torch.from_numpy(fr.view(np.uint8)).to(dev)
        self.hl = (2 if fl < 126 else (4 if fl <= 0xFFFF else 10)) + 4
        self.wire_bytes = n * (fl + self.hl)
        self.payload_bytes = n * fl
        self.dst = torch.empty(self.wire_bytes + 256, dtype=torch.uint8, device=dev)
        self.off = torch.empty(n + 1, dtype=torch.int64, device=dev)

    @property
    def algo_bytes(self):                  # read every payload byte, write every wire byte
        return self.payload_bytes + self.wire_bytes

    def step(self):
        self.W.batch_encode_device(self.src, self.frames, self.dst, self.off, capacity=self.wire_bytes)

    def verify(self):
        """decode the encoded wire on the device (rx segments of fps frames) and compare with the source"""
        t = self.torch
        n, fps = self.nframes, self.fps
        fl = self.wire_bytes // n
        so = t.arange(0, n, fps, device=self.dev, dtype=t.int64) * fl
        sl = t.full_like(so, fps * fl)
        desc = t.empty(len(so) * fps * 32, dtype=t.uint8, device=self.dev)
        res = t.empty(len(so) * 16, dtype=t.uint8, device=self.dev)
        ok = int(self.off[-1].item()) == self.wire_bytes
        self.W.batch_decode_device(self.dst, so, sl, fps, desc, res)
        body = self.dst[:self.wire_bytes].view(n, fl)[:, self.hl:]
        ok = ok and t.equal(body, self.src.view(n, self.plen))
        # output hash of the encoded frames, as decoded back (util_amd/dist.py:frame_hash)
        h = t.zeros(1, dtype=t.int64, device=self.dev)
        self.W.frame_hash_device(self.dst, desc, res, len(so), fps, h)
        self.hash = int(h.item()) & 0xFFFFFFFFFFFFFFFF
        return 0 if ok else 1


def run_encode(args, dev, world, rank):
    import torch
    from util_amd import dist as D
    wl = EncodeWorkload(args.config, dev, seed_offset=rank)
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    wall, step_ms = timed_region(wl.step, args.steps, world)
    elapsed = D.allreduce([wall], op="max", device=dev)[0]
    kern_ms = np.array([step_ms])
    mism = int(D.allreduce([wl.verify()], device=dev)[0])
    mean_kern = float(kern_ms.mean()) / 1e3
    achieved = wl.algo_bytes / mean_kern / 1e9
    metric = "WebSocket client encode+mask GiB/s (device-resident), %d x %d B frames" % (wl.nframes, wl.plen)
    pmc = pmc_traffic("ws_enc_copy_kernel", wl.algo_bytes, metric)
    out = {
        "metric": metric,
        "value": round(wl.payload_bytes * world * args.steps / elapsed / 2**30, 2), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (torch.randint payloads in HBM)",
        "config": {"workload": "encode " + Workload.DESCRIPTION[args.config], "config": args.config,
                   "frames_per_gpu": wl.nframes, "wire_bytes_per_gpu": wl.wire_bytes,
                   "payload_bytes_per_gpu": wl.payload_bytes},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": int(pmc[1]["traffic_bytes_per_launch"]) if pmc else None,
                     "traffic_source": os.path.relpath(pmc[0], REPO) if pmc else None,
                     "kernel": "ws_enc_copy_kernel", "algo_bytes_per_launch": wl.algo_bytes,
                     "timed": "HIP events at the two ends of the timed region on the calls' stream / steps: ws_enc_tsum_kernel + "
                              "ws_enc_tscan_kernel + ws_enc_front_kernel + ws_enc_copy_kernel",
                     "kernel_ms_mean": round(mean_kern * 1e3, 4)},
        "verified": mism == 0,
        "output_hash": "%016x" % D.allreduce_u64([wl.hash], device=dev)[0],
        "cpu_baseline": cpu_encode_baseline(wl, args.cpu_threads or granted_cpus()[0])
        if rank == 0 and world == 1 and not args.no_cpu else None,
    }
    if getattr(args, "cpu_defer", False):      # run_paths: timed on the CPU after every GPU path
        out["_cpu_later"] = (lambda smp=encode_cpu_sample(wl): cpu_encode_baseline(
            None, args.cpu_threads or granted_cpus()[0], sample=smp))
    return out, mism


def encode_cpu_sample(wl, nframes=65536):
    """the first `nframes` frames of an encode workload, copied to host memory"""
    n = min(nframes, wl.nframes)
    fr = wl.frames[:n * wl.W.ENC_DTYPE.itemsize].cpu().numpy().view(wl.W.ENC_DTYPE).copy()
    src = wl.src[:n * wl.plen].cpu().numpy().copy()
    return fr, src


def cpu_encode_baseline(wl, threads, nframes=65536, min_seconds=1.0, sample=None):
    """the reference's header encoder + client masking loop (oracle/ref_loop.c:ref_encode_frames)
    on host cores, over the first `nframes` frames of the workload (or a sample taken earlier by
    encode_cpu_sample)"""
    ref = os.path.join(REPO, "oracle", "_ref", "libwsref_loop.so")
    if not os.path.exists(ref):
        return None
    lib = C.CDLL(ref)
    fn = lib.ref_encode_frames
    fn.restype = C.c_ulonglong
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint, C.c_void_p]
    fr, src = sample if sample is not None else encode_cpu_sample(wl, nframes)
    n = len(fr)
    so = np.ascontiguousarray(fr["src_off"])
    ln = np.ascontiguousarray(fr["len"])
    key = np.ascontiguousarray(fr["mask_key"])
    bounds = np.linspace(0, n, threads + 1).astype(int)
    dsts = [np.empty(int(ln[bounds[i]:bounds[i + 1]].sum()) + (bounds[i + 1] - bounds[i]) * 14 + 16, np.uint8)
            for i in range(threads)]

    def run(i, passes):
        a, b = bounds[i], bounds[i + 1]
        for _ in range(passes):
            fn(src.ctypes.data, so[a:].ctypes.data, ln[a:].ctypes.data, key[a:].ctypes.data, b - a, dsts[i].ctypes.data)

    def timed(nthreads, passes):
        ths = [threading.Thread(target=run, args=(i, passes)) for i in range(nthreads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0
    payload = int(ln.sum())
    t1 = timed(1, 1) * threads                     # thread 0 does 1/threads of the frames
    passes = max(2, int(min_seconds / max(1e-6, t1 / threads)))
    tn = timed(threads, passes)
    g, src = granted_cpus()
    return {"value": round(payload * passes / tn / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "granted_cpus": g, "grant_sources": src,
            "single_thread_gibs": round(payload / t1 / 2**30, 3), "cpu_seconds": round(tn * threads + t1, 2),
            "sample": "%d frames (%.1f MiB payload) of the same workload, %d passes x %d threads, reference "
                      "websocketframeEncode headers + client masking loop (restated)" %
                      (n, payload / 2**20, passes, threads)}


def reasm_fused(wl):
    """websocketframeBatchReassembleDevice's path choice for this batch (ws_reasm.hip): the
    fused per-segment kernel for >= 1024 segments of <= 256 KiB average, max_frames <= 64"""
    opt = dict(kv.split("=") for kv in filter(None, os.environ.get("WSFRAME_AMD_OPTIONS", "").split(",")))
    p = int(opt.get("reasm_path", 0))
    if p:
        return p == 1 and wl.fps <= 64
    return wl.fps <= 64 and wl.nseg >= 1024 and wl.wire_bytes <= wl.nseg << 18


def run_stream(args, dev, world, rank):
    """The batch's wire as ONE raw rx stream (a single connection's inbuf, no frame or
    segment offsets from the host): websocketframeStreamDecodeDevice finds the frame
    boundaries on the device (speculative grid-wide passes whose loop state stays on the
    device) and unmasks with the piece kernel. Same algorithmic bytes as the decode. An
    eager call on a stream this long reads the pass state back once per group of rounds;
    --graph replays one captured call (no host reads at all)."""
    import torch
    from util_amd import dist as D
    from util_amd import wsframe as W
    nfr = args.frames or Workload.CONFIGS[args.config][0]
    wl = Workload.make(args.config, dev, nframes=args.frames, first_frame=rank * nfr)
    res = torch.zeros(16, dtype=torch.uint8, device=dev)

    def call():
        W.stream_decode_device(wl.buf, wl.wire_bytes, wl.nframes, wl.desc, res)
    graph = None
    if args.graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            call()

    def step():
        if graph is not None:
            graph.replay()
        else:
            call()
        wl.decodes += 1
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    wall, step_ms = timed_region(step, args.steps, world)
    elapsed = D.allreduce([wall], op="max", device=dev)[0]
    r = res.cpu().numpy().view(W.SEGRES_DTYPE)[0]
    bad = int(wl.verify(expect_plain=(wl.decodes % 2 == 1)) != 0)
    bad += int(int(r["n_frames"]) != wl.nframes or int(r["consumed"]) != wl.wire_bytes or int(r["status"]) != 0)
    if wl.decodes % 2 == 0:                  # the hash of the decoded (plaintext) stream
        call()
        wl.decodes += 1
    h = torch.zeros(1, dtype=torch.int64, device=dev)
    W.frame_hash_device(wl.buf, wl.desc, res, 1, wl.nframes, h)
    ghash = D.allreduce_u64([int(h.item())], device=dev)[0]
    mism = int(D.allreduce([bad], device=dev)[0])
    mean_kern = step_ms / 1e3
    metric = "WebSocket unmask GiB/s of one raw rx stream (device-resident, device-side frame boundaries)"
    pmc = pmc_traffic("ws_piece_unmask_kernel", wl.algo_bytes, metric, graph=bool(args.graph))
    out = {
        "metric": metric,
        "value": round(wl.payload_bytes * world * args.steps / elapsed / 2**30, 2), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded counter-based generator util_amd/csrc/ws_synth.h, generated in HBM)",
        "config": {"workload": "one stream: " + Workload.DESCRIPTION[args.config], "config": args.config,
                   "hip_graph": args.graph, "frames_per_gpu": wl.nframes, "wire_bytes_per_gpu": wl.wire_bytes,
                   "payload_bytes_per_gpu": wl.payload_bytes},
        "roofline": {"bound": "hbm", "achieved": round(wl.algo_bytes / mean_kern / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(wl.algo_bytes / mean_kern / 1e9 / PEAK_HBM_GBS, 4),
                     "traffic": int(pmc[1]["traffic_bytes_per_launch"]) if pmc else None,
                     "traffic_source": os.path.relpath(pmc[0], REPO) if pmc else None,
                     "kernel": "ws_piece_unmask_kernel", "algo_bytes_per_launch": wl.algo_bytes,
                     "timed": "HIP events at the two ends of the timed region / steps: ws_stream_init_kernel, "
                              "ws_stream_pass_kernel rounds (state on the device), ws_stream_finish_kernel (gated) "
                              "+ ws_piece_unmask_kernel",
                     "kernel_ms_mean": round(step_ms, 4)},
        "verified": mism == 0,
        "output_hash": "%016x" % ghash,
        "cpu_baseline": None,
    }
    return out, mism


def run_reasm(args, dev, world, rank):
    """Fused decode + message reassembly: the wire stays in HBM
    untouched, every message body is gathered unmasked into a contiguous output region.
    Algorithmic bytes: read every wire byte + write every body byte (8,623,489,024 B at cfg5)."""
    import torch
    from util_amd import dist as D
    from util_amd import wsframe as W
    wl = Workload.make(args.config, dev, first_frame=rank * Workload.CONFIGS[args.config][0])
    out = torch.empty(wl.wire_bytes + 64, dtype=torch.uint8, device=dev)
    msg = torch.empty(wl.nseg * wl.fps * 32, dtype=torch.uint8, device=dev)
    nmsg = torch.empty(wl.nseg, dtype=torch.int32, device=dev)

    rc_max = getattr(args, "readcache", 0) or 0
    cached = torch.zeros(wl.nseg, dtype=torch.int32, device=dev) if rc_max else None

    def step():
        W.batch_reassemble_device(wl.buf, wl.seg_off, wl.seg_len, wl.fps, wl.desc, wl.res, out, msg, nmsg,
                                  readcache_max=rc_max, cached=cached)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    wall, step_ms = timed_region(step, args.steps, world)
    elapsed = D.allreduce([wall], op="max", device=dev)[0]
    kern_ms = np.array([step_ms])
    # check: the wire is still masked; decoding it in place must yield the gathered bodies
    bad = int(wl.verify(expect_plain=False) != 0)
    wl.decode()
    t = torch
    plen, hl = wl.plen_h, wl.wirelen_h - wl.plen_h
    if wl.plen_kind == 0 and wl.nframes % wl.fps == 0:   # fixed-size frames: every body compared
        n, fl = wl.nframes, int(wl.wirelen_h[0])
        bodies = wl.buf[:wl.wire_bytes].view(n, fl)[:, int(hl[0]):]
        # output regions start at seg_off (= s * fps * wire length); bodies of a segment back to back
        seg_body = int(plen[0]) * wl.fps
        outv = out[:wl.wire_bytes].view(wl.nseg, wl.fps * fl)[:, :seg_body]
        bad += int(not t.equal(outv.reshape(-1), bodies.reshape(-1)))
        nm = nmsg.cpu().numpy()
        bad += int(not (nm == (1 if wl.b0_kind == 2 else wl.fps)).all())
    wl.decode()                              # back to the masked wire
    # output hash of the delivered messages: util_amd/dist.py:frame_hash over every message
    # body (len, complete as fin, type 0), through the hash kernel with the message table as
    # descriptors (message m of segment s in slot s * max_frames + m)
    m64 = msg.view(t.int64).view(-1, 4)
    d = t.zeros_like(m64)
    d[:, 1], d[:, 2], d[:, 3] = m64[:, 0], m64[:, 1], (m64[:, 3] & 0xFFFFFFFF) << 32
    r = t.zeros(wl.nseg, 2, dtype=t.int64, device=dev)
    r[:, 1] = nmsg.to(t.int64)
    h = t.zeros(1, dtype=t.int64, device=dev)
    W.frame_hash_device(out, d.view(t.uint8).view(-1), r.view(t.uint8).view(-1), wl.nseg, wl.fps, h)
    ghash = D.allreduce_u64([int(h.item())], device=dev)[0]
    del d, r, m64
    mism = int(D.allreduce([bad], device=dev)[0])
    mean_kern = float(kern_ms.mean()) / 1e3
    algo = wl.wire_bytes + wl.payload_bytes
    fused = reasm_fused(wl)
    kname = "ws_reasm_seg_kernel" if fused else "ws_reasm_gather_kernel"
    metric = "WebSocket fused unmask + message reassembly GiB/s of bodies (device-resident)"
    pmc = pmc_traffic(kname, algo, metric)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl.host_sample(262144), args.cpu_threads or None, op="reasm", frames_per_segment=wl.fps)
    later = None
    if getattr(args, "cpu_defer", False):      # run_paths: timed on the CPU after every GPU path
        later = (lambda smp=wl.host_sample(262144), fps=wl.fps: cpu_baseline(smp, args.cpu_threads or None,
                                                                             op="reasm", frames_per_segment=fps))
    out_json = {
        "metric": metric,
        "value": round(wl.payload_bytes * world * args.steps / elapsed / 2**30, 2), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded counter-based generator util_amd/csrc/ws_synth.h, generated in HBM)",
        "config": {"workload": "reassemble " + Workload.DESCRIPTION[args.config], "config": args.config,
                   "readcache_max_size": rc_max,
                   "frames_per_gpu": wl.nframes, "segments_per_gpu": wl.nseg, "wire_bytes_per_gpu": wl.wire_bytes,
                   "payload_bytes_per_gpu": wl.payload_bytes},
        "roofline": {"bound": "hbm", "achieved": round(algo / mean_kern / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(algo / mean_kern / 1e9 / PEAK_HBM_GBS, 4),
                     "traffic": int(pmc[1]["traffic_bytes_per_launch"]) if pmc else None,
                     "traffic_source": os.path.relpath(pmc[0], REPO) if pmc else None,
                     "kernel": kname,
                     "algo_bytes_per_launch": algo,
                     "timed": "HIP events at the two ends of the timed region on the calls' stream / steps: " + (
                         "ws_reasm_seg_kernel (one launch: decode + layout + gather per rx segment)" if fused else
                         "ws_piece_scan_kernel + ws_reasm_layout_kernel + ws_reasm_gather_kernel"),
                     "kernel_ms_mean": round(mean_kern * 1e3, 4)},
        "verified": mism == 0,
        "output_hash": "%016x" % ghash,
        "cpu_baseline": cpu,
    }
    if later is not None:
        out_json["_cpu_later"] = later
    return out_json, mism


def end_to_end(wl, runs=2):
    """websocketframeBatchDecodeHost on a pinned host copy of the whole batch: H2D + decode + D2H,
    pipelined over ~64 MiB segment groups on 3 streams (SURVEY §8d end-to-end). Reported beside
    `value`, never as it. Leaves wl.buf decoded an odd number of extra times (returned in `flips`)."""
    import torch
    from util_amd.wsframe import DESC_DTYPE, SEGRES_DTYPE
    from util_amd import load_lib
    hb = torch.empty(wl.wire_bytes, dtype=torch.uint8, pin_memory=True)
    hb.copy_(wl.buf[:wl.wire_bytes])
    desc = torch.empty(wl.nseg * wl.fps * 32, dtype=torch.uint8, pin_memory=True)
    res = torch.empty(wl.nseg * 16, dtype=torch.uint8, pin_memory=True)
    so = np.ascontiguousarray(wl.seg_off_h, dtype=np.uint64)
    sl = np.ascontiguousarray(wl.seg_len_h, dtype=np.uint64)
    lib = load_lib()

    def once():
        rc = lib.websocketframeBatchDecodeHost(hb.data_ptr(), wl.wire_bytes, so.ctypes.data, sl.ctypes.data, wl.nseg,
                                               wl.fps, desc.data_ptr(), res.data_ptr(), torch.cuda.current_device())
        if rc:
            raise RuntimeError(lib.websocketframeGpuLastError().decode())
    torch.cuda.synchronize()
    once()                                             # warm: slot allocation
    t0 = time.perf_counter()
    for _ in range(runs):
        once()
    dt = (time.perf_counter() - t0) / runs
    wl.buf[:wl.wire_bytes].copy_(hb, non_blocking=False)
    # the same call on pageable host memory (what the reference's realloc'd m_inbuf is): the
    # runtime stages the copies; a scratch copy of the batch, checked against the pinned result
    hp = np.empty(wl.wire_bytes, dtype=np.uint8)
    hp[:] = hb.numpy()

    def once_pageable():
        rc = lib.websocketframeBatchDecodeHost(hp.ctypes.data, wl.wire_bytes, so.ctypes.data, sl.ctypes.data, wl.nseg,
                                               wl.fps, desc.data_ptr(), res.data_ptr(), torch.cuda.current_device())
        if rc:
            raise RuntimeError(lib.websocketframeGpuLastError().decode())
    t0 = time.perf_counter()
    for _ in range(2):
        once_pageable()
    dtp = (time.perf_counter() - t0) / 2
    pageable = {"value": round(wl.payload_bytes / dtp / 2**30, 2), "unit": "GiB/s", "ms": round(dtp * 1e3, 2),
                "runs": 2, "host_buffer": "pageable (numpy)", "verified": bool(np.array_equal(hp, hb.numpy()))}
    del hp
    # the multi-device entry on the same pinned arena (websocketframeBatchDecodeHostMulti): every
    # visible GPU takes a byte-balanced range over its own PCIe link; on a one-GPU box the device
    # listed twice (its two ranges one after the other: the cost of the split itself)
    ndev = torch.cuda.device_count()
    devs = np.arange(ndev, dtype=np.int32) if ndev > 1 else np.zeros(2, dtype=np.int32)
    hm = torch.empty(wl.wire_bytes, dtype=torch.uint8, pin_memory=True)
    hm.copy_(hb)

    def once_multi():
        rc = lib.websocketframeBatchDecodeHostMulti(hm.data_ptr(), wl.wire_bytes, so.ctypes.data, sl.ctypes.data,
                                                    wl.nseg, wl.fps, desc.data_ptr(), res.data_ptr(),
                                                    devs.ctypes.data, len(devs))
        if rc:
            raise RuntimeError(lib.websocketframeGpuLastError().decode())
    once_multi()                                       # warm: every device's slots
    t0 = time.perf_counter()
    once_multi()
    dtm = (time.perf_counter() - t0)
    multi = {"value": round(wl.payload_bytes / dtm / 2**30, 2), "unit": "GiB/s", "ms": round(dtm * 1e3, 2),
             "runs": 1, "devices": devs.tolist(), "host_buffer": "pinned",
             "path": "websocketframeBatchDecodeHostMulti: byte-balanced segment ranges, one per device, each "
                     "websocketframeBatchDecodeHost's pipeline from its own host thread",
             "verified": bool(torch.equal(hm, hb))}
    del hm
    return {"value": round(wl.payload_bytes / dt / 2**30, 2), "unit": "GiB/s", "ms": round(dt * 1e3, 2),
            "runs": runs, "host_buffer": "pinned (hipHostMalloc via torch pin_memory)",
            "path": "websocketframeBatchDecodeHost: H2D | decode | D2H over 64 MiB groups, 3 streams",
            "pageable": pageable, "multi_device": multi}, runs + 1


def granted_cpus():
    """The CPUs this job may actually use: the affinity mask, capped by the cgroup's CPU quota
    (v2 cpu.max or v1 cfs_quota/period, rounded up) and by OMP_NUM_THREADS (the GPU box sets it
    to the job's share, 16, while nproc shows the whole machine). Returns (count, sources)."""
    import math
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = math.ceil(int(q) / int(p))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0 and p > 0:
                quota = math.ceil(q / p)
        except (OSError, ValueError):
            pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    g = aff
    if quota:
        g = min(g, quota)
    if omp:
        g = min(g, omp)
    return max(1, g), {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "omp_num_threads": omp or None}


def cpu_thread_counts():
    """(1, the CPUs granted to this job (granted_cpus: 16 on the GPU box), every CPU of the
    affinity mask (oversubscribed beyond the grant: a table entry only)), deduplicated, ascending"""
    g, src = granted_cpus()
    return sorted({1, g, src["affinity_cpus"]})


def cpu_baseline(sample, threads=None, min_seconds=2.0, op="decode", frames_per_segment=16):
    """Time the reference's own websocketframeDecode (oracle/_ref, compiled from the reference
    sources, driven by the reactor loop net_reactor.c:515-526: kind "reference") and the
    oracle restatement (oracle/ws_oracle.c: kind "port") on host cores, on a bounded sample of
    the workload, at 1 thread, at the job's CPU share and at every CPU of the process
    (threads=None) — SURVEY §8d. op "reasm": the same loop delivering messages as the reactor's
    stream hook does (oracle/ref_loop.c:ref_reassemble_segments). `value` is the all-CPU rate."""
    buf, so, sl, payload = sample
    ref = os.path.join(REPO, "oracle", "_ref", "libwsref_loop.so")
    what = "reactor loop net_reactor.c:515-526 over websocketframeDecode"
    runners = {}
    if os.path.exists(ref):
        lib = C.CDLL(ref)
        fn = lib.ref_reassemble_segments if op == "reasm" else lib.ref_decode_segments
        fn.restype = C.c_ulonglong
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint, C.POINTER(C.c_ulonglong)]

        def run_ref(lo, hi, _fn=fn):
            nf = C.c_ulonglong()
            _fn(buf.ctypes.data, so[lo:hi].ctypes.data, sl[lo:hi].ctypes.data, hi - lo, C.byref(nf))
        runners["reference" if op == "decode" else "port"] = run_ref
        if op == "reasm":
            what += " + fragment cache/merge delivery net_channel_ex.c:55-157 (restated glue)"
    if op == "decode":
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from oracle_lib import load_oracle
        from util_amd.wsframe import DESC_DTYPE, SEGRES_DTYPE
        olib = load_oracle()

        def run_port(lo, hi):
            d = np.empty((hi - lo) * frames_per_segment, DESC_DTYPE)
            r = np.empty(hi - lo, SEGRES_DTYPE)
            olib.ws_oracle_decode_segments(buf.ctypes.data, so[lo:hi].ctypes.data, sl[lo:hi].ctypes.data, hi - lo,
                                           frames_per_segment, None, d.ctypes.data, r.ctypes.data)
        runners.setdefault("port", run_port)
    if not runners:
        return None
    nseg = len(so)

    def timed(run, nthreads, passes):
        bounds = np.linspace(0, nseg, nthreads + 1).astype(int)

        def worker(i):
            for _ in range(passes):
                run(bounds[i], bounds[i + 1])
        ths = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0

    granted, src = granted_cpus()
    counts = cpu_thread_counts() if threads is None else sorted({1, threads})
    share = granted
    rates, wall = {}, 0.0
    for kind, run in runners.items():
        t1 = timed(run, 1, 2)                 # two passes: the buffer returns to its masked state
        p1 = max(2, int(min_seconds * 2 / t1) * 2)
        t1p = timed(run, 1, p1)               # one thread for about min_seconds
        wall += t1 + t1p
        t1 = t1p / p1
        rates[kind] = {1: payload / t1 / 2**30}
        for n in counts[1:]:
            # `passes` whole samples, sized so the run lasts about min_seconds on the CPUs the job
            # may actually use (the box grants OMP_NUM_THREADS of them, whatever nproc says);
            # even: the buffer returns to its masked state
            passes = max(2, int(min_seconds * min(n, share) / max(1e-6, t1)))
            passes += passes % 2
            tn = timed(run, n, passes)
            wall += tn
            rates[kind][n] = payload * passes / tn / 2**30
    kind = "reference" if "reference" in rates else "port"
    # value: the best rate on at most the granted CPUs (thread counts above the grant only
    # contend for the same cores: they stay in the table); cores: the grant
    within = {n: v for n, v in rates[kind].items() if n <= max(granted, 1)} or rates[kind]
    best_n = max(within, key=within.get)
    out = {"value": round(within[best_n], 3), "unit": "GiB/s", "cores": max(n for n in within), "kind": kind,
           "best_threads": best_n,
           "threads": {str(n): round(v, 3) for n, v in rates[kind].items()},
           "single_thread_gibs": round(rates[kind][1], 3),
           "granted_cpus": granted, "grant_sources": src, "cpu_count": os.cpu_count(),
           "wall_seconds": round(wall, 2),
           "sample": "%d frames (%d rx segments, %.1f MiB payload) of the same workload, %s; threads %s "
                     "(value: best rate on <= the %d granted CPUs)"
                     % (nseg * frames_per_segment, nseg, payload / 2**20, what, counts, granted)}
    if kind == "reference" and "port" in rates:
        out["port"] = {"kind": "port", "what": "oracle/ws_oracle.c (the restatement, same flags)",
                       "threads": {str(n): round(v, 3) for n, v in rates["port"].items()}}
    return out


STRONG = {"cfg4": 8 << 20,      # config -> global frames of its strong-scaling batch (BASELINE configs[3])
          "cfg3s": 8 << 20}     # cfg3's length mix as one global batch (mixed lengths: byte-balanced shards)
STRONG_ROUND_BYTES = 64 << 30   # default HBM budget per round for mixed-length batches (wire bytes)


def strong_layout(config, n_total):
    """The global batch of a strong-scaling config on the host: every frame's payload and wire
    length (generator frames 0 .. n_total - 1, util_amd/synth.py) and every rx segment's wire
    bytes — what util_amd/dist.py:run_shard balances the shards and bounds the rounds by"""
    from util_amd import synth
    n, pk, fl, bk, seed, fps = Workload.CONFIGS[config]
    assert n_total % fps == 0, "strong mode: whole segments"
    plen = synth.plens(pk, fl, seed, n_total, 0)
    wl = synth.wirelens(plen)
    seg_bytes = wl.reshape(-1, fps).sum(axis=1, dtype=np.uint64).astype(np.int64)
    return plen, wl, seg_bytes


def run_strong(args, dev, world, rank):
    """BASELINE configs[3] as strong scaling: ONE global batch (8 M x 64 KiB masked frames,
    16-frame rx segments, 549.9 GB of wire; or --config cfg3s: 8 M frames of cfg3's length mix)
    split over the ranks by segment ranges balanced by wire bytes (util_amd/dist.py:run_shard,
    SURVEY §8e); each rank generates its share where it decodes it (frames by global index,
    websocketframeSynthDeviceRange), in rounds of at most --round-frames frames and (mixed
    lengths) --round-bytes wire bytes (defaults: 1 M frames = 68.7 GB of cfg4: 8 rounds on one GPU,
    one on each of 8). Per round: generate, `warmup` decodes, `steps` decodes timed with HIP events
    at the region's two ends, one more if needed so the buffer holds plaintext, the output hash,
    the generator check. A step = one pass over the whole batch: ms_per_step = max over ranks of
    the sum over its rounds of the per-call decode time; value = the batch's payload / that."""
    import torch
    from util_amd import dist as D
    from util_amd import wsframe as W
    n_total = args.global_frames or STRONG[args.config]
    n, pk, fl, bk, seed, fps = Workload.CONFIGS[args.config]
    nseg_total = n_total // fps
    plen_all, wl_all, seg_bytes = strong_layout(args.config, n_total)
    foff_all = np.zeros(n_total + 1, dtype=np.int64)
    np.cumsum(wl_all.astype(np.int64), out=foff_all[1:])
    per_round = max(1, (args.round_frames or (1 << 20)) // fps)
    max_bytes = args.round_bytes or (STRONG_ROUND_BYTES if pk else None)
    cuts = D.shard_cuts(nseg_total, world, seg_bytes)
    first_seg, count = cuts[rank], cuts[rank + 1] - cuts[rank]
    rounds = D.shard_rounds(first_seg, count, per_round, seg_bytes, max_bytes)
    max_segs = max([1] + [nr for _, nr in rounds])
    cap = max([0] + [int(foff_all[(s + nr) * fps] - foff_all[s * fps]) for s, nr in rounds])
    buf = torch.empty(cap + 256, dtype=torch.uint8, device=dev)
    buf[cap:].zero_()
    desc = torch.empty(max_segs * fps * 32, dtype=torch.uint8, device=dev)
    res = torch.empty(max_segs * 16, dtype=torch.uint8, device=dev)
    hsh = torch.zeros(1, dtype=torch.int64, device=dev)
    mm = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def decode_round(s, nseg):
        nf = nseg * fps
        f0 = s * fps
        foff_h = foff_all[f0:f0 + nf + 1] - foff_all[f0]
        nbytes = int(foff_h[-1])
        foff = torch.from_numpy(np.ascontiguousarray(foff_h[:-1])).to(dev)
        so = foff[::fps].contiguous()
        sl = torch.from_numpy(np.ascontiguousarray(seg_bytes[s:s + nseg])).to(dev)
        b = buf[:nbytes + 256]
        b[nbytes:].zero_()
        W.synth_device(b, foff, nf, pk, fl, bk, seed, first_frame=f0)

        def call():
            W.batch_decode_device(b, so, sl, fps, desc, res)
        for _ in range(args.warmup):
            call()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(args.steps):
            call()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / max(1, args.steps)
        if (args.warmup + args.steps) % 2 == 0:
            call()                                                # odd: the buffer holds plaintext
        hsh.zero_()
        mm.zero_()
        W.frame_hash_device(b, desc, res, nseg, fps, hsh)
        W.synth_verify_device(b, foff, nf, pk, fl, seed, True, mm, first_frame=f0)
        r = res[:nseg * 16].view(torch.int64).view(-1, 2)
        frames = int((r[:, 1] & 0xFFFFFFFF).sum())
        bad_status = int(((r[:, 1] >> 32) != 0).sum()) + int(int(r[:, 0].sum()) != nbytes)
        torch.cuda.synchronize()
        return dict(frames=frames, payload=int(plen_all[f0:f0 + nf].sum()), wire=nbytes,
                    errors=int(mm.item()) + bad_status, hash=int(hsh.item()) & 0xFFFFFFFFFFFFFFFF, seconds=ms / 1e3)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    loc, glob = D.run_shard(nseg_total, world, rank, per_round, decode_round, device=dev, seg_bytes=seg_bytes,
                            max_bytes_per_round=max_bytes)
    wall = D.allreduce([time.perf_counter() - t0], op="max", device=dev)[0]
    step_s = glob["seconds"]
    algo = glob["wire"] + glob["payload"]
    rw = glob["rank_wire"]
    desc_txt = ("8M masked binary frames x 64 KiB" if args.config == "cfg4" else
                "%d frames, payload uniform from {125 B, 1500 B, 64 KiB}" % n_total if pk else
                "%d frames x %d B" % (n_total, fl))
    out = {
        "metric": "WebSocket unmask GiB/s (device-resident), 8M x 64KiB frames sharded across GPUs"
        if args.config == "cfg4" else "WebSocket unmask GiB/s (device-resident), one mixed-length batch sharded "
                                      "across GPUs",
        "value": round(glob["payload"] / step_s / 2**30, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded counter-based generator util_amd/csrc/ws_synth.h, each shard generated in HBM "
                "by global frame index)",
        "config": {"workload": desc_txt + ", 16-frame rx segments, one batch sharded by byte-balanced segment "
                                          "ranges", "config": args.config, "global_frames": n_total,
                   "global_wire_bytes": glob["wire"], "global_payload_bytes": glob["payload"],
                   "rounds_per_rank": loc["rounds"], "frames_per_round": per_round * fps,
                   "round_bytes_max": max_bytes, "alloc": args.alloc,
                   "rank_wire_bytes": rw,
                   "rank_wire_imbalance": round(max(rw) / (sum(rw) / world), 6) if sum(rw) else None,
                   "parallelism": "byte-balanced segment-range shards over %d GPU(s), no data-path collective"
                                  % world},
        "roofline": {"bound": "hbm", "achieved": round(algo / world / step_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s per GPU", "frac": round(algo / world / step_s / 1e9 / PEAK_HBM_GBS, 4),
                     "traffic": None, "kernel": "ws_piece_unmask_kernel", "algo_bytes_per_step": algo,
                     "algo_bytes_per_launch": int(foff_all[(rounds[0][0] + rounds[0][1]) * fps] -
                                                  foff_all[rounds[0][0] * fps]) +
                     int(plen_all[rounds[0][0] * fps:(rounds[0][0] + rounds[0][1]) * fps].sum()) if rounds else 0,
                     "kernel_ms_mean": round(step_s * 1e3 / max(1, loc["rounds"]), 4),
                     "timed": "per round: HIP events at the two ends of `steps` back-to-back decode calls; step = "
                              "sum over the rank's rounds, max over ranks (generation, hashing and checks between "
                              "rounds are outside)"},
        "verified": glob["errors"] == 0 and glob["frames"] == n_total,
        "output_hash": "%016x" % glob["hash"],
        "allreduced": {"frames": glob["frames"], "payload_bytes": glob["payload"], "errors": glob["errors"]},
        "wall_s_incl_generation": round(wall, 2),
        "cpu_baseline": None,
    }
    return out, 0 if out["verified"] else 1


def run_inflight(args, wl0, dev, world, rank):
    """K independent batches of the same config in flight together, one HIP stream each
    (websocketframeBatchDecodeDevice keeps one workspace per stream): batch i's walk can
    run beside batch i-1's unmask, so the per-call fixed cost (K1's dependent walk, the
    kernel boundary, K2's ramp-up and drain) overlaps other work. Same contract as the
    main region: barrier + synchronize on both sides, events on the base stream at the
    two ends only (every stream waits on the first and the base stream on every stream
    before the second). Not part of `value`."""
    import torch
    import torch.distributed as dist
    k = args.inflight
    wls = [wl0] + [Workload.make(args.config, dev, nframes=args.frames, fps=args.fps, plen=args.plen,
                                 first_frame=wl0.first_frame, seed_offset=7919 * i) for i in range(1, k)]
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    base = torch.cuda.current_stream()
    base.synchronize()
    for i in range(max(args.warmup, 2 * k)):
        wls[i % k].decode(stream=streams[i % k])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(base)
    for s in streams:
        s.wait_event(e0)
    payload = 0
    for i in range(args.steps):
        wls[i % k].decode(stream=streams[i % k])
        payload += wls[i % k].payload_bytes
    for s in streams:
        base.wait_stream(s)
    e1.record(base)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    dev_ms = e0.elapsed_time(e1)
    from util_amd import dist as D
    wall = D.allreduce([wall], op="max", device=dev)[0]
    mism = sum(w.verify(expect_plain=(w.decodes % 2 == 1)) for w in wls)
    for w in wls[1:]:
        w.free()
    algo = sum(wls[i % k].algo_bytes for i in range(args.steps))
    return {"batches_in_flight": k, "streams": k,
            "value": round(payload * world / wall / 2**30, 2), "unit": "GiB/s",
            "ms_per_batch": round(wall / args.steps * 1e3, 4),
            "device_ms_per_batch": round(dev_ms / args.steps, 4),
            "frac": round(algo / (dev_ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
            "what": "K independent batches of this config, one HIP stream each, calls issued round-robin; "
                    "not part of value", "verified": mism == 0}, mism


def run_decode(args, dev, world, rank, wl=None, path=DEFAULT_PATH):
    """The batch decode (websocketframeBatchDecodeDevice, in place, inputs resident in HBM) of
    args.config, weak scaling: warm-up, the contract's timed region, the dominant kernel's own
    launch time in a second region (k2_timing), the generator check and the output hash.
    Returns (bench line without the extras main() adds, mismatch count of this rank)."""
    import torch
    from util_amd import dist as D
    if wl is None:
        nfr = args.frames or Workload.CONFIGS[args.config][0]
        wl = Workload.make(args.config, dev, nframes=args.frames, fps=args.fps, plen=args.plen,
                           first_frame=rank * nfr)
    for _ in range(args.warmup):
        wl.decode()
    torch.cuda.synchronize()
    step = wl.decode
    if args.graph:                    # the call is host-sync free once its workspace exists
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            wl.W.batch_decode_device(wl.buf, wl.seg_off, wl.seg_len, wl.fps, wl.desc, wl.res)

        def step():
            graph.replay()
            wl.decodes += 1
    elapsed, step_ms = timed_region(step, args.steps, world)
    elapsed = D.allreduce([elapsed], op="max", device=dev)[0]      # bench contract: max over ranks

    # the dominant kernel's own launch duration, live: the piece path's K2 timed by HIP
    # events recorded around each K2 launch on the calls' stream (library option
    # k2_timing), over a second region of the same calls (events between kernels would
    # perturb the contract's region above, so it is not timed this way)
    kpath = decode_path(path, wl)
    k2_ms = None
    if kpath == 3 and not args.graph:
        wl.W.set_option("k2_timing", 1)
        c0, n0 = wl.W.get_stat("k2_calls"), wl.W.get_stat("k2_ns")
        for _ in range(args.steps):
            wl.decode()
        torch.cuda.synchronize()
        k2_calls, k2_ns = wl.W.get_stat("k2_calls") - c0, wl.W.get_stat("k2_ns") - n0
        wl.W.set_option("k2_timing", 0)
        if k2_calls:
            k2_ms = k2_ns / k2_calls / 1e6
    # correctness of the timed run: after an odd number of decodes the buffer holds plaintext
    mism = wl.verify(expect_plain=(wl.decodes % 2 == 1))
    # the output hash of the decoded batch (plaintext state), summed over ranks: the global
    # stream's frames [0, world * n) (util_amd/dist.py:frame_hash)
    if wl.decodes % 2 == 0:
        wl.decode()
    h = wl.output_hash()
    mism += wl.verify(expect_plain=True)
    mism = int(mism)
    ghash = D.allreduce_u64([h], device=dev)[0]

    value = wl.payload_bytes * world * args.steps / elapsed / 2**30
    step_kern = step_ms / 1e3
    mean_kern = k2_ms / 1e3 if k2_ms else step_kern
    achieved = wl.algo_bytes / step_kern / 1e9                      # the step: the contract's timed region
    metric = "WebSocket unmask GiB/s (device-resident) + %HBM peak, 1M x 4KiB frames"
    pmc = pmc_traffic(KERNELS[kpath], wl.algo_bytes, metric)
    timed = ("HIP events at the two ends of the contract's timed region on the calls' stream / steps: " +
             STEP_KERNELS.get(kpath, KERNELS[kpath]))
    kernel_timed = ("HIP events recorded around every %s launch on the calls' stream (library "
                    "option k2_timing), a second region of %d calls" % (KERNELS[kpath], args.steps)) if k2_ms else timed
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded counter-based generator util_amd/csrc/ws_synth.h, generated in HBM)",
        "config": {"workload": Workload.DESCRIPTION[args.config], "config": args.config, "hip_graph": args.graph,
                   "frames_per_gpu": wl.nframes, "frames_per_segment": wl.fps, "segments_per_gpu": wl.nseg,
                   "wire_bytes_per_gpu": wl.wire_bytes, "payload_bytes_per_gpu": wl.payload_bytes,
                   "parallelism": "frame-range shards, %d independent GPU(s)" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": int(pmc[1]["traffic_bytes_per_launch"]) if pmc else None,
                     "traffic_source": os.path.relpath(pmc[0], REPO) if pmc else None,
                     "traffic_kernels": pmc[1].get("kernels_summed") if pmc else None,
                     "kernel": KERNELS[kpath], "algo_bytes_per_launch": wl.algo_bytes,
                     "timed": timed,
                     "step_ms_mean": round(step_kern * 1e3, 4),
                     "kernel_ms_mean": round(mean_kern * 1e3, 4),
                     "kernel_frac": round(wl.algo_bytes / mean_kern / 1e9 / PEAK_HBM_GBS, 4),
                     "kernel_timed": kernel_timed,
                     "per_kernel_ns_profiled": pmc[1].get("per_kernel_avg_ns") if pmc else None},
        "verified": mism == 0,
        "output_hash": "%016x" % ghash,
        "cpu_baseline": None,
    }
    return out, mism


# the single-GPU paths of SURVEY §8 beside the headline (VERDICT r05 "next" 1): name ->
# (runner, config, graph). Each is timed with the headline's protocol (--steps after
# --warmup, barrier + synchronize, events at the region's two ends).
PATHS = {
    "decode_cfg3": ("decode", "cfg3"),    # websocketframe.c:112-165 under net_reactor.c:515-526, mixed lengths
    "reasm_cfg5": ("reasm", "cfg5"),      # + net_channel_ex.c:110-157 message delivery, readcache_max_size set
    "stream_cfg3": ("stream", "cfg3"),    # net_reactor.c:515-526 boundary discovery, one raw stream, eager
    "encode_cfg2": ("encode", "cfg2"),    # websocketframe.c:167-202 + client masking
}
PATH_READCACHE = 1 << 20                  # reasm_cfg5's readcache_max_size: 1 MiB > a 16 KiB message


def profile_check(out):
    """the newest committed rocprofv3 summary of this path (profiles/*_pmc.json, same
    dominant kernel, algorithmic bytes and metric): its traced step's fraction and this run's
    fraction over it"""
    rf = out["roofline"]
    pmc = pmc_traffic(rf["kernel"], rf["algo_bytes_per_launch"], out["metric"],
                      graph=bool(out["config"].get("hip_graph")))
    if not pmc:
        return None
    rec = pmc[1]
    step = rec.get("bench_ms_per_step")
    kern = rec.get("timed_region_kernel_ms_per_step")
    res = {"file": os.path.relpath(pmc[0], REPO), "traced_frac": rec.get("bench_frac"),
           "traced_kernel_ms_per_step": kern,
           "kernel_trace_frac": round(rf["algo_bytes_per_launch"] / (kern / 1e3) / 1e9 / PEAK_HBM_GBS, 4)
           if kern else None,
           "traffic_over_algo": round(rec["traffic_over_algo"], 4) if rec.get("traffic_over_algo") else None,
           "traced_ms_per_step": step}
    ref = res["traced_frac"] or res["kernel_trace_frac"]
    if ref:
        res["frac_over_traced"] = round(rf["frac"] / ref, 4)
    return res


def run_paths(args, dev):
    """SURVEY §8's other single-GPU paths, each on its own synthetic batch resident in HBM,
    timed by the headline's protocol in this same process; every entry verified against the
    generator / a second decode and hashed (util_amd/dist.py:frame_hash). The raw stream of
    cfg3 is the same frames as the batch decode of cfg3: their output hashes must be equal."""
    import copy
    import torch
    from util_amd import wsframe as W
    entries, mism, later = {}, 0, {}
    fns = {"decode": run_decode, "reasm": run_reasm, "stream": run_stream, "encode": run_encode}
    only = [x for x in (args.paths or "").split(",") if x]
    for name, (op, cfg) in PATHS.items():
        if only and name not in only:
            continue
        a = copy.copy(args)
        a.config, a.op, a.graph, a.frames, a.fps, a.plen, a.inflight = cfg, op, False, None, None, None, 1
        a.readcache = PATH_READCACHE if op == "reasm" else 0
        # CPU baselines run after every path is timed: the GPU never idles for seconds between
        # paths (a decode after idle time runs its first calls slower, DESIGN §4 "Short timed regions")
        a.cpu_defer, a.no_cpu = not args.no_cpu, True
        t0 = time.perf_counter()
        if op == "decode":
            out, m = run_decode(a, dev, 1, 0, path=DEFAULT_PATH)
        else:
            out, m = fns[op](a, dev, 1, 0)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        mism += m
        rf = out["roofline"]
        e = {"metric": out["metric"], "value": out["value"], "unit": out["unit"],
             "ms_per_step": out["ms_per_step"], "steps": out["steps"], "warmup": out["warmup"],
             "verified": out["verified"], "output_hash": out.get("output_hash"),
             "workload": out["config"]["workload"],
             "roofline": {"algo_bytes": rf["algo_bytes_per_launch"], "frac": rf["frac"], "kernel": rf["kernel"],
                          "step_ms_mean": rf.get("step_ms_mean", rf.get("kernel_ms_mean")),
                          "kernel_frac": rf.get("kernel_frac"), "traffic": rf.get("traffic"),
                          "timed": rf["timed"]},
             "profile": profile_check(out), "wall_s": round(time.perf_counter() - t0, 2)}
        if out.get("_cpu_later"):
            later[name] = out.pop("_cpu_later")
        if op == "reasm":
            e["readcache_max_size"] = a.readcache
        entries[name] = e
    if "decode_cfg3" in entries and "stream_cfg3" in entries:
        if entries["decode_cfg3"]["output_hash"] != entries["stream_cfg3"]["output_hash"]:
            mism += 1
            entries["stream_cfg3"]["verified"] = False
        entries["stream_cfg3"]["hash_equals_decode_cfg3"] = \
            entries["decode_cfg3"]["output_hash"] == entries["stream_cfg3"]["output_hash"]
    W.set_option("k2_timing", 0)
    for name, fn in later.items():
        entries[name]["cpu_baseline"] = fn()
    return entries, mism


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, poll_s=0.1, grace_s=10.0):
    """`python bench.py --gpus N` without a launcher: start N ranks of this same command as
    child processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, one GPU
    each; WS_BENCH_RANKS_PER_GPU > 1 packs ranks onto fewer GPUs for rehearsal), relay rank 0's
    JSON line, and return non-zero if any rank failed. Every rank is polled: as soon as one
    exits non-zero the others are terminated (they would otherwise block in a rendezvous or a
    collective until torch.distributed's timeout). This process never touches a GPU."""
    import subprocess
    import tempfile
    import time
    port = str(free_port())
    procs = []
    out_f = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out_f if r == 0 else subprocess.DEVNULL))
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        failed = next((r for r, p in enumerate(procs) if p.poll() not in (None, 0)), None)
        if failed is None:
            time.sleep(poll_s)
    if failed is None:
        failed = next((r for r, p in enumerate(procs) if p.returncode), None)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    rcs = [p.returncode for p in procs]
    out_f.seek(0)
    out = out_f.read()
    out_f.close()
    if out and failed is None:
        _RESULT_OUT.write(out.decode())
        _RESULT_OUT.flush()
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc]
    if bad:
        sys.stderr.write("bench.py: ranks failed: %s (first: rank %s)\n" % (bad, failed))
    return 1 if bad or not out else 0


def main():
    # the contract's single JSON line goes to the real stdout; everything else any library
    # prints to fd 1 (gloo's "Rank k is connected to ..." lines, runtime chatter) to stderr
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: 1, the job's share (OMP_NUM_THREADS) and every CPU of the process)")
    ap.add_argument("--path", type=int, default=None, help="decode variant (websocketframeGpuSetOption path)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer end-to-end measurement")
    ap.add_argument("--no-paths", action="store_true",
                    help="skip the other single-GPU paths (cfg3 decode, cfg5 reassembly, cfg3 raw stream, cfg2 "
                         "encode) the default cfg2 run at N = 1 times beside the headline (`paths`)")
    ap.add_argument("--paths", default="",
                    help="comma list of the `paths` entries to time (default: all of %s)" % ",".join(PATHS))
    ap.add_argument("--readcache", type=int, default=0,
                    help="--op reasm: readcache_max_size (net_channel_ex.c:45-53; 0 = no limit)")
    ap.add_argument("--no-xor-stream", action="store_true", help="skip the plain XOR-stream reference run")
    ap.add_argument("--graph", action="store_true",
                    help="decode: capture one call into a HIP graph and replay it for every step")
    ap.add_argument("--scatter", action="store_true",
                    help="N > 1: also time rank 0 sending its wire batch to every other rank (a NIC-attached "
                         "rx buffer on one GPU; RCCL point-to-point over xGMI), reported separately")
    ap.add_argument("--frames", type=int, default=None, help="override the config's frame count (experiments)")
    ap.add_argument("--fps", type=int, default=None, help="override frames per rx segment (experiments)")
    ap.add_argument("--plen", type=int, default=None, help="override the fixed payload length (experiments)")
    ap.add_argument("--global-frames", type=int, default=None,
                    help="strong-scaling configs (cfg4): frames of the global batch (default 8M)")
    ap.add_argument("--round-frames", type=int, default=None,
                    help="strong-scaling configs: frames per round on one GPU (default 1M = 68.7 GB of wire)")
    ap.add_argument("--round-bytes", type=int, default=None,
                    help="strong-scaling configs: wire bytes per round at most (default: 64 GiB for mixed lengths)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="decode: also time K independent batches of the config in flight together, one HIP "
                         "stream each (a reactor with successive rx batches), reported as the 'inflight' field "
                         "(1 = off)")
    ap.add_argument("--alloc", default="torch", choices=["torch", "contiguous"],
                    help="device buffers from torch's caching allocator (default), or every allocation "
                         "physically contiguous (libwsframe_amd_bench.so as torch's pluggable allocator; "
                         "DESIGN §4: cfg4's slow mode on boxes whose memory earlier processes fragmented)")
    ap.add_argument("--op", default="decode", choices=["decode", "encode", "reasm", "stream"],
                    help="decode (the headline), client-side encode + mask of the same frames, fused "
                         "decode + message reassembly (use with --config cfg5), or the whole batch as ONE raw "
                         "rx stream with no frame offsets (device-side boundary discovery)")
    args = ap.parse_args()
    # --gpus N means N ranks: launched here (one child process per GPU, before anything touches
    # a GPU) unless a launcher (torchrun) already set WORLD_SIZE, which must then equal N
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
    elif os.environ.get("WS_BENCH_LAUNCH_ECHO"):                   # launcher test (tests/test_dist.py)
        emit({"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
              "local_rank": int(os.environ["LOCAL_RANK"]), "master_port": os.environ["MASTER_PORT"]})
        if os.environ["RANK"] == "0" and os.environ.get("WS_BENCH_LAUNCH_ECHO_HANG"):
            import time                                            # a rank stuck in a rendezvous
            time.sleep(float(os.environ["WS_BENCH_LAUNCH_ECHO_HANG"]))
        sys.exit(int(os.environ.get("WS_BENCH_LAUNCH_ECHO_RC", "0")) if os.environ["RANK"] != "0" else 0)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%s: refusing to report a %s-rank run as %d GPUs\n"
                         % (args.gpus, os.environ["WORLD_SIZE"], os.environ["WORLD_SIZE"], args.gpus))
        sys.exit(2)
    from util_amd import wsframe as W
    path = DEFAULT_PATH if args.path is None else args.path
    if args.path is not None:
        W.set_option("path", args.path)

    import torch
    import torch.distributed as dist
    if args.alloc == "contiguous":                                 # before any device allocation
        from util_amd import _lib
        torch.cuda.memory.change_current_allocator(torch.cuda.memory.CUDAPluggableAllocator(
            _lib.BENCH_LIB_PATH, "websocketframeBenchTorchAlloc", "websocketframeBenchTorchFree"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; WS_BENCH_RANKS_PER_GPU > 1 rehearses the multi-rank path on fewer GPUs
    # (ranks share a device; RCCL needs distinct devices, so that rehearsal runs over gloo)
    per_gpu = int(os.environ.get("WS_BENCH_RANKS_PER_GPU", "1"))
    gpu = local // per_gpu
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if per_gpu > 1:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu)
    if args.op in ("encode", "reasm", "stream") or (args.op == "decode" and args.config in STRONG):
        fn = {"encode": run_encode, "reasm": run_reasm, "stream": run_stream, "decode": run_strong}[args.op]
        out, mism = fn(args, dev, world, rank)
        out["config"]["alloc"] = args.alloc
        if rank == 0:
            emit(out)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(1 if mism else 0)

    nfr = args.frames or Workload.CONFIGS[args.config][0]
    wl = Workload.make(args.config, dev, nframes=args.frames, fps=args.fps, plen=args.plen, first_frame=rank * nfr)
    torch.cuda.synchronize()
    sample = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = wl.host_sample(262144)
    from util_amd import dist as D

    # a plain streaming reference on the same bytes with the same timing method: an in-place XOR
    # of the wire in one-shot 256 x 4 blocks over 16 KiB pieces in the same two windows, no
    # frame logic (calibration kernel, libwsframe_amd_bench.so mode 72) — how close the decode
    # step is to moving the same bytes with nothing else to do; an even number of calls leaves
    # the buffer as it was. (Measured before the decode's warm-up; it does not warm the device
    # up for the decode — tools/exp_ramp.py, DESIGN §4 "Short timed regions".)
    xor_stream = None
    if not args.no_xor_stream:
        lib = wl.W.load_bench_lib()
        nb = wl.wire_bytes // 16 * 16
        st = torch.cuda.current_stream().cuda_stream

        def cstep():
            rc = lib.websocketframeGpuCalibrate(wl.buf.data_ptr(), wl.buf.data_ptr(), nb, 72, 1, 2, st)
            assert rc == 0, "websocketframeGpuCalibrate"
        for _ in range(2):
            cstep()
        n_c = max(100, args.steps + (args.steps & 1))
        _, c_ms = timed_region(cstep, n_c, world)
        c_ms = D.allreduce([c_ms], op="max", device=dev)[0]
        xor_stream = {"what": "in-place XOR of the same wire bytes, one-shot 256 x 4 blocks over 16 KiB pieces in two "
                              "windows (K2's access pattern without frame logic; websocketframeGpuCalibrate mode 72), "
                              "%d calls timed like the step" % n_c,
                      "ms": round(c_ms, 4), "frac": round(2 * nb / (c_ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4)}
    out, mism = run_decode(args, dev, world, rank, wl=wl, path=path)
    if xor_stream is not None:
        xor_stream["step_rate_over_xor_stream"] = round(xor_stream["ms"] / out["roofline"]["step_ms_mean"], 4)
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e, flips = end_to_end(wl)
        wl.decodes += flips
        e2e_mism = wl.verify(expect_plain=(wl.decodes % 2 == 1))
        e2e["verified"] = e2e_mism == 0 and e2e["pageable"]["verified"] and e2e["multi_device"]["verified"]
        mism += e2e_mism
    if args.inflight > 1:
        inflight, m = run_inflight(args, wl, dev, world, rank)
        mism += m
        out["inflight"] = inflight
    out["xor_stream"] = xor_stream
    out["e2e"] = e2e
    if args.scatter and world > 1:                                 # SURVEY §8e (1), outside the timed region
        recv = None if rank == 0 else torch.empty(wl.wire_bytes, dtype=torch.uint8, device=dev)
        dt = D.allreduce([D.scatter_from_root(wl.buf, recv, wl.wire_bytes)], op="max", device=dev)[0]
        out["scatter"] = {"what": "rank 0 sends its wire batch to each other rank, point-to-point sends posted "
                                  "together (RCCL over xGMI), not part of value",
                          "backend": dist.get_backend(), "bytes_per_rank": wl.wire_bytes, "ms": round(dt * 1e3, 3),
                          "GBps_per_link": round(wl.wire_bytes / dt / 1e9, 1),
                          "GBps_total": round((world - 1) * wl.wire_bytes / dt / 1e9, 1)}
        del recv
    # every other single-GPU path of SURVEY §8, timed by the same protocol in the same run
    # (N = 1 only: the scaling points time the headline alone)
    if world == 1 and not args.no_paths and args.config == "cfg2" and args.frames is None:
        wl.free()
        del wl
        out["paths"], m = run_paths(args, dev)
        mism += m
    if sample is not None:                                         # host cores, after every GPU timing
        out["cpu_baseline"] = cpu_baseline(sample, args.cpu_threads or None)
    mism = int(D.allreduce([mism], device=dev)[0])
    out["verified"] = out["verified"] and mism == 0
    out["config"]["alloc"] = args.alloc
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()
    if mism:
        sys.exit(1)


if __name__ == "__main__":
    main()
