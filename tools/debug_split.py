"""Debug helper: run one batch through the default path and report where it differs from the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import wsynth
    from oracle_lib import oracle_segments, used_descs
    from util_amd import wsframe as W
    dev = torch.device("cuda:0")
    for (n, pk, fl, fps) in [(32, 0, 4096, 16), (64, 1, 0, 16), (16, 0, 100, 4)]:
        wire, off, pl, plain = wsynth.make_batch(n, pk, fl, 0, 7)
        seg_off = [int(off[i]) for i in range(0, n, fps)]
        ends = [int(off[i + fps]) if i + fps < n else len(wire) for i in range(0, n, fps)]
        seg_len = [e - s for s, e in zip(seg_off, ends)]
        d = torch.zeros(len(wire) + 64, dtype=torch.uint8, device=dev)
        d[:len(wire)] = torch.from_numpy(wire.copy()).to(dev)
        so = torch.tensor(seg_off, dtype=torch.int64, device=dev)
        sl = torch.tensor(seg_len, dtype=torch.int64, device=dev)
        desc = torch.zeros(len(seg_off) * fps * 32, dtype=torch.uint8, device=dev)
        res = torch.zeros(len(seg_off) * 16, dtype=torch.uint8, device=dev)
        W.batch_decode_device(d, so, sl, fps, desc, res)
        torch.cuda.synchronize()
        gb = d[:len(wire)].cpu().numpy()
        gd = desc.cpu().numpy().view(W.DESC_DTYPE)
        gr = res.cpu().numpy().view(W.SEGRES_DTYPE)
        ob = wire.copy()
        od, orr = oracle_segments(ob, seg_off, seg_len, fps)
        print("case", n, pk, fl, fps, "res_eq", np.array_equal(gr, orr), "desc_eq",
              np.array_equal(used_descs(gd, gr, fps), used_descs(od, orr, fps)))
        bad = np.nonzero(gb != ob)[0]
        print("  bad bytes", len(bad), "of", len(ob))
        if len(bad):
            fr = np.searchsorted(off.astype(np.int64), bad, side="right") - 1
            rel = bad - off[fr].astype(np.int64)
            print("  first bad", bad[:10], "frames", fr[:10], "rel", rel[:10])
            print("  got", gb[bad[:8]], "want", ob[bad[:8]], "wire", wire[bad[:8]])
            print("  frames with bad bytes", np.unique(fr)[:20], "count", len(np.unique(fr)))


if __name__ == "__main__":
    main()


def random_case(seed=1, max_frames=16, nseg=3000):
    import torch
    from test_gpu_parity import random_stream, gpu_decode
    from oracle_lib import oracle_segments, used_descs
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, nseg)
    gb, gd, gr = gpu_decode(torch.device("cuda:0"), wire.copy(), so, sl, max_frames)
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, max_frames)
    bad = np.nonzero(gr != orr)[0]
    print("random seed", seed, "max_frames", max_frames, "bad segments", len(bad))
    for i in bad[:5]:
        print("  seg", i, "off", so[i], "len", sl[i], "gpu", gr[i], "oracle", orr[i])
        seg = ob[so[i]:so[i] + sl[i]]
        # walk with the oracle result to show frame lengths
        from util_amd import wsframe as W
        print("   first bytes", wire[so[i]:so[i] + 24].tobytes().hex())
    print("  bytes differ", int((gb != ob).sum()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "rand":
    for sd, mf in [(1, 16), (2, 3), (3, 1), (4, 64)]:
        random_case(sd, mf)


def isolate(seed=3, max_frames=1):
    import torch
    from test_gpu_parity import random_stream, gpu_decode
    from oracle_lib import oracle_segments
    from util_amd import wsframe as W
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 3000)
    dev = torch.device("cuda:0")
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, max_frames)
    for path in (2, 0, 1):
        W.set_option("path", path)
        gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, max_frames)
        bad = np.nonzero(gr != orr)[0]
        print("path", path, "bad segs", len(bad), "bytes differ", int((gb != ob).sum()), "first", bad[:6])
    W.set_option("path", 0)
    gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, max_frames)
    bad = np.nonzero(gr != orr)[0]
    for i in bad[:4]:
        one = wire[so[i]:so[i] + sl[i]].copy()
        b1, d1, r1 = gpu_decode(dev, one, [0], [sl[i]], max_frames)
        pad = np.concatenate([np.zeros(5, np.uint8), one])
        b2, d2, r2 = gpu_decode(dev, pad, [5], [sl[i]], max_frames)
        print("seg", i, "batch", gr[i], "alone", r1[0], "alone@5", r2[0], "oracle", orr[i])
    # only every other segment (no neighbours)
    idx = np.arange(0, len(so), 2)
    gb, gd, gr = gpu_decode(dev, wire.copy(), [so[j] for j in idx], [sl[j] for j in idx], max_frames)
    ob2 = wire.copy()
    od2, orr2 = oracle_segments(ob2, [so[j] for j in idx], [sl[j] for j in idx], max_frames)
    print("even segments only: bad", int((gr != orr2).sum()))
    # one segment per launch... serial
    import time
    torch.cuda.synchronize()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "iso":
    isolate()


def locate(seed=3, max_frames=1):
    import torch
    from test_gpu_parity import random_stream, gpu_decode
    from oracle_lib import oracle_segments
    from util_amd import wsframe as W
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 3000)
    dev = torch.device("cuda:0")
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, max_frames)
    owner = np.full(len(wire), -1, np.int64)
    for i in range(len(so)):
        owner[so[i]:so[i] + sl[i]] = i
    for nt in (1, 0):
        W.set_option("nt", nt)
        gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, max_frames)
        bad = np.nonzero(gr != orr)[0]
        diff = np.nonzero(gb != ob)[0]
        print("nt", nt, "bad segs", len(bad), "diff bytes", len(diff))
        # bytes outside any segment that changed
        outside = diff[owner[diff] < 0]
        print("  changed bytes outside segments:", len(outside), outside[:8])
        # bytes inside segment i that changed although oracle did not change them
        unchanged_in_oracle = diff[(ob[diff] == wire[diff])]
        print("  bytes the oracle leaves alone but GPU changed:", len(unchanged_in_oracle),
              [(int(x), int(owner[x]), int(x - so[owner[x]]) if owner[x] >= 0 else -1) for x in unchanged_in_oracle[:8]])
        for i in bad[:3]:
            hdr_changed = np.nonzero(gb[so[i]:so[i] + 14] != wire[so[i]:so[i] + 14])[0]
            print("  seg", i, "gpu", gr[i], "oracle", orr[i], "header bytes changed at", hdr_changed)
    W.set_option("nt", 1)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "loc":
    locate()


def walkonly(seed=3, max_frames=1):
    import torch
    from test_gpu_parity import random_stream, gpu_decode
    from oracle_lib import oracle_segments
    from util_amd import wsframe as W
    rng = np.random.default_rng(seed)
    wire, so, sl = random_stream(rng, 3000)
    dev = torch.device("cuda:0")
    ob = wire.copy()
    od, orr = oracle_segments(ob, so, sl, max_frames)
    for dbg in (1, 0, 1, 0):
        W.set_option("debug", dbg)
        gb, gd, gr = gpu_decode(dev, wire.copy(), so, sl, max_frames)
        bad = np.nonzero(gr != orr)[0]
        print("debug", dbg, "bad segs", len(bad), bad[:5], "bytes changed vs input", int((gb != wire).sum()))
    W.set_option("debug", 0)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "walk":
    walkonly()
