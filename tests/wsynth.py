"""numpy restatement of util_amd/csrc/ws_synth.h (synthetic input generator).

Test helper only: builds masked frame batches on the host at test sizes, and
lets tests check that the C/HIP generator produces the same bytes.
"""
import numpy as np

from util_amd.synth import (  # noqa: F401  (shared length/offset rules)
    U64, PLEN_FIXED, PLEN_MIX3, B0_BINARY, B0_TEXT, B0_FRAG16, mix64, fseed, plens, headlen, wirelens)


def keys(seed, f):
    return (mix64(fseed(seed, f) ^ U64(0x6B6579)) & U64(0xFFFFFFFF)).astype(np.uint32)


def b0s(b0_kind, n):
    f = np.arange(n)
    if b0_kind == B0_TEXT:
        return np.full(n, 0x81, np.uint8)
    if b0_kind == B0_FRAG16:
        j = f & 15
        return np.where(j == 0, 0x02, np.where(j == 15, 0x80, 0x00)).astype(np.uint8)
    return np.full(n, 0x82, np.uint8)


def plain_payload(seed, f, plen):
    """plaintext payload bytes of frame f (uint8 array of length plen)"""
    nw = (int(plen) + 7) // 8
    j = np.arange(nw, dtype=np.uint64)
    with np.errstate(over="ignore"):
        w = mix64(fseed(seed, f) + U64(0x9E3779B97F4A7C15) * (j + U64(1)))
    return w.astype("<u8").view(np.uint8)[: int(plen)]


def header(b0, plen, key):
    plen = int(plen)
    h = [int(b0)]
    if plen < 126:
        h.append(0x80 | plen)
    elif plen <= 0xFFFF:
        h += [0x80 | 126, plen >> 8, plen & 0xFF]
    else:
        h.append(0x80 | 127)
        h += [(plen >> (56 - 8 * i)) & 0xFF for i in range(8)]
    h += [(int(key) >> (8 * i)) & 0xFF for i in range(4)]
    return np.array(h, dtype=np.uint8)


def make_batch(nframes, plen_kind=PLEN_FIXED, fixed_len=4096, b0_kind=B0_BINARY, seed=1, first=0):
    """returns (wire bytes uint8, frame_off uint64, plen uint64, plain bytes concatenated
    in wire layout, i.e. the expected buffer after one decode) of generator frames
    first .. first + nframes - 1"""
    pl = plens(plen_kind, fixed_len, seed, nframes, first)
    wl = wirelens(pl)
    off = np.zeros(nframes, dtype=np.uint64)
    if nframes > 1:
        off[1:] = np.cumsum(wl[:-1], dtype=np.uint64)
    total = int(wl.sum()) if nframes else 0
    wire = np.empty(total, dtype=np.uint8)
    plain = np.empty(total, dtype=np.uint8)
    ks = keys(seed, np.arange(first, first + nframes, dtype=np.uint64))
    b0 = b0s(b0_kind, first + nframes)[first:]
    for f in range(nframes):
        h = header(b0[f], pl[f], ks[f])
        o = int(off[f])
        hl = len(h)
        p = plain_payload(seed, first + f, pl[f])
        kb = np.frombuffer(int(ks[f]).to_bytes(4, "little"), dtype=np.uint8)
        m = p ^ np.resize(kb, len(p)) if len(p) else p
        wire[o:o + hl] = h
        wire[o + hl:o + hl + len(p)] = m
        plain[o:o + hl] = h
        plain[o + hl:o + hl + len(p)] = p
    return wire, off, pl, plain
