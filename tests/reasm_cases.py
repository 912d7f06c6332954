"""Byte streams for the reassembly fixtures (tests/golden/reassemble.json).

Each case is ONE connection's rx byte stream, as a peer would send it; the reference's own
reactor stack (oracle/reactor_harness.c: NetReactor_handle -> on_read_stream -> fragment
cache -> on_recv, net_channel_ex.c:110-157) produced the fixture's deliveries from it, with
the channel's readcache_max_size set to the case's limit. The streams are rebuilt here from
a seed (numpy PCG64); the fixture pins each one by its SHA-256, so a generator change fails
loudly instead of silently testing other bytes.
"""
import hashlib

import numpy as np

FRAG_FIRST, FRAG_MID, FRAG_LAST = 0x02, 0x00, 0x80


def frame(rng, b0, plen, masked=True, form=None):
    """one RFC 6455 frame: header (7/16/64-bit length form; `form` forces a non-minimal one),
    optional 4-byte key, payload (masked with the key when `masked`)"""
    form = form or (7 if plen < 126 else (16 if plen <= 0xFFFF else 64))
    h = bytearray([b0])
    m = 0x80 if masked else 0
    if form == 7:
        h.append(m | plen)
    elif form == 16:
        h += bytes([m | 126]) + plen.to_bytes(2, "big")
    else:
        h += bytes([m | 127]) + plen.to_bytes(8, "big")
    body = rng.integers(0, 256, plen, dtype=np.uint8)
    if masked:
        key = rng.integers(0, 256, 4, dtype=np.uint8)
        h += key.tobytes()
        body = body ^ np.resize(key, plen) if plen else body
    return bytes(h) + body.tobytes()


def message(rng, sizes, masked=True, opcode=2, forms=None):
    """a message of len(sizes) fragments: first carries the opcode, last has FIN"""
    out = []
    n = len(sizes)
    for k, plen in enumerate(sizes):
        b0 = (opcode if k == 0 else 0) | (0x80 if k == n - 1 else 0)
        out.append(frame(rng, b0, int(plen), masked=masked, form=None if forms is None else forms[k]))
    return b"".join(out)


def _cfg5(rng):
    return b"".join(message(rng, [1024] * 16) for _ in range(64)), 0


def _mixed(rng):
    parts = []
    sizes = [0, 1, 5, 125, 126, 127, 1000, 3000, 65535, 65536, 70000]
    w = np.array([3, 3, 3, 3, 2, 2, 4, 3, 1, 1, 1], float)
    w /= w.sum()
    for i in range(300):
        nfr = int(rng.integers(1, 7))
        sz = [int(rng.choice(sizes, p=w)) for _ in range(nfr)]
        masked = rng.random() < 0.9
        forms = None
        if i % 7 == 3:   # non-minimal length encodings (accepted, websocketframe.c:129-145)
            forms = [int(rng.choice([16, 64])) if s < 126 else (64 if s <= 0xFFFF else None) for s in sz]
        m = message(rng, sz, masked=masked, opcode=int(rng.choice([1, 2])), forms=forms)
        if nfr > 1 and i % 5 == 0:
            # a ping (FIN) right after the first fragment: the stream hook caches it as one more
            # fragment and it closes the message (pktype NETPACKET_FRAGMENT for every frame)
            op = int(rng.choice([1, 2]))
            m = (frame(rng, op, sz[0], masked=masked) + frame(rng, 0x89, int(rng.integers(0, 126))) +
                 b"".join(frame(rng, 0x80 if k == nfr - 1 else 0, sz[k], masked=masked) for k in range(1, nfr)))
        parts.append(m)
    return b"".join(parts), 0


def _open_end(rng):
    s = b"".join(message(rng, [int(x) for x in rng.integers(0, 2000, int(rng.integers(1, 5)))]) for _ in range(20))
    open_msg = message(rng, [700, 800, 900])
    cut = len(open_msg) - len(frame(np.random.default_rng(1), 0x80, 900))   # drop the FIN fragment
    return s + open_msg[:cut], 0


def _tail(rng):
    s = b"".join(message(rng, [int(x) for x in rng.integers(0, 3000, int(rng.integers(1, 4)))]) for _ in range(20))
    last = message(rng, [5000])
    return s + last[:2500], 0   # ends inside a frame: the reactor keeps the tail (net_reactor.c:536-539)


def _overflow_count(rng):
    # limit 5000, 1000-B fragments: the 6th fragment of a 7-fragment message overflows
    s = b"".join(message(rng, [1000] * int(n)) for n in (1, 3, 5, 2))
    s += message(rng, [1000] * 7)
    s += message(rng, [10, 10])          # never reached: the channel is detached
    return s, 5000


def _overflow_single(rng):
    # limit 2000: a single non-FIN fragment of 3000 B (max_limit < add_bytes)
    s = message(rng, [500, 500]) + frame(rng, 0x80 | 2, 4000) + message(rng, [3000, 10])
    return s, 2000


def _fin_unchecked(rng):
    # limit 100: a FIN frame with nothing pending is delivered without the check, whatever its
    # size; 40 + 40 fits, 60 + 50 does not (60 > 100 - 50)
    s = frame(rng, 0x82, 5000) + message(rng, [40, 40]) + frame(rng, 0x81, 300) + message(rng, [60, 50])
    return s, 100


def _boundary(rng):
    # limit 3000: cached 2000 + 1000 is exactly the limit (not an overflow: 2000 > 3000 - 1000
    # is false); the next message's 2001 + 1000 overflows
    s = message(rng, [1000, 1000, 1000]) + message(rng, [2001, 1000]) + message(rng, [5])
    return s, 3000


def _zero_len(rng):
    parts = []
    for i in range(40):
        n = int(rng.integers(1, 6))
        parts.append(message(rng, [int(x) for x in rng.integers(0, 3, n)], masked=bool(i % 3)))
    return b"".join(parts), 0


def _interleaved_limit(rng):
    # limit 64 KiB over a long stream of mixed messages, with one too-large message at the end
    s = b"".join(message(rng, [int(x) for x in rng.integers(0, 9000, int(rng.integers(1, 8)))]) for _ in range(120))
    s += message(rng, [30000, 30000, 30000])
    return s, 65536


CASES = {
    "cfg5_shape": (_cfg5, 5),
    "mixed": (_mixed, 6),
    "open_end": (_open_end, 7),
    "tail": (_tail, 8),
    "overflow_count": (_overflow_count, 9),
    "overflow_single": (_overflow_single, 10),
    "fin_unchecked": (_fin_unchecked, 11),
    "boundary": (_boundary, 12),
    "zero_len": (_zero_len, 13),
    "interleaved_limit": (_interleaved_limit, 14),
}


def build(name):
    """(wire bytes as a uint8 array, readcache_max_size) of case `name`"""
    fn, seed = CASES[name]
    wire, limit = fn(np.random.default_rng(seed))
    return np.frombuffer(wire, dtype=np.uint8).copy(), limit


def sha256(b):
    return hashlib.sha256(bytes(b)).hexdigest()
