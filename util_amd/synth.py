"""Host-side layout of synthetic batches (numpy restatement of the length/offset
rules of util_amd/csrc/ws_synth.h). Bench/test input only: the bytes themselves
are generated on the device by websocketframeSynthDevice."""
import numpy as np

U64 = np.uint64
PLEN_FIXED, PLEN_MIX3 = 0, 1
B0_BINARY, B0_TEXT, B0_FRAG16 = 0, 1, 2


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + U64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> U64(30))) * U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U64(27))) * U64(0x94D049BB133111EB)
        return z ^ (z >> U64(31))


def fseed(seed, f):
    f = np.asarray(f, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(U64(seed) ^ (f * U64(0xD1B54A32D192ED03)))


def plens(plen_kind, fixed_len, seed, n, first=0):
    """payload lengths of generator frames first .. first + n - 1"""
    f = np.arange(first, first + n, dtype=np.uint64)
    if plen_kind == PLEN_MIX3:
        r = mix64(fseed(seed, f) ^ U64(0x4C454E)) % U64(3)
        return np.choose(r.astype(np.int64), [125, 1500, 65536]).astype(np.uint64)
    return np.full(n, fixed_len, dtype=np.uint64)


def headlen(plen):
    plen = np.asarray(plen, dtype=np.uint64)
    return np.where(plen < 126, 2, np.where(plen <= 0xFFFF, 4, 10)).astype(np.uint64)


def wirelens(plen):
    return headlen(plen) + U64(4) + np.asarray(plen, dtype=np.uint64)
