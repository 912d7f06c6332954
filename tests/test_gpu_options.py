"""Every value of every launch option websocketframeGpuSetOption documents
(include/wsframe_amd.h) gives results bit-identical to the oracle: one matrix case per
(option, value), each running the same small workloads through the decode (irregular and
uniform batches), raw stream, reassembly and encode entry points. The focused tests of each
option (test_gpu_stream.py, test_gpu_reasm.py, test_gpu_encode.py,
test_gpu_parity.py::test_window_mappings) cover the shapes where a value changes the launch."""
import numpy as np
import pytest

import wsynth
from oracle_lib import oracle_encode_frames
from test_gpu_encode import gpu_encode, random_frames
from test_gpu_parity import _host_vs_oracle, assert_same, random_stream
from test_gpu_reasm import check as reasm_check
from test_gpu_stream import long_stream, mix3, run as stream_run
from util_amd import wsframe as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

DEFAULTS = {"path": -1, "scan_alpha": 1, "host_chunk_mb": 64, "piece_lds": 0,
            "piece_win": -1, "seg_win": -1, "reasm_path": 0, "reasm_cfg": 0, "enc_front": 1, "stream_rw": 1,
            "stream_rw_cmax": 22, "stream_rounds": 4, "stream_plink": 1, "stream_split": 8, "stream_split_wait": 0,
            "stream_c0": 3, "stream_side_prio": 0, "stream_split2": 48, "stream_c1": 2, "stream_split_capture": 1, "stream_win": 2, "k2_timing": 0}

VALUES = {"path": [-1, 1, 3, 4], "scan_alpha": [0, 1],
          "host_chunk_mb": [1, 64], "piece_lds": [0, 1, 56000], "piece_win": [-1, 0, 1, 2, 3, 4, 5, 6],
          "seg_win": [-1, 0, 1, 2, 3], "reasm_path": [0, 1, 2], "reasm_cfg": [0, 1, 2], "enc_front": [0, 1],
          "stream_rw": [0, 1, 2], "stream_rw_cmax": [16, 20, 23, 26], "stream_rounds": [1, 4, 64], "stream_plink": [0, 1],
          "stream_split": [0, 1, 16, 128, 255], "stream_split_wait": [0, 1, 2], "stream_c0": [0, 2, 6],
          "stream_side_prio": [0, 1, 2], "stream_split2": [0, 64, 200], "stream_c1": [0, 1, 3], "stream_split_capture": [0, 1], "stream_win": [-1, 0, 1, 3],
          "k2_timing": [0, 1]}

# options that act only inside the piece path: the case runs it
CONTEXT = {"piece_lds": {"path": 3}, "piece_win": {"path": 3}, "scan_alpha": {"path": 3}}

CASES = [(o, v) for o, vals in VALUES.items() for v in vals]


def test_matrix_names_every_option():
    """the matrix and the header list the same option names"""
    hdr = open(__file__.rsplit("/tests/", 1)[0] + "/include/wsframe_amd.h").read()
    block = hdr[hdr.index("/* Launch tuning knobs"):hdr.index("WSFRAME_AMD_EXPORT int websocketframeGpuSetOption")]
    import re
    named = set(re.findall(r'"([a-z0-9_]+)"', block))
    assert named == set(VALUES), named ^ set(VALUES)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def work():
    rng = np.random.default_rng(4242)
    irregular = random_stream(rng, 300)
    uw, off, *_ = wsynth.make_batch(16 * 300, 0, 1024, 2, 91)
    so = [int(off[i]) for i in range(0, 16 * 300, 16)]
    uniform = (uw, so, [e - s for s, e in zip(so, so[1:] + [len(uw)])])
    mixed, moff, *_ = wsynth.make_batch(2100, wsynth.PLEN_MIX3, 0, wsynth.B0_BINARY, 92)
    mso = [int(moff[i]) for i in range(0, 2100, 16)]
    mixed = (mixed, mso, [e - s for s, e in zip(mso, mso[1:] + [len(mixed)])])
    short_stream = long_stream(np.random.default_rng(93), 1 << 20, mix3)
    big_stream = long_stream(np.random.default_rng(94), 17 << 20, mix3)
    enc = random_frames(np.random.default_rng(95), 300)
    return irregular, uniform, mixed, short_stream, big_stream, enc


@pytest.mark.parametrize("opt,val", CASES, ids=["%s=%d" % c for c in CASES])
def test_option_value_parity(dev, work, opt, val):
    irregular, uniform, mixed, short_stream, big_stream, (src, fr) = work
    ctx = dict(CONTEXT.get(opt, {}))
    try:
        for k, v in ctx.items():
            W.set_option(k, v)
        W.set_option(opt, val)
        tag = "%s=%d" % (opt, val)
        for rep in range(2):            # twice: the adaptive choice and the hint take effect on the 2nd call
            for i, (wire, so, sl) in enumerate((uniform, mixed, irregular)):
                assert_same(dev, wire, so, sl, 16, tag="%s batch %d rep %d" % (tag, i, rep))
        if opt == "host_chunk_mb":
            _host_vs_oracle(uniform[0].copy(), uniform[1], uniform[2], 16, tag)
        stream_run(dev, short_stream, 1 << 14)
        if opt.startswith("stream_") or opt == "path":
            stream_run(dev, big_stream, 1 << 16)
        wire, so, sl = irregular
        reasm_check(dev, wire, so, sl, 16, tag=tag)
        want, woff = oracle_encode_frames(src, fr)
        out, off = gpu_encode(dev, src, fr)
        assert np.array_equal(off, woff), tag
        assert np.array_equal(out[:len(want)], np.frombuffer(want, dtype=np.uint8)), tag
        if opt == "k2_timing" and val:
            assert W.get_stat("k2_calls") > 0
    finally:
        for k in set(ctx) | {opt}:
            W.set_option(k, DEFAULTS[k])


def test_out_of_range_values_refused():
    for opt, bad in [("path", 2), ("piece_win", 7), ("seg_win", 4), ("seg_win", -2), ("scan_alpha", 2),
                     ("reasm_path", 3), ("reasm_cfg", 3), ("enc_front", 2), ("stream_rw_cmax", 27),
                     ("stream_rounds", 0), ("host_chunk_mb", 0), ("piece_lds", -1),
                     ("stream_split", 256), ("stream_split_wait", 3), ("stream_c0", 7), ("stream_split2", 256),
                     ("stream_c1", 7), ("stream_split_capture", 2), ("stream_win", 7), ("stream_win", -2)]:
        with pytest.raises(ValueError):
            W.set_option(opt, bad)
