"""The GPU batch binding at the reactor, on the GPU: the reference's own
reactor and stream hook (oracle/_ref, compiled from the reference sources — test
infrastructure, present wherever `make -C oracle ref` ran) with several connections whose
streams arrive in small writes; every round ONE websocketframeBatchDecodeHost call (GPU)
decodes every readable connection's whole inbuf (the previous read's undecoded tail first),
and each connection's on_read loop replays it through websocketframeOnDecodeBatch. Deliveries
must equal the reference reactor's own (tests/golden/reassemble.json)."""
import ctypes as C

import pytest

from test_oracle_golden import _batched_reactor_check, _reference_reactor
from util_amd import load_lib

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


# (chunk 7 = 1.6 M batch decodes: on the oracle only, tests/test_oracle_golden.py; chunk 100 = 113 K)
@pytest.mark.parametrize("chunk,max_frames", [(100, 64), (1500, 64), (1500, 3), (65536, 64), (65536, 3)])
def test_batched_reactor_binding_gpu(golden, chunk, max_frames):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _reference_reactor()
    fn = C.cast(load_lib().websocketframeBatchDecodeHost, C.c_void_p).value
    assert _batched_reactor_check(golden, chunk, gpu_fn=fn, max_frames=max_frames) > 0
