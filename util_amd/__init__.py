"""util_amd — MI355X-native drop-in for hujianzhe/util's WebSocket frame decode path.

The product is the C-ABI library ``libwsframe_amd.so`` (include/wsframe_amd.h):
the eight ``websocketframe*`` symbols of inc/crt/protocol/websocketframe.h:42-49
plus a batch API whose kernels run on gfx950. This package is the thin Python
mirror used by tests and bench.py; it never computes anything itself.
"""
from ._lib import LIB_PATH, load_lib, build_lib  # noqa: F401
from .wsframe import (  # noqa: F401
    WEBSOCKET_CONTINUE_FRAME, WEBSOCKET_TEXT_FRAME, WEBSOCKET_BINARY_FRAME, WEBSOCKET_CLOSE_FRAME,
    WEBSOCKET_PING_FRAME, WEBSOCKET_PONG_FRAME, WEBSOCKET_MAX_ENCODE_HEADLENGTH,
    DESC_DTYPE, SEGRES_DTYPE, ENC_DTYPE, DATA_OFF_NULL,
    SEG_OK, SEG_MAX_FRAMES, SEG_ERR_DECODE, SEG_ERR_LEN_WRAP,
    websocketframeDecode, websocketframeEncodeHeadLength, websocketframeEncode,
    websocketframeComputeSecAccept, websocketframeDecodeHandshakeRequest,
    websocketframeEncodeHandshakeResponse, websocketframeEncodeHandshakeResponseWithProtocol,
    batch_decode_device, batch_decode_host, batch_encode_device, synth_device, synth_verify_device,
)
