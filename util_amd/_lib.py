"""Locate, build and load libwsframe_amd.so (in-tree, next to this file).

Fails loudly: there is no Python or CPU fallback for the batch path.
"""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# (WSFRAME_AMD_LIB: another build of the same library, for A/B measurements only)
LIB_PATH = os.environ.get("WSFRAME_AMD_LIB") or os.path.join(HERE, "libwsframe_amd.so")
# bench / test support (synthetic batches generated in HBM, calibration): NOT the drop-in
BENCH_LIB_PATH = os.path.join(HERE, "libwsframe_amd_bench.so")
_lib = None
_bench = None


class WsDesc(C.Structure):
    _fields_ = [("frame_off", C.c_ulonglong), ("data_off", C.c_ulonglong), ("datalen", C.c_ulonglong),
                ("ret", C.c_int), ("is_fin", C.c_ubyte), ("type", C.c_ubyte), ("masked", C.c_ubyte),
                ("hdrlen", C.c_ubyte)]


class WsSegRes(C.Structure):
    _fields_ = [("consumed", C.c_ulonglong), ("n_frames", C.c_uint), ("status", C.c_int)]


# the reference's eight symbols (inc/crt/protocol/websocketframe.h:42-49)
REFERENCE_EXPORTS = [
    "websocketframeComputeSecAccept", "websocketframeDecodeHandshakeRequest",
    "websocketframeEncodeHandshakeResponse", "websocketframeEncodeHandshakeResponseWithProtocol",
    "websocketframeFreeString", "websocketframeDecode", "websocketframeEncodeHeadLength",
    "websocketframeEncode",
]
# every symbol include/wsframe_amd.h + include/wsframe_amd_channel.h declare: the whole
# dynamic symbol table of libwsframe_amd.so
EXPORTS = REFERENCE_EXPORTS + [
    "websocketframeBatchDecodeDevice", "websocketframeBatchDecodeHost", "websocketframeBatchDecodeHostMulti",
    "websocketframeBatchEncodeDevice", "websocketframeBatchReassembleDevice",
    "websocketframeBatchReassembleDeviceEx", "websocketframeStreamDecodeDevice",
    "websocketframeGpuLastError", "websocketframeGpuSetOption", "websocketframeGpuGetStat",
    "websocketframeOnDecode", "websocketframeOnDecodeBatch",
]
# include/wsframe_amd_bench.h (libwsframe_amd_bench.so)
BENCH_EXPORTS = ["websocketframeSynthDevice", "websocketframeSynthVerifyDevice", "websocketframeGpuCalibrate",
                 "websocketframeBenchLastError", "websocketframeSynthDeviceRange",
                 "websocketframeSynthVerifyDeviceRange", "websocketframeFrameHashDevice",
                 "websocketframeBenchAlloc", "websocketframeBenchFree", "websocketframeBenchTorchAlloc",
                 "websocketframeBenchTorchFree"]


def build_lib(force=False):
    """make -C util_amd/csrc (hipcc --offload-arch=gfx950 + gcc)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "csrc")] + (["-B"] if force else []), check=True)
    return LIB_PATH


def _one_hip_runtime():
    """Load torch (when installed) before our libraries: torch's ROCm wheel carries its own
    libamdhip64 (soname libamdhip64.so.7, NEEDED as "libamdhip64.so"), so a library of ours
    loaded first would pull /opt/rocm's copy in and the process would hold two HIP runtimes
    (kernels of the second one then see no device). Loaded after torch, ours bind to torch's."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_lib():
    global _lib
    if _lib is not None:
        return _lib
    _one_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libwsframe_amd.so not built: run __graft_entry__.build() "
                           "(make -C util_amd/csrc); there is no fallback path")
    lib = C.CDLL(LIB_PATH)
    vp, u64, u32, i32 = C.c_void_p, C.c_ulonglong, C.c_uint, C.c_int
    P = C.POINTER
    lib.websocketframeDecode.restype = i32
    lib.websocketframeDecode.argtypes = [vp, u64, P(vp), P(u64), P(i32), P(i32)]
    lib.websocketframeEncodeHeadLength.restype = u32
    lib.websocketframeEncodeHeadLength.argtypes = [u64]
    lib.websocketframeEncode.restype = None
    lib.websocketframeEncode.argtypes = [vp, i32, i32, i32, u64]
    lib.websocketframeComputeSecAccept.restype = vp
    lib.websocketframeComputeSecAccept.argtypes = [C.c_char_p, u32, vp]
    lib.websocketframeDecodeHandshakeRequest.restype = i32
    lib.websocketframeDecodeHandshakeRequest.argtypes = [vp, u32, P(vp), P(u32), P(vp), P(u32)]
    lib.websocketframeEncodeHandshakeResponse.restype = vp
    lib.websocketframeEncodeHandshakeResponse.argtypes = [C.c_char_p, u32, vp]
    lib.websocketframeEncodeHandshakeResponseWithProtocol.restype = vp
    lib.websocketframeEncodeHandshakeResponseWithProtocol.argtypes = [C.c_char_p, u32, C.c_char_p, u32]
    lib.websocketframeFreeString.restype = None
    lib.websocketframeFreeString.argtypes = [vp]
    lib.websocketframeBatchDecodeDevice.restype = i32
    lib.websocketframeBatchDecodeDevice.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, vp, vp]
    lib.websocketframeBatchReassembleDevice.restype = i32
    lib.websocketframeBatchReassembleDevice.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.websocketframeStreamDecodeDevice.restype = i32
    lib.websocketframeStreamDecodeDevice.argtypes = [vp, u64, u32, vp, vp, vp]
    lib.websocketframeBatchEncodeDevice.restype = i32
    lib.websocketframeBatchEncodeDevice.argtypes = [vp, vp, u32, vp, u64, vp, vp]
    lib.websocketframeBatchDecodeHost.restype = i32
    lib.websocketframeBatchDecodeHost.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, i32]
    lib.websocketframeBatchDecodeHostMulti.restype = i32
    lib.websocketframeBatchDecodeHostMulti.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, vp, i32]
    lib.websocketframeGpuLastError.restype = C.c_char_p
    lib.websocketframeGpuLastError.argtypes = []
    lib.websocketframeGpuSetOption.restype = i32
    lib.websocketframeGpuSetOption.argtypes = [C.c_char_p, C.c_longlong]
    lib.websocketframeGpuGetStat.restype = i32
    lib.websocketframeGpuGetStat.argtypes = [C.c_char_p, P(C.c_ulonglong)]
    lib.websocketframeBatchReassembleDeviceEx.restype = i32
    lib.websocketframeBatchReassembleDeviceEx.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, vp, vp, vp, vp, vp, u32, vp,
                                                          vp]
    lib.websocketframeOnDecode.restype = None
    lib.websocketframeOnDecode.argtypes = [vp, vp, C.c_size_t, vp]
    lib.websocketframeOnDecodeBatch.restype = None
    lib.websocketframeOnDecodeBatch.argtypes = [vp, vp, C.c_size_t, vp]
    # launch tuning from the environment, e.g. WSFRAME_AMD_OPTIONS="path=0,seg_cfg=10"
    for kv in filter(None, os.environ.get("WSFRAME_AMD_OPTIONS", "").split(",")):
        name, _, value = kv.partition("=")
        if lib.websocketframeGpuSetOption(name.strip().encode(), int(value)) != 0:
            raise ValueError("WSFRAME_AMD_OPTIONS: unknown option %r" % name)
    _lib = lib
    return lib


def load_bench_lib():
    """libwsframe_amd_bench.so: synthetic batches in HBM + calibration kernels (bench/tests)"""
    global _bench
    if _bench is not None:
        return _bench
    _one_hip_runtime()
    if not os.path.exists(BENCH_LIB_PATH):
        raise RuntimeError("libwsframe_amd_bench.so not built: run __graft_entry__.build()")
    lib = C.CDLL(BENCH_LIB_PATH)
    vp, u64, i32 = C.c_void_p, C.c_ulonglong, C.c_int
    lib.websocketframeGpuCalibrate.restype = i32
    lib.websocketframeGpuCalibrate.argtypes = [vp, vp, u64, i32, i32, i32, vp]
    lib.websocketframeSynthDevice.restype = i32
    lib.websocketframeSynthDevice.argtypes = [vp, vp, u64, i32, u64, i32, u64, vp]
    lib.websocketframeSynthVerifyDevice.restype = i32
    lib.websocketframeSynthVerifyDevice.argtypes = [vp, vp, u64, i32, u64, u64, i32, vp, vp]
    lib.websocketframeSynthDeviceRange.restype = i32
    lib.websocketframeSynthDeviceRange.argtypes = [vp, vp, u64, u64, i32, u64, i32, u64, vp]
    lib.websocketframeSynthVerifyDeviceRange.restype = i32
    lib.websocketframeSynthVerifyDeviceRange.argtypes = [vp, vp, u64, u64, i32, u64, u64, i32, vp, vp]
    lib.websocketframeFrameHashDevice.restype = i32
    lib.websocketframeFrameHashDevice.argtypes = [vp, vp, vp, C.c_uint, C.c_uint, vp, vp]
    lib.websocketframeBenchLastError.restype = C.c_char_p
    lib.websocketframeBenchLastError.argtypes = []
    _bench = lib
    return lib


def check(rc, what):
    if rc != 0:
        err = load_lib().websocketframeGpuLastError().decode(errors="replace")
        raise RuntimeError("%s failed (%d): %s" % (what, rc, err))


def check_bench(rc, what):
    if rc != 0:
        err = load_bench_lib().websocketframeBenchLastError().decode(errors="replace")
        raise RuntimeError("%s failed (%d): %s" % (what, rc, err))
