"""The batch C ABI from plain C (no Python, no torch on the call path): tests/c/batch_host.c
decodes 2,000 host-memory rx inbufs with websocketframeBatchDecodeHost on the GPU and
checks every descriptor, segment result and byte against the reference's per-frame loop
over websocketframeDecode (the host symbols) on a copy."""
import os
import subprocess

import pytest

import util_amd
from util_amd import _lib

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_batch_host_program(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    util_amd.load_lib()
    exe = str(tmp_path / "batch_host")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "batch_host.c"), "-L", libdir, "-lwsframe_amd",
                    "-Wl,-rpath," + libdir, "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("batch_host ok ")
    assert int(out.stdout.split()[-1]) > 5000


def test_c_stream_device_program(tmp_path):
    """tests/c/stream_dev.c: a 24 MiB client stream of changing frame lengths (the
    chunk-parallel walk) through websocketframeStreamDecodeDevice from plain C with the HIP
    runtime API, checked against the reference loop over websocketframeDecode"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    util_amd.load_lib()
    exe = str(tmp_path / "stream_dev")
    libdir = os.path.dirname(_lib.LIB_PATH)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(rocm, "include"),
                    os.path.join(REPO, "tests", "c", "stream_dev.c"), "-L", libdir, "-lwsframe_amd",
                    "-L", os.path.join(rocm, "lib"), "-lamdhip64", "-Wl,-rpath," + libdir,
                    "-Wl,-rpath," + os.path.join(rocm, "lib"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("stream_dev ok ")
    assert int(out.stdout.split()[-1]) > 1000
