"""Host bookkeeping of libmq_aead.so without a GPU.

tests/csrc/test_runtime.cpp drives milli_quic_amd/csrc/mq_runtime.h — the per-thread device
selection behind mq_device_init, the device guard every call on a key table / context runs under,
and the side streams per (device, caller stream) of the forked tile kernels — against a fake
backend that models HIP's per-thread current device, built with AddressSanitizer and
UndefinedBehaviorSanitizer. The C ABI's device entry points are checked through ctypes."""
import ctypes
import os
import shutil
import subprocess

import pytest

from milli_quic_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_runtime_bookkeeping_asan_ubsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "test_runtime"
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-Werror", "-pthread",
                    os.path.join(ROOT, "tests", "csrc", "test_runtime.cpp"), "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "runtime ok" in r.stdout


def test_device_entry_points_without_gpu(mqlib):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert mqlib.mq_device_init(0) == _lib.MQ_ERR_NO_DEVICE
    assert mqlib.mq_device_init(-1) == _lib.MQ_ERR_NO_DEVICE
    assert mqlib.mq_device_current() == -1
    assert mqlib.mq_keytable_device(None) == -1
    mqlib.mq_stream_release(None)  # nothing registered: a no-op
    h = ctypes.c_void_p()
    km = (_lib.KeyMaterial * 1)()
    assert mqlib.mq_keytable_create(km, 1, ctypes.byref(h)) == _lib.MQ_ERR_NO_DEVICE and not h.value
