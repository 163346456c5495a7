"""Host-side race / memory-error detection for the native code that runs on
CPU threads: the GIL-free JPEG encoder (deconv_api_amd/csrc/jpeg_enc.cpp). It is compiled with
ThreadSanitizer and with AddressSanitizer + UBSan into a standalone stress binary
(tests/native/jpeg_stress.cpp) that encodes the same batches from several caller threads at once.
GPU code is not sanitized (no GPU ASan / XNACK on this pool); device kernels are covered by
bounds-checked bindings, deterministic-repeat and serialized-launch tests (test_kernels_gpu.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "deconv_api_amd", "csrc")
SRC = [os.path.join(ROOT, "tests", "native", "jpeg_stress.cpp"), os.path.join(CSRC, "jpeg_enc.cpp")]


def _build_run(tmp_path, flags, env_extra):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "jpeg_stress")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-pthread", "-DDVJPEG_NO_CLONES", *flags, f"-I{CSRC}", *SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, **env_extra)
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must be first in the process
    r = subprocess.run([exe, "4"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "mismatches=0" in r.stdout
    return r


def test_jpeg_encoder_threadsanitizer(tmp_path):
    r = _build_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_jpeg_encoder_address_ub_sanitizer(tmp_path):
    r = _build_run(tmp_path, ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0"})
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
