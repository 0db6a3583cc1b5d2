"""Host-code sanitizers over the native runtime: ThreadSanitizer on the lock-free
trace ring written by 8 threads, AddressSanitizer + UBSan on the scheduler and arena layout.
(GPU-side sanitizers are not available on this pool; device kernels are covered by the fp32-oracle
numerics tests instead.)"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "native", "runtime_stress.cpp"),
       os.path.join(os.path.dirname(HERE), "fedml_amd", "csrc", "runtime.cpp"),
       os.path.join(os.path.dirname(HERE), "fedml_amd", "csrc", "stream_check.cpp")]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_runtime_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / f"stress_{san.split(',')[0]}")
    cmd = ["g++", "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread", *SRC,
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer toolchain unavailable: {r.stderr[-300:]}")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime stress ok" in r.stdout
