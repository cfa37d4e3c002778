"""Build the native runtime cores (block manager, AES-GCM) into a standalone binary under
AddressSanitizer + UndefinedBehaviorSanitizer and run it (host code only — GPU sanitizers are
unavailable on this pool).  Mirrors the reference's race-detector test runs
(``go test -race``) for the native parts of this framework."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_native_cores_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "test_native")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-I", os.path.join(REPO, "csrc"),
           os.path.join(REPO, "csrc", "tests", "test_native.cpp"), "-lcrypto", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native tests OK" in r.stdout
