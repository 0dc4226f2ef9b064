"""The host-only native code under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY §5): csrc/sais.h (host suffix sorting), csrc/fileformat.h (fm_save /
fm_load's parse, with truncated and corrupt files) and oracle/cpu_ref.cpp,
compiled here with g++ into tests/native/host_checks.cpp's harness and run.
CPU only: GPU code is never run under a sanitizer (the pool refuses it)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.timeout(600)
def test_host_code_under_asan_ubsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_checks"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-pthread", os.path.join(HERE, "native", "host_checks.cpp"),
           os.path.join(REPO, "oracle", "cpu_ref.cpp"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None) if "asan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env, timeout=500)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "all host checks passed" in out
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-6000:]
