"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
section 5).  CPU only, no GPU: tests/tools/asan.mk builds the C-ABI host
sources (hpdct_api.cpp, hpdct_compat.cpp, hpdct_stream.cpp), the oracle and
host/image_io.hpp with g++ -fsanitize=address,undefined into
build/asan/asan_host_check, which drives every host path that runs without a
device (helpers, quant-table mutex from 8 threads, argument validation of
every entry point, oracle transforms at ragged sizes, PGM parsing of hostile
headers).  Any sanitizer report fails the run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MK = os.path.join(ROOT, "tests", "tools", "asan.mk")
KOBJ = os.path.join(ROOT, "cuda-dct-idct_amd", "build", "hpdct_fwd_u8.o")


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="needs g++ and the ROCm headers")
@pytest.mark.skipif(not os.path.exists(KOBJ), reason="library objects not built (__graft_entry__.build())")
def test_host_code_clean_under_asan_ubsan(tmp_path):
    b = subprocess.run(["make", "-s", "-f", MK], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "asan_host_check"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asan_host_check: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
