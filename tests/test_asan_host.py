"""Host-code sanitizer run (SURVEY.md §5 "race detection / sanitizers"): the CPU suite's C-ABI
tests (tests/test_host.py, tests/test_sch_host.py — argument validation of every entry point,
ldpc5g_sch_config, the mixed-Zc and per-TB plans) re-run in a subprocess against
build/asan/libldpc5g.so, the library's host code compiled with AddressSanitizer +
UndefinedBehaviorSanitizer (python_5gtoolbox_amd.build.build_asan; host-only objects, so no
device code).  Any ASan / UBSan report aborts the subprocess and fails this test."""
import os
import subprocess
import sys

import pytest

from python_5gtoolbox_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(2400)   # a stale sanitizer build recompiles changed TUs first
def test_capi_host_code_under_asan_ubsan():
    lib = build.build_asan()
    rt = build.asan_runtime()
    assert os.path.exists(rt), rt
    env = dict(os.environ, LD_PRELOAD=rt, LDPC5G_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "not gpu", "tests/test_host.py", "tests/test_sch_host.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=580)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in tail and "runtime error" not in tail, tail
