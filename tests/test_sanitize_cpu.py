"""Host-code sanitizers (no sanitizer build of the host library):
the expression compiler and the CSV reader of libdfmi, and the CPU oracle,
built with AddressSanitizer + UndefinedBehaviorSanitizer (tests/native) and
driven over random expressions / batches and generated CSV files. Device
code is not sanitized here (GPU ASan is not available on the pool)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_asan_ubsan(tmp_path):
    out = str(tmp_path / "sanitize_driver")
    b = subprocess.run(["make", "-s", "-C", os.path.join(HERE, "native"), "OUT=" + out], capture_output=True,
                       text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([out], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "sanitize driver: clean" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
