"""The host products (norm_amd/csrc/host_gf8.cpp) under AddressSanitizer + UBSan: every length
0..299, every form this CPU has, exact-size buffers (tests/native/host_gf_asan.cpp).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None,
                    reason="needs hipcc (host compile only)")
def test_host_products_clean_under_asan():
    b = subprocess.run(["make", "-s", "-C", NATIVE, "asan"], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(NATIVE, "_build", "host_gf_asan")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "asan driver done" in r.stdout
