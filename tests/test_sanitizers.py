"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (tools/sanitize_host.sh).

The first build takes a few minutes (the HIP translation unit is compiled for gfx950 with an
instrumented host side); later runs reuse the objects under build/sanitize."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(shutil.which('/opt/rocm/bin/hipcc') is None, reason='no ROCm toolchain')
def test_host_code_clean_under_asan_ubsan():
    r = subprocess.run([os.path.join(ROOT, 'tools', 'sanitize_host.sh')], cwd=ROOT, capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert 'host selftest: all checks passed' in r.stdout
    assert 'pool selftest: all checks passed' in r.stdout  # ThreadSanitizer run of csrc/thread_pool.h
