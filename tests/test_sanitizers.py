"""Host C++ under the sanitizers (tools/sanitize_host.sh): the host crypto self-test under ASan + UBSan and
the host pool under TSan; libFuzzer + ASan + UBSan on the network parsers (tx decoder, HTTP/WebSocket
framing, the span JSON parser differential against json.loads); and the Python tests of every pybind11
module with the whole extension instrumented, under ASan + UBSan and (the threaded ones) TSan.

The first run builds the instrumented objects and extensions (several minutes); later runs reuse them
under build/sanitize and build/native-{asan,tsan}."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(shutil.which('/opt/rocm/bin/hipcc') is None, reason='no ROCm toolchain')
def test_host_code_clean_under_sanitizers_and_fuzzing():
    # the span-parser fuzzer's 10 M-execution run is tools/sanitize_host.sh's own default; here a short one
    env = dict(os.environ, FUZZ_SECONDS=os.environ.get('FUZZ_SECONDS', '10'),
               FUZZ_JSONSPAN_RUNS=os.environ.get('FUZZ_JSONSPAN_RUNS', '100000'), FUZZ_JOBS='4')
    r = subprocess.run([os.path.join(ROOT, 'tools', 'sanitize_host.sh')], cwd=ROOT, capture_output=True, text=True,
                       timeout=2400, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    out = r.stdout
    assert 'host selftest: all checks passed' in out
    assert 'pool selftest: all checks passed' in out  # ThreadSanitizer run of csrc/thread_pool.h
    assert 'fuzz http: Done' in out and 'fuzz txdecode: Done' in out
    assert 'fuzz jsonspan:' in out and 'no json.loads difference' in out
    assert 'python tests under ASan + UBSan:' in out and 'python tests under TSan:' in out
    assert 'sanitize_host: all stages passed' in out
