"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer runs:
the C oracle driven by tools/sanitize/oracle_checks.c and the C ABI's host code
(mcpx_api.cpp, sanitized on the host side) driven by tools/sanitize/abi_checks.cpp
from 8 threads.  CPU only: GPU sanitizers are unavailable on the pool."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_host_sanitizer_builds(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "run.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "oracle_checks: ok (0 failures)" in r.stdout
    assert "abi_checks: ok (0 failures)" in r.stdout
