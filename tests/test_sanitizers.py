"""Host code under sanitizers ("Race detection /
sanitizers"): tools/sanitize builds the host half of liblincheck (EDN reader
and writer, lc_pack, lc_report, the synthetic generator) and the C oracle
with AddressSanitizer + UndefinedBehaviorSanitizer, and again with
ThreadSanitizer (the parallel EDN split and the worker threads of lc_pack,
lc_synth and the oracle), and drives them over generated histories,
history.edn round trips, mangled EDN text and malformed op sequences.  CPU
only: no GPU code is involved."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")

pytestmark = pytest.mark.skipif(not shutil.which("/opt/rocm/llvm/bin/clang++"), reason="no ROCm clang++")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_under_sanitizer(kind):
    r = subprocess.run(["make", "-C", SAN, kind], capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 failed checks" in out
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error" not in out  # UBSan
