"""Host code under sanitizers (SURVEY.md §5 build counterpart), CPU only:
the OccEpoch shim's epoch map with four worker threads (against a stub
engine), the .dccb reader / writer with every truncation and a sweep of
corruptions, and the oracle restatements — built with ASan+UBSan and with
TSan (tests/san/Makefile) and run; any report fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "san")


def _build():
    if not os.path.exists(os.path.join(SAN, "Makefile")):
        pytest.skip("tests/san not present (not shipped to GPU boxes)")
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    p = subprocess.run(["make", "-C", SAN], capture_output=True, text=True, timeout=600)
    if p.returncode != 0 and "cannot find -l" in p.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert p.returncode == 0, p.stderr[-3000:]


@pytest.mark.parametrize("variant", ["san_asan", "san_tsan"])
def test_host_code_clean_under_sanitizer(variant, tmp_path):
    _build()
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "exitcode=66 halt_on_error=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    for _ in range(3 if variant == "san_tsan" else 1):  # TSan sees interleavings, not all
        p = subprocess.run([os.path.join(SAN, "out", variant), str(tmp_path)], capture_output=True,
                           text=True, timeout=300, env=env)
        assert p.returncode == 0 and "harness clean" in p.stdout, (p.stdout + p.stderr)[-4000:]
