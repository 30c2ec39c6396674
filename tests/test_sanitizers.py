"""AddressSanitizer + UndefinedBehaviorSanitizer over the host code that parses
untrusted input (the FASTA/FASTQ(.gz) reader), the 2-bit packer, the host
serials / summary columns, and the CPU oracle (SURVEY §5:
race detection / sanitizers).  Builds tests/san/san_driver (g++ -fsanitize)
and runs it; any sanitizer report fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_host_code_under_asan_ubsan(tmp_path):
    out = tmp_path / "build"
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "san"), f"OUT={out}"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    work = tmp_path / "work"
    work.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", NT_READER_SYNC_CLOSE="1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(out / "san_driver"), str(work)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "san_driver: OK" in r.stdout
