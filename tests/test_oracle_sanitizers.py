"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer:
oracle/Makefile's `sanitize` target builds the same C sources with -fsanitize=address,undefined
(-fno-sanitize-recover), and the CPU oracle test files run again in a child Python that has
the ASan runtime preloaded and loads that build. Any report fails the child, hence this test."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

SAN_LIB = os.path.join(ROOT, "oracle", "libkdtn_oracle_san.so")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(600)
def test_oracle_tests_clean_under_asan_ubsan():
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("gcc's libasan runtime is not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    env = dict(os.environ, KDTN_ORACLE_LIB=SAN_LIB, LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    files = ["tests/test_oracle_golden.py", "tests/test_reach_cpu.py", "tests/test_wire_cpu.py",
             "tests/test_ingest_cpu.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *files],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=580)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail
