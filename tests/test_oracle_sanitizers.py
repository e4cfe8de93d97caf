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


_TSAN_CHILD = r"""
import sys
sys.path[:0] = [{pkg!r}, {orc!r}, {tst!r}]
import numpy as np
import oracle as O
from helpers import random_epoch
from kdtn import synth
from kdtn.model import pack
for seed in range(3):
    topos, vnis = random_epoch(seed, T=300, p_err=0.2)
    inp = pack(topos, vnis)
    a, b = O.reconcile(inp), O.reconcile_parallel(inp, threads=6)
    assert not a.mismatches(b), seed
inp = synth.make(2, total_pods=20000)
from concurrent.futures import ThreadPoolExecutor
bounds = [inp.topos.n * k // 8 for k in range(9)]
with ThreadPoolExecutor(8) as ex:          # bench.py cpu_baseline's pattern
    list(ex.map(lambda k: O.reconcile(inp, t_begin=bounds[k], t_end=bounds[k + 1], timing=[]), range(8)))
assert not O.reconcile(inp).mismatches(O.reconcile_parallel(inp, threads=8))
print("tsan child ok")
"""


@pytest.mark.timeout(600)
def test_oracle_threaded_paths_clean_under_tsan():
    """The oracle's threaded uses — reconcile_parallel (full-size GPU parity) and the CPU
    baseline's worker pool — under ThreadSanitizer: concurrent or_reconcile_epoch calls on
    shared input tables must not race."""
    tsan = _runtime("libtsan.so")
    if tsan is None:
        pytest.skip("gcc's libtsan runtime is not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "tsan"], check=True)
    env = dict(os.environ, KDTN_ORACLE_LIB=os.path.join(ROOT, "oracle", "libkdtn_oracle_tsan.so"),
               LD_PRELOAD=tsan, TSAN_OPTIONS="exitcode=88:halt_on_error=1:report_signal_unsafe=0")
    code = _TSAN_CHILD.format(pkg=os.path.join(ROOT, "kube-dtn_amd"), orc=os.path.join(ROOT, "oracle"),
                              tst=os.path.join(ROOT, "tests"))
    r = subprocess.run(["setarch", "-R", sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=580)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0 and "tsan child ok" in r.stdout, tail
    assert "ThreadSanitizer" not in tail, tail
