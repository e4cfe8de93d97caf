"""The C++ host layer (kube-dtn_amd/host/kubedtn.hpp: TopologyReconciler::CalcDiff /
Reconcile, MakeQdiscs, the daemon batch semantics) through its own test binary
(tests/cpp/test_kubedtn.cpp, built by `make -C kube-dtn_amd`)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "kube-dtn_amd", "bin", "test_kubedtn")


def _run(timeout=120):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built; run `make -C kube-dtn_amd`")
    return subprocess.run([BIN], capture_output=True, text=True, timeout=timeout)


def test_host_binary_refuses_without_gpu():
    """Without a gfx950 device the engine refuses to start (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = _run()
    assert r.returncode == 2 and "kdtn_init" in r.stderr, (r.stdout, r.stderr)


@pytest.mark.gpu
def test_host_cpp_suite():
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    for t in ("TestReconcileSamples", "TestCalcDiffDuplicates", "TestMakeQdiscs", "TestAddLinksBatchAbort"):
        assert f"PASS {t}" in r.stdout, r.stdout + r.stderr
