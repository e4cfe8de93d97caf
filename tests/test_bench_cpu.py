"""CPU: bench.py's launcher contract, checked before anything touches a GPU.

`--gpus N` under an external launcher must match WORLD_SIZE (one process per GPU); a
mismatch exits with status 2 instead of timing the wrong number of ranks. The self-spawn
path (no WORLD_SIZE) is exercised on the GPU box (tests/test_bench_gpu.py)."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2, p.stderr[-2000:]
    assert "one process per GPU" in p.stderr


def test_config1_is_single_gpu():
    p = _run(["--gpus", "2", "--config", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "one-GPU workload" in p.stderr
