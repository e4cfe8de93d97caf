"""bench.py's multi-rank path as the driver invokes it: `python bench.py --gpus N` with no
launcher spawns its N ranks itself (torch.distributed.run as a child process). On the one-GPU
test box the two ranks share the device, so RCCL cannot hold them and every rank takes the
host transport together (gloo all-gather of the pod-status rows inside each timed epoch).
The line must report n_gpus = comm_ranks = 2, and the ranks' dumped outputs must equal the
unsharded oracle epoch per topology (peers as global pod ids)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from multishard import gid_table, per_topology, unsharded_by_gid

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PODS = 20000


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]          # rank 0 prints exactly one line
    return json.loads(lines[0])


def test_bench_gpus2_spawns_two_ranks_with_parity():
    import oracle as O
    from kdtn import synth
    with tempfile.TemporaryDirectory() as d:
        line = _bench("--gpus", "2", "--pods", str(PODS), "--steps", "3", "--warmup", "1",
                      "--no-cpu-baseline", "--no-wire", "--no-ingest", "--no-e2e", "--dump", d)
        ranks = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(2)]
    assert line["n_gpus"] == 2 and line["config"]["comm_ranks"] == 2
    assert line["config"]["launcher"].startswith("bench.py --gpus")
    assert line["config"]["exchange"].startswith("host transport")
    assert line["config"]["links_per_epoch"] == 10 * PODS and line["value"] > 0
    from kdtn.tables import BatchesOut
    gids = [r["gid"] for r in ranks]
    peer_gid = gid_table(int(ranks[0]["pod_slice"]), gids)
    got = []
    for r, z in enumerate(ranks):
        inp = synth.make(2, total_pods=PODS, shard=r, nshards=2)
        assert np.array_equal(inp.gid, z["gid"])
        out = BatchesOut(*[z[f] for f in BatchesOut.FIELDS])
        got.append(per_topology(inp, out, peer_gid))
    full = synth.make(2, pods_per_shard=PODS)
    want = unsharded_by_gid(per_topology(full, O.reconcile(full, tick=synth_tick())), gids)
    got = np.concatenate(got)
    assert len(got) == full.topos.n
    bad = np.nonzero((got != want).any(axis=1))[0].tolist()
    assert not bad, f"{len(bad)} topologies differ from the unsharded oracle, first {bad[:5]}"


def synth_tick() -> float:
    """bench.py builds its Engine with the host's psched tick (kdtn_psched_tick_in_usec)."""
    from kdtn import lib
    return float(lib().kdtn_psched_tick_in_usec())


def test_bench_gpus1_line_unchanged():
    line = _bench("--gpus", "1", "--pods", str(PODS), "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline", "--no-wire", "--no-ingest", "--no-e2e")
    assert line["n_gpus"] == 1 and line["config"]["comm_ranks"] == 1
    assert line["config"]["exchange"] == "none" and line["config"]["launcher"] == "none"
    assert line["roofline"]["kernel"] == "k_reconcile" and 0 < line["roofline"]["frac"] < 1


def test_bench_config1_line():
    line = _bench("--config", "1", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert line["n_gpus"] == 1 and line["config"]["config"] == 1
    assert line["counts_per_epoch_rank0"] == {"add": 0.0, "upd": 100000.0, "del": 0.0}
