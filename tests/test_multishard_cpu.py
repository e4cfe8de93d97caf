"""Multi-shard path on CPU (world size 2, gloo): each rank owns a contiguous block of
topologies, fills its pod-status rows exactly as k_pods_fill does, all-gathers them (the
collective the engine runs over RCCL), and reconciles its shard against the global table.
The concatenated per-topology results must equal the unsharded epoch's, bit for bit.
The reconcile here is the oracle (this test covers the sharding logic and the exchange;
tests/test_parity_gpu.py pins the engine to the oracle)."""
import hashlib
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from kdtn import synth

PODS = 3000
WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pod_rows(inp):
    """k_pods_fill: {ns, name, src_ip, net_ns | spec_nil<<31} per local pod (pod_slice rows)."""
    t = inp.topos
    rows = np.zeros((inp.pod_slice, 4), np.uint32)
    rows[:, :2] = 0xFFFFFFFF                 # padding rows are never inserted
    rows[:t.n, 0], rows[:t.n, 1], rows[:t.n, 2] = t.ns, t.name, t.src_ip
    rows[:t.n, 3] = t.net_ns | np.where(t.flags & 2, 0x80000000, 0).astype(np.uint32)
    return rows


def global_pods(rows: np.ndarray) -> dict:
    keep = rows[:, 0] != 0xFFFFFFFF
    r = rows[keep]
    return {"ns": r[:, 0], "name": r[:, 1], "src_ip": r[:, 2], "net_ns": r[:, 3] & 0x7FFFFFFF,
            "flags": np.where(r[:, 3] & 0x80000000, 2, 0).astype(np.uint8), "base": 0}


def _kstr(inp, i: int) -> bytes:
    o = inp.kdict.offs
    return inp.kdict.bytes_[o[i]:o[i + 1]].tobytes()


def per_topology(inp, out) -> np.ndarray:
    """SHA-1 per topology of its outputs, indices made topology-relative. Per-link strings
    have shard-local ids, so the one id that is such a string (the vtep of a PHYSICAL link:
    the peer_pod string) is hashed as text."""
    t = inp.topos
    add_res = out.add_res.copy()
    phys = np.nonzero(add_res["kind"] == 2)[0]
    ptxt = {int(e): _kstr(inp, int(add_res["vtep"][e])) for e in phys}
    add_res["vtep"][phys] = 0
    res = np.zeros((t.n, 20), np.uint8)
    for k in range(t.n):
        a0, a1 = out.add_off[k], out.add_off[k + 1]
        d0, d1 = out.del_off[k], out.del_off[k + 1]
        u0, u1 = out.upd_off[k], out.upd_off[k + 1]
        h = hashlib.sha1(bytes([int(out.action[k])]))
        for e in range(a0, a1):
            if e in ptxt:
                h.update(ptxt[e])
        for part in ((out.add_idx[a0:a1] - t.des_off[k]), add_res[a0:a1], out.add_qdisc[a0:a1],
                     (out.del_idx[d0:d1] - t.real_off[k]), out.del_res[d0:d1],
                     (out.upd_idx[u0:u1] - t.des_off[k]), out.upd_res[u0:u1], out.upd_qdisc[u0:u1]):
            h.update(np.ascontiguousarray(part).tobytes())
            h.update(b"|")
        res[k] = np.frombuffer(h.digest(), np.uint8)
    return res


def _rank(rank: int, port: int, config: int, outdir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    inp = synth.make(config, pods_per_shard=PODS, shard=rank, nshards=WORLD)
    mine = torch.from_numpy(pod_rows(inp).view(np.int32).copy())
    parts = [torch.empty_like(mine) for _ in range(WORLD)]
    dist.all_gather(parts, mine)                        # the engine's ncclAllGather
    rows = torch.cat(parts).numpy().view(np.uint32)
    out = O.reconcile(inp, pods=global_pods(rows))
    # the engine reports peers as global pod indices: rank * pod_slice + local index
    np.save(os.path.join(outdir, f"peers{rank}.npy"), out.add_res["peer_topo"].copy())
    np.save(os.path.join(outdir, f"r{rank}.npy"), per_topology(inp, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", [2, 3, 4])
def test_two_shards_equal_unsharded(config):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(_free_port(), config, d), nprocs=WORLD, join=True,
                           start_method="fork")
        sharded = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(WORLD)])
        peers = np.concatenate([np.load(os.path.join(d, f"peers{r}.npy")) for r in range(WORLD)])
    full = synth.make(config, pods_per_shard=PODS * WORLD)
    ref = O.reconcile(full)
    want = per_topology(full, ref)
    assert len(sharded) == len(want)
    bad = np.nonzero((sharded != want).any(axis=1))[0].tolist()
    assert not bad, f"{len(bad)} topologies differ, first {bad[:5]}"
    assert np.array_equal(peers, ref.add_res["peer_topo"])
    # the exchange matters: some peers live on the other shard
    assert ((ref.add_res["peer_topo"] >= PODS) & (ref.add_res["peer_topo"] != 0xFFFFFFFF)).any()
