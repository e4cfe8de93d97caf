"""Multi-shard algebra on CPU (world size 2 and 3, gloo), with the oracle as the per-shard
reconcile: topologies are hash-sharded (kdtn_topology_shard), each rank fills its
pod-status rows exactly as k_pods_fill does, all-gathers them (the engine's one exchange),
and reconciles its shard against the gathered table. Per topology the results equal the
unsharded epoch's bit for bit (peers compared as global pod ids). The engine itself runs
the same protocol in tests/test_multishard_gpu.py (two engine shards on one GPU)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from kdtn import synth, topology_shard
from multishard import compact_pods, free_port, gid_table, per_topology, pod_rows, unsharded_by_gid

PODS = 3000


def _rank(rank: int, world: int, port: int, config: int, outdir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp = synth.make(config, total_pods=PODS, shard=rank, nshards=world)
    mine = torch.from_numpy(pod_rows(inp).view(np.int32).copy())
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)                        # the engine's ncclAllGather
    rows = torch.cat(parts).numpy().view(np.uint32)
    gids = [None] * world
    dist.all_gather_object(gids, inp.gid)
    pods, engine_index = compact_pods(rows)
    out = O.reconcile(inp, pods=pods)
    # the oracle reports peers as compact indices; map them to global pod ids
    peer_gid = gid_table(inp.pod_slice, gids)[engine_index]
    np.save(os.path.join(outdir, f"r{rank}.npy"), per_topology(inp, out, peer_gid))
    np.save(os.path.join(outdir, f"g{rank}.npy"), inp.gid)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config,world", [(2, 2), (3, 2), (4, 2), (2, 3)])
def test_hash_shards_equal_unsharded(config, world):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(world, free_port(), config, d), nprocs=world, join=True,
                           start_method="fork")
        sharded = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
        gids = [np.load(os.path.join(d, f"g{r}.npy")) for r in range(world)]
    full = synth.make(config, pods_per_shard=PODS)
    ref = O.reconcile(full)
    want = unsharded_by_gid(per_topology(full, ref), gids)
    assert len(sharded) == len(want) == full.topos.n
    bad = np.nonzero((sharded != want).any(axis=1))[0].tolist()
    assert not bad, f"{len(bad)} topologies differ, first {bad[:5]}"


def test_shard_function_is_the_engines():
    """Every synthetic shard holds exactly the topologies kdtn_topology_shard assigns it."""
    for r in range(3):
        inp = synth.make(4, total_pods=900, shard=r, nshards=3)
        for t in range(inp.topos.n):
            ns, nm = inp.kdict.get(int(inp.topos.ns[t])), inp.kdict.get(int(inp.topos.name[t]))
            assert topology_shard(ns, nm, 3) == r
    assert topology_shard(b"default", b"p1", 1) == 0
