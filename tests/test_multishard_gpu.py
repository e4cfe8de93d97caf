"""Engine shards on one GPU (world size 2 and 3, gloo as the host transport): each process
runs libkdtn.so on its hash shard (kdtn_topology_shard) — kdtn_comm_set_ranks, upload,
kdtn_pods_export, gloo all-gather of the pod-status rows, kdtn_pods_import, epoch — which is
the RCCL path's data flow with the collective done by the caller. Per topology, the
concatenated shard outputs equal the unsharded oracle epoch bit for bit (peers compared as
global pod ids), and the RemotePod fan-out of the shards together equals the unsharded one."""
import os
import tempfile

import numpy as np
import pytest

from multishard import free_port, gid_table, per_topology, unsharded_by_gid

pytestmark = pytest.mark.gpu
PODS = 20000


def _rank(rank: int, world: int, port: int, config: int, outdir: str):
    import torch
    import torch.distributed as dist
    from kdtn import Engine, KdtnError, abi, synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp = synth.make(config, total_pods=PODS, shard=rank, nshards=world)
    eng = Engine(device=0, tick_in_usec=15.625)
    eng.set_ranks(world, rank)
    eng.upload(inp)
    try:                                                   # the import is required
        eng.run()
        raise AssertionError("kdtn_epoch_run without kdtn_pods_import must fail")
    except KdtnError as e:
        assert e.code == abi.EINVAL
    mine = torch.from_numpy(eng.pods_export(inp.pod_slice).view(np.int32).copy())
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    eng.pods_import(torch.cat(parts).numpy().view(np.uint32))
    eng.run()
    eng.sync()
    out = eng.download()
    gids = [None] * world
    dist.all_gather_object(gids, inp.gid)
    peer_gid = gid_table(inp.pod_slice, gids)
    np.save(os.path.join(outdir, f"r{rank}.npy"), per_topology(inp, out, peer_gid))
    np.save(os.path.join(outdir, f"g{rank}.npy"), inp.gid)
    node, off, idx = eng.fanout()
    sends = np.zeros(len(idx), np.int64)
    for k in range(len(node)):
        sends[off[k]:off[k + 1]] = node[k]
    # (global pod id of the sender, its add-entry rank within the topology, destination node)
    t_of = np.searchsorted(out.add_off, idx, side="right") - 1
    np.save(os.path.join(outdir, f"f{rank}.npy"),
            np.stack([inp.gid[t_of], idx - out.add_off[t_of], sends]).T if len(idx) else np.zeros((0, 3), np.int64))
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _fan_rows(inp, out, node, off, idx, gid):
    sends = np.zeros(len(idx), np.int64)
    for k in range(len(node)):
        sends[off[k]:off[k + 1]] = node[k]
    t_of = np.searchsorted(out.add_off, idx, side="right") - 1
    return np.stack([gid[t_of], idx - out.add_off[t_of], sends]).T


@pytest.mark.parametrize("config,world", [(2, 2), (3, 2), (4, 2), (2, 3)])
def test_engine_shards_equal_unsharded_oracle(config, world):
    import torch.multiprocessing as mp
    import oracle as O
    from kdtn import synth
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(world, free_port(), config, d), nprocs=world, join=True,
                           start_method="spawn")
        sharded = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
        gids = [np.load(os.path.join(d, f"g{r}.npy")) for r in range(world)]
        fan = np.concatenate([np.load(os.path.join(d, f"f{r}.npy")) for r in range(world)])
    full = synth.make(config, pods_per_shard=PODS)
    ref = O.reconcile(full, tick=15.625)
    want = unsharded_by_gid(per_topology(full, ref), gids)
    assert len(sharded) == len(want) == full.topos.n
    bad = np.nonzero((sharded != want).any(axis=1))[0].tolist()
    assert not bad, f"{len(bad)} topologies differ, first {bad[:5]}"
    # cross-shard peers exist (the exchange matters)
    g = np.concatenate(gids)
    owner = np.zeros(full.topos.n, np.int64)
    for r, gr in enumerate(gids):
        owner[gr] = r
    p = ref.add_res["peer_topo"]
    t_of = np.searchsorted(ref.add_off, np.arange(len(p)), side="right") - 1
    hit = p != 0xFFFFFFFF
    assert (owner[p[hit]] != owner[t_of[hit]]).any() and len(g) == full.topos.n
    # RemotePod fan-out: the shards' sends together are the unsharded sends
    wn, wo, wi = O.fanout(ref, full.topos.n)
    want_fan = _fan_rows(full, ref, wn, wo, wi, np.arange(full.topos.n))
    key = lambda a: a[np.lexsort(a.T[::-1])]
    assert np.array_equal(key(fan), key(want_fan))


def test_rccl_one_rank_communicator_equals_local_epoch():
    """The production transport on one GPU: kdtn_comm_init with a one-rank RCCL communicator
    makes kdtn_epoch_run all-gather the pod-status rows with ncclAllGather on the comm
    stream (in place, slice = every pod). The epoch equals the oracle's bit for bit."""
    import oracle as O
    from kdtn import Engine, comm_unique_id, synth
    inp = synth.make(4, total_pods=5000)
    want = O.reconcile(inp, tick=15.625)
    with Engine(device=0, tick_in_usec=15.625) as eng:
        eng.comm_init(comm_unique_id(), 1, 0)
        eng.upload(inp)
        for _ in range(2):                       # the second epoch reuses the communicator
            eng.run()
            eng.sync()
            got = eng.download()
            assert "pods_allgather" in eng.kernel_times()
            bad = got.mismatches(want)
            assert not bad, f"RCCL one-rank epoch differs from the oracle in {bad}"


def _vni_rank(rank: int, world: int, port: int, config: int, outdir: str):
    import torch.distributed as dist
    from kdtn import Engine, synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp = synth.make(config, total_pods=PODS, shard=rank, nshards=world)
    eng = Engine(device=0, tick_in_usec=15.625)
    eng.set_ranks(world, rank)
    eng.upload(inp)
    mine = eng.pods_export(inp.pod_slice)
    rows = [None] * world
    dist.all_gather_object(rows, mine)
    table = np.concatenate(rows)
    eng.pods_import(table)
    eng.run()
    eng.sync()
    out = eng.download()
    dels, adds = eng.vni_ops_export()
    got = [None] * world
    dist.all_gather_object(got, (dels, adds))
    eng.vni_ops_import(np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]))
    vm = eng.vni_apply()
    np.savez(os.path.join(outdir, f"v{rank}.npz"), node=vm.node, vni=vm.vni, net_ns=vm.net_ns, table=table,
             t_src=inp.topos.src_ip, t_netns=inp.topos.net_ns, snap_node=inp.vnis.node, snap_vni=inp.vnis.vni,
             snap_netns=inp.vnis.net_ns, **{f: getattr(out, f) for f in out.FIELDS})
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config,world", [(4, 2), (3, 3)])
def test_sharded_vni_apply_equals_rank_order_oracle(config, world):
    """kdtn_epoch_vni_apply on engine shards (host transport): every rank exports its VXLAN
    ops, imports everyone's in rank order, and applies them against the replicated snapshot.
    All ranks leave the same map, equal to the oracle's apply of the ranks' batches
    concatenated in rank order (the sharded order: rank r's ops before rank r+1's)."""
    import types
    import torch.multiprocessing as mp
    import oracle as O
    from kdtn.tables import BatchesOut, Topos, Vnis
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_vni_rank, args=(world, free_port(), config, d), nprocs=world, join=True,
                           start_method="spawn")
        z = [dict(np.load(os.path.join(d, f"v{r}.npz"))) for r in range(world)]
    for r in range(1, world):                                   # one node-global map
        for f in ("node", "vni", "net_ns", "snap_node", "snap_vni", "snap_netns"):
            assert np.array_equal(z[r][f], z[0][f]), (r, f)
    # the ranks' batches as one rank-ordered epoch
    cat = {}
    for f in ("action", "del_idx", "add_idx", "upd_idx", "del_res", "add_res", "upd_res", "add_qdisc", "upd_qdisc"):
        cat[f] = np.concatenate([x[f] for x in z])
    for f in ("del_off", "add_off", "upd_off"):
        parts, base = [], 0
        for x in z:
            parts.append(x[f][:-1].astype(np.int64) + base)
            base += int(x[f][-1])
        cat[f] = np.concatenate(parts + [np.array([base])]).astype(np.uint32)
    out = BatchesOut(*[cat[f] for f in BatchesOut.FIELDS])
    T = len(cat["action"])
    t_src = np.concatenate([x["t_src"] for x in z])
    t_netns = np.concatenate([x["t_netns"] for x in z])
    fake = types.SimpleNamespace(topos=types.SimpleNamespace(n=T, src_ip=t_src, net_ns=t_netns),
                                 vnis=Vnis(z[0]["snap_node"], z[0]["snap_vni"], z[0]["snap_netns"]))
    want = O.vni_apply(fake, out, pod_netns=z[0]["table"][:, 3] & 0x7FFFFFFF)
    assert np.array_equal(z[0]["node"], want[0]) and np.array_equal(z[0]["vni"], want[1])
    assert np.array_equal(z[0]["net_ns"], want[2])
    assert len(want[0]) > 100
