"""Shared helpers of the multi-shard tests (tests/test_multishard_cpu.py, _gpu.py).

Topologies are sharded as the engine shards them: kdtn_topology_shard(namespace, name, G) =
hash64(namespace/name) mod G; rank r's topologies take the global pod
indices [r*pod_slice, r*pod_slice + T_r). Outputs are compared per topology against the
unsharded epoch after mapping peer indices back to global pod ids."""
import hashlib
import socket

import numpy as np

NONE = 0xFFFFFFFF


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pod_rows(inp) -> np.ndarray:
    """k_pods_fill: {ns, name, src_ip, net_ns | spec_nil<<31} per local pod (pod_slice rows,
    padding rows ns = name = ~0)."""
    t = inp.topos
    rows = np.zeros((inp.pod_slice, 4), np.uint32)
    rows[:, :2] = NONE
    rows[:t.n, 0], rows[:t.n, 1], rows[:t.n, 2] = t.ns, t.name, t.src_ip
    rows[:t.n, 3] = t.net_ns | np.where(t.flags & 2, 0x80000000, 0).astype(np.uint32)
    return rows


def compact_pods(rows: np.ndarray):
    """Oracle pod table from the gathered rows (padding dropped) and, per compact index, the
    engine's global pod index."""
    keep = np.nonzero(rows[:, 0] != NONE)[0]
    r = rows[keep]
    pods = {"ns": r[:, 0], "name": r[:, 1], "src_ip": r[:, 2], "net_ns": r[:, 3] & 0x7FFFFFFF,
            "flags": np.where(r[:, 3] & 0x80000000, 2, 0).astype(np.uint8), "base": 0}
    return pods, keep.astype(np.uint32)


def gid_table(slice_: int, gids: list) -> np.ndarray:
    """Engine global pod index → global pod id (rank r's t-th topology is r*slice + t)."""
    g = np.full(slice_ * len(gids), NONE, np.int64)
    for r, gr in enumerate(gids):
        g[r * slice_: r * slice_ + len(gr)] = gr
    return g


def _kstr(inp, i: int) -> bytes:
    o = inp.kdict.offs
    return inp.kdict.bytes_[o[i]:o[i + 1]].tobytes()


def per_topology(inp, out, peer_gid=None) -> np.ndarray:
    """SHA-1 per topology of its outputs, indices made topology-relative, peers as global pod
    ids (peer_gid maps the output's peer index; None = already global ids). Per-link strings
    have shard-local ids, so the one such id in the outputs (the vtep of a PHYSICAL link: the
    peer_pod string) is hashed as text."""
    t = inp.topos
    add_res = out.add_res.copy()
    if peer_gid is not None:
        p = add_res["peer_topo"]
        hit = p != NONE
        add_res["peer_topo"][hit] = peer_gid[p[hit]].astype(np.uint32)
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


def unsharded_by_gid(want: np.ndarray, gids: list) -> np.ndarray:
    """The unsharded per-topology hashes in the sharded outputs' order (rank, then local)."""
    return np.concatenate([want[g] for g in gids])
