"""Independent encoder for the wire-format checks: the Python protobuf runtime
(google.protobuf, upb) driven by a descriptor that restates proto/v1/kube_dtn.proto:8-53,65-79
(Pod, Link, LinkProperties, LinksBatchQuery, RemotePod; field numbers and types as in the
reference).

`batch_bytes` builds the request Reconcile sends for one list of one Topology
(controllers/topology_controller.go:180-188, 223-231, 266-274): LocalPod is always set, every
Link carries a (possibly empty) Properties message (api/v1/topology_types.go:97-109,178-194).
It returns None where Go's proto.Marshal would fail (a string that is not valid UTF-8).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from kdtn import abi

_F = descriptor_pb2.FieldDescriptorProto
_STR, _I64, _U32, _MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_UINT32, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

_SCHEMA = {
    "Pod": [("name", 1, _STR), ("src_ip", 2, _STR), ("net_ns", 3, _STR), ("kube_ns", 4, _STR),
            ("links", 5, _MSG, ".proto.v1.Link", _REP)],
    "Link": [("peer_pod", 1, _STR), ("local_intf", 2, _STR), ("peer_intf", 3, _STR),
             ("local_ip", 4, _STR), ("peer_ip", 5, _STR), ("uid", 6, _I64),
             ("properties", 7, _MSG, ".proto.v1.LinkProperties"), ("local_mac", 8, _STR),
             ("peer_mac", 9, _STR)],
    "LinkProperties": [("latency", 1, _STR), ("latency_corr", 2, _STR), ("jitter", 3, _STR),
                       ("loss", 4, _STR), ("loss_corr", 5, _STR), ("rate", 6, _STR),
                       ("gap", 7, _U32), ("duplicate", 8, _STR), ("duplicate_corr", 9, _STR),
                       ("reorder_prob", 10, _STR), ("reorder_corr", 11, _STR),
                       ("corrupt_prob", 12, _STR), ("corrupt_corr", 13, _STR)],
    "LinksBatchQuery": [("local_pod", 1, _MSG, ".proto.v1.Pod"),
                        ("links", 2, _MSG, ".proto.v1.Link", _REP)],
    "RemotePod": [("net_ns", 1, _STR), ("intf_name", 2, _STR), ("intf_ip", 3, _STR),
                  ("peer_vtep", 4, _STR), ("kube_ns", 5, _STR), ("vni", 6, _F.TYPE_INT32),
                  ("properties", 7, _MSG, ".proto.v1.LinkProperties"), ("name", 8, _STR)],
}


def _classes():
    fdp = descriptor_pb2.FileDescriptorProto(name="kdtn_test_kube_dtn.proto", package="proto.v1",
                                             syntax="proto3")
    for name, fields in _SCHEMA.items():
        m = fdp.message_type.add(name=name)
        for f in fields:
            fd = m.field.add(name=f[0], number=f[1], type=f[2],
                             label=f[4] if len(f) > 4 else _OPT)
            if f[2] == _MSG:
                fd.type_name = f[3]
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"proto.v1.{n}"))
            for n in _SCHEMA}


_C = _classes()


def _s(tab, i: int) -> str:
    return tab.get(int(i)).decode("utf-8")          # raises on invalid UTF-8


def batch_bytes(inp, t: int, lst: int, idx) -> bytes | None:
    """Serialized LinksBatchQuery of topology t, list lst (0 del, 1 add, 2 upd) over the
    record indices idx; b"" when idx is empty (no RPC); None on a Marshal error."""
    if len(idx) == 0:
        return b""
    kd, pd, T = inp.kdict, inp.pdict, inp.topos
    L = inp.realised if lst == 0 else inp.desired
    try:
        q = _C["LinksBatchQuery"]()
        pod = q.local_pod
        pod.SetInParent()
        pod.name, pod.src_ip = _s(kd, T.name[t]), _s(kd, T.src_ip[t])
        pod.net_ns, pod.kube_ns = _s(kd, T.net_ns[t]), _s(kd, T.ns[t])
        for j in idx:
            j = int(j)
            l = q.links.add()
            for k, col in enumerate(abi.KEY_COLS):
                setattr(l, col, _s(kd, L.key[k, j]))
            l.uid = int(L.uid[j])
            p = l.properties
            p.SetInParent()
            for k, col in enumerate(abi.PROP_COLS):
                setattr(p, col, _s(pd, L.prop[k, j]))
            p.gap = int(L.gap[j])
        return q.SerializeToString()
    except (UnicodeDecodeError, ValueError):
        return None


def epoch_bytes(inp, out):
    """{(lst, t): bytes | None} for every batch of an epoch's outputs (kdtn_batches order)."""
    res = {}
    offs = (out.del_off, out.add_off, out.upd_off)
    idxs = (out.del_idx, out.add_idx, out.upd_idx)
    for lst in range(3):
        for t in range(inp.topos.n):
            e0, e1 = int(offs[lst][t]), int(offs[lst][t + 1])
            res[(lst, t)] = batch_bytes(inp, t, lst, idxs[lst][e0:e1])
    return res


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def remote_pod_bytes(inp, out, e: int, t: int, physical: bool, peer_netns) -> bytes | None:
    """Length-delimited RemotePod of add entry e (topology t): UpdateRemote's payload
    (common/utils.go:42-51) or, for a physical peer, the local Update's
    (daemon/kubedtn/handler.go:353-362); None on a Marshal error (invalid UTF-8)."""
    kd, pd, T, L = inp.kdict, inp.pdict, inp.topos, inp.desired
    j = int(out.add_idx[e])
    r = out.add_res[e]
    key = lambda c: kd.get(int(L.key[abi.KEY_COLS.index(c), j]))
    try:
        m = _C["RemotePod"]()
        if physical:
            m.net_ns = _s(kd, T.net_ns[t])
            m.intf_name, m.intf_ip = key("local_intf").decode(), key("local_ip").decode()
            m.peer_vtep = key("peer_pod")[len(b"physical/"):].decode()
        else:
            m.net_ns = _s(kd, peer_netns[int(r["peer_topo"])])
            m.intf_name, m.intf_ip = key("peer_intf").decode(), key("peer_ip").decode()
            m.peer_vtep = _s(kd, T.src_ip[t])
        m.kube_ns = _s(kd, T.ns[t])
        m.vni = int(r["vni"])
        p = m.properties
        p.SetInParent()
        for k, col in enumerate(abi.PROP_COLS):
            setattr(p, col, _s(pd, L.prop[k, j]))
        p.gap = int(L.gap[j])
        m.name = key("peer_pod").decode()
        b = m.SerializeToString()
        return _varint(len(b)) + b
    except (UnicodeDecodeError, ValueError):
        return None
