"""Reference-shaped host types and the batched reconcile driver.

Mirrors the reference's CRD types (api/v1/topology_types.go:28-206) and the call
surface the engine replaces, so callers (and the parity tests) read like the reference:

  TopologyReconciler.calc_diff(old, new)      ↔ controllers/topology_controller.go:288
  TopologyReconciler.reconcile_all(topos)     ↔ Reconcile :61-156 for every dirty Topology
  make_qdiscs(engine, props)                  ↔ common/qdisc.go:20 MakeQdiscs
  KubeDTN.add_links / del_links / update_links↔ daemon/kubedtn/handler.go:592-671 (pure prefix)
  peer_misses + Engine.late_pods              ↔ getPod's API-server fallback, handler.go:27-41

Everything here only packs/unpacks tables; the work happens in libkdtn.so on the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import abi
from .engine import Engine
from .tables import BatchesOut, EpochInput, Interner, Links, StrTab, Topos, Vnis

PROP_FIELDS = abi.PROP_COLS


@dataclass
class LinkProperties:          # api/v1/topology_types.go:119-176
    latency: str = ""
    latency_corr: str = ""
    jitter: str = ""
    loss: str = ""
    loss_corr: str = ""
    rate: str = ""
    gap: int = 0
    duplicate: str = ""
    duplicate_corr: str = ""
    reorder_prob: str = ""
    reorder_corr: str = ""
    corrupt_prob: str = ""
    corrupt_corr: str = ""

    @classmethod
    def from_dict(cls, d: dict | None) -> "LinkProperties":
        d = d or {}
        kw = {f: str(d.get(f, "")) for f in PROP_FIELDS if d.get(f) is not None}
        return cls(gap=int(d.get("gap", 0) or 0), **kw)


@dataclass
class Link:                    # api/v1/topology_types.go:59-95
    local_intf: str = ""
    local_ip: str = ""
    local_mac: str = ""
    peer_intf: str = ""
    peer_ip: str = ""
    peer_mac: str = ""
    peer_pod: str = ""
    uid: int = 0
    properties: LinkProperties = field(default_factory=LinkProperties)

    @classmethod
    def from_dict(cls, d: dict) -> "Link":
        return cls(local_intf=str(d.get("local_intf", "")), local_ip=str(d.get("local_ip", "") or ""),
                   local_mac=str(d.get("local_mac", "") or ""), peer_intf=str(d.get("peer_intf", "")),
                   peer_ip=str(d.get("peer_ip", "") or ""), peer_mac=str(d.get("peer_mac", "") or ""),
                   peer_pod=str(d.get("peer_pod", "")), uid=int(d.get("uid", 0)),
                   properties=LinkProperties.from_dict(d.get("properties")))


@dataclass
class Topology:                # api/v1/topology_types.go:200-206 (Spec.Links, Status.*)
    name: str
    namespace: str = "default"
    spec_links: list[Link] | None = None     # None = nil slice
    status_links: list[Link] | None = None
    src_ip: str = ""
    net_ns: str = ""


def topologies_from_manifest(docs) -> list[Topology]:
    """Topology objects of a parsed K8s manifest (a List or single documents)."""
    out = []
    for doc in docs:
        if not doc:
            continue
        items = doc.get("items", [doc]) if doc.get("kind") == "List" else [doc]
        for it in items:
            if it.get("kind") != "Topology":
                continue
            md = it.get("metadata", {})
            spec = it.get("spec") or {}
            links = spec.get("links")
            status = it.get("status") or {}
            slinks = status.get("links")
            out.append(Topology(
                name=md["name"], namespace=md.get("namespace", "default"),
                spec_links=None if links is None else [Link.from_dict(l) for l in links],
                status_links=None if slinks is None else [Link.from_dict(l) for l in slinks],
                src_ip=status.get("src_ip", "") or "", net_ns=status.get("net_ns", "") or ""))
    return out


def pack(topos: list[Topology], vnis: list[tuple[str, int, str]] = (),
         kdict: Interner | None = None, pdict: Interner | None = None) -> EpochInput:
    """Intern and lay out topologies as the engine's SoA tables (status = realised side)."""
    kd = kdict or Interner()
    pd = pdict or Interner()
    T = len(topos)
    ns = np.zeros(T, np.uint32)
    name = np.zeros(T, np.uint32)
    src = np.zeros(T, np.uint32)
    netns = np.zeros(T, np.uint32)
    flags = np.zeros(T, np.uint8)
    roff = np.zeros(T + 1, np.uint32)
    noff = np.zeros(T + 1, np.uint32)
    sides = ([], [])
    for t, tp in enumerate(topos):
        ns[t], name[t], src[t], netns[t] = kd(tp.namespace), kd(tp.name), kd(tp.src_ip), kd(tp.net_ns)
        flags[t] = (abi.TOPO_STATUS_NIL if tp.status_links is None else 0) | \
                   (abi.TOPO_SPEC_NIL if tp.spec_links is None else 0)
        sides[0].extend(tp.status_links or [])
        sides[1].extend(tp.spec_links or [])
        roff[t + 1] = len(sides[0])
        noff[t + 1] = len(sides[1])

    def links(ls: list[Link]) -> Links:
        L = Links.empty(len(ls))
        for i, l in enumerate(ls):
            for k, col in enumerate(abi.KEY_COLS):
                L.key[k, i] = kd(getattr(l, col))
            L.uid[i] = l.uid
            for k, col in enumerate(PROP_FIELDS):
                L.prop[k, i] = pd(getattr(l.properties, col))
            L.gap[i] = l.properties.gap
        return L

    realised, desired = links(sides[0]), links(sides[1])
    vn = Vnis(np.array([kd(n) for n, _, _ in vnis], np.uint32),
              np.array([v for _, v, _ in vnis], np.int32),
              np.array([kd(s) for _, _, s in vnis], np.uint32))
    return EpochInput(kd.table(), pd.table(), Topos(ns, name, src, netns, flags, roff, noff),
                      realised, desired, vn)


@dataclass
class TopologyBatches:
    """What Reconcile sends for one Topology: action and the three LinksBatchQuery lists."""
    action: int
    add: list[Link]
    delete: list[Link]
    properties_changed: list[Link]
    add_res: np.ndarray
    del_res: np.ndarray
    upd_res: np.ndarray
    add_qdisc: np.ndarray
    upd_qdisc: np.ndarray


class TopologyReconciler:
    """Batched counterpart of controllers/topology_controller.go's TopologyReconciler."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def calc_diff(self, old: list[Link], new: list[Link]):
        """CalcDiff(old, new) → (add, del, propertiesChanged) (topology_controller.go:288-318)."""
        tp = Topology("calc-diff", spec_links=list(new), status_links=list(old))
        b = self.reconcile_all([tp])[0]
        if b.action != abi.ACT_DIFF:   # CalcDiff itself is not gated: equal lists ⇒ nothing changed
            return [], [], []
        return b.add, b.delete, b.properties_changed

    def reconcile_all(self, topos: list[Topology], vnis=(), fetch=None) -> list[TopologyBatches]:
        """fetch(namespace, name) -> Topology | None: the API-server GET getPod falls back to
        when the informer store (`topos`) misses a peer (handler.go:35-39). The misses of the
        first run are fetched, their pod rows passed to kdtn_epoch_late_pods and the epoch run
        again; a key fetch does not know stays KDTN_E_PEER_LOOKUP."""
        kd, pd = Interner(), Interner()
        inp = pack(topos, vnis, kd, pd)
        out = self.engine.reconcile(inp)
        misses = peer_misses(inp, out) if fetch is not None else []
        late = [x for x in (fetch(ns.decode(), name.decode()) for ns, name in misses) if x is not None]
        if late:
            rows = late_pod_rows(late, kd)
            D0 = inp.kdict.n
            if len(kd) > D0:                     # the fetched pods' strings extend the dictionary
                from .delta import build_delta
                grown = EpochInput(kd.table(), inp.pdict, inp.topos, inp.realised, inp.desired, inp.vnis)
                self.engine.upload_delta(build_delta(inp, grown, D0, inp.pdict.n))
            self.engine.late_pods(rows)
            self.engine.run()
            self.engine.sync()
            out = self.engine.download()
        return unpack(topos, out)


def peer_misses(inp: EpochInput, out: BatchesOut) -> list[tuple[bytes, bytes]]:
    """Distinct getPod keys (namespace, or "default" when empty; link.PeerPod) of the AddLinks
    entries whose peer lookup missed (kdtn_resolved.err == KDTN_E_PEER_LOOKUP), in first-entry
    order: what the driver GETs from the API server (handler.go:35-39, :375) before
    kdtn_epoch_late_pods."""
    e = np.nonzero(out.add_res["err"] == abi.E_PEER_LOOKUP)[0]
    if not len(e):
        return []
    t = np.searchsorted(out.add_off.astype(np.int64), e, side="right") - 1
    kb, ko = inp.kdict.bytes_, inp.kdict.offs
    s = lambda i: bytes(kb[ko[i]:ko[i + 1]])
    pcol = abi.KEY_COLS.index("peer_pod")
    keys: dict[tuple[bytes, bytes], None] = {}
    for ei, ti in zip(e, t):
        keys.setdefault((s(inp.topos.ns[ti]) or b"default", s(inp.desired.key[pcol, out.add_idx[ei]])), None)
    return list(keys)


def late_pod_rows(late: list[Topology], kd: Interner) -> np.ndarray:
    """kdtn_pod_row of each fetched Topology (ns, name, status src_ip, net_ns | spec-nil << 31),
    interning its strings into `kd` (append-only)."""
    rows = np.zeros((len(late), 4), np.uint32)
    for i, tp in enumerate(late):
        nil = 0x80000000 if tp.spec_links is None else 0
        rows[i] = (kd(tp.namespace), kd(tp.name), kd(tp.src_ip), kd(tp.net_ns) | nil)
    return rows


def unpack(topos: list[Topology], out: BatchesOut) -> list[TopologyBatches]:
    res = []
    for t, tp in enumerate(topos):
        st, sp = tp.status_links or [], tp.spec_links or []
        r0 = sum(len(x.status_links or []) for x in topos[:t])
        n0 = sum(len(x.spec_links or []) for x in topos[:t])
        d0, d1 = out.del_off[t], out.del_off[t + 1]
        a0, a1 = out.add_off[t], out.add_off[t + 1]
        u0, u1 = out.upd_off[t], out.upd_off[t + 1]
        res.append(TopologyBatches(
            int(out.action[t]),
            [sp[j - n0] for j in out.add_idx[a0:a1]],
            [st[i - r0] for i in out.del_idx[d0:d1]],
            [sp[j - n0] for j in out.upd_idx[u0:u1]],
            out.add_res[a0:a1], out.del_res[d0:d1], out.upd_res[u0:u1],
            out.add_qdisc[a0:a1], out.upd_qdisc[u0:u1]))
    return res


@dataclass
class BatchResult:
    """What a daemon batch handler would return, and the per-link plans behind it:
    `response` False with `first_failed` = the link whose step failed first (the handler
    returns there: handler.go:604-605, 625-626, 650-662), `err` its kdtn_err."""
    response: bool
    first_failed: int
    err: int
    plans: np.ndarray            # kdtn_resolved per link
    qdiscs: np.ndarray | None    # kdtn_qdisc per link (AddLinks / UpdateLinks)


class KubeDTN:
    """Daemon-side counterpart of daemon/kubedtn/handler.go's batch handlers (the pure
    prefix before the first syscall), for one node: the informer's pods plus the node's
    VxlanManager entries."""

    def __init__(self, engine: Engine, pods: list[Topology], vxlan: list[tuple[str, int, str]] = ()):
        self.engine = engine
        self.kd, self.pd = Interner(), Interner()
        self.pods = pods
        self._index = {(p.namespace, p.name): i for i, p in reversed(list(enumerate(pods)))}
        self._vxlan = list(vxlan)

    def _tables(self):
        kd = self.kd
        P = len(self.pods)
        t = Topos(np.array([kd(p.namespace) for p in self.pods], np.uint32),
                  np.array([kd(p.name) for p in self.pods], np.uint32),
                  np.array([kd(p.src_ip) for p in self.pods], np.uint32),
                  np.array([kd(p.net_ns) for p in self.pods], np.uint32),
                  np.array([abi.TOPO_SPEC_NIL if p.spec_links is None else 0 for p in self.pods], np.uint8),
                  np.zeros(P + 1, np.uint32), np.zeros(P + 1, np.uint32))
        v = Vnis(np.array([kd(n) for n, _, _ in self._vxlan], np.uint32),
                 np.array([x for _, x, _ in self._vxlan], np.int32),
                 np.array([kd(s) for _, _, s in self._vxlan], np.uint32))
        return t, v

    def _links(self, links: list[Link]) -> Links:
        L = Links.empty(len(links))
        for i, l in enumerate(links):
            for k, col in enumerate(abi.KEY_COLS):
                L.key[k, i] = self.kd(getattr(l, col))
            L.uid[i] = l.uid
            for k, col in enumerate(PROP_FIELDS):
                L.prop[k, i] = self.pd(getattr(l.properties, col))
            L.gap[i] = l.properties.gap
        return L

    def _batch(self, local_pod: str, kube_ns: str, links: list[Link], kind: int):
        local = self._index[(kube_ns or "default", local_pod)]
        L = self._links(links)
        t, v = self._tables()
        return self.engine.resolve(self.kd.table(), self.pd.table(), t, local, L, kind, v)

    @staticmethod
    def _outcome(plans, errs, qd):
        bad = np.nonzero(errs)[0]
        if len(bad) == 0:
            return BatchResult(True, -1, 0, plans, qd)
        return BatchResult(False, int(bad[0]), int(errs[bad[0]]), plans, qd)

    def add_links(self, local_pod: str, kube_ns: str, links: list[Link]) -> BatchResult:
        """AddLinks (handler.go:592-611): addLink per link, first error aborts."""
        res, q = self._batch(local_pod, kube_ns, links, abi.BATCH_ADD)
        # addLink's qdisc step runs inside SetupVeth / SetupVxLan (same-node, cross-node,
        # physical), i.e. after a successful classification
        qerr = np.where(np.isin(res["kind"], [abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL]),
                        q["err"], 0)
        errs = np.where(res["err"] != 0, res["err"], qerr)
        # a cross-node link whose RemotePod the peer daemon rejects fails after its local
        # steps (UpdateRemote's error, handler.go:448-451)
        errs = np.where(errs != 0, errs, res["remote_err"])
        return self._outcome(res, errs, q)

    def del_links(self, local_pod: str, kube_ns: str, links: list[Link]) -> BatchResult:
        """DelLinks (handler.go:613-632): delLink per link, first error aborts."""
        res, _ = self._batch(local_pod, kube_ns, links, abi.BATCH_DEL)
        return self._outcome(res, res["err"], None)

    def update_links(self, local_pod: str, kube_ns: str, links: list[Link]) -> BatchResult:
        """UpdateLinks (handler.go:634-671): MakeVeth(local) then MakeQdiscs per link."""
        res, q = self._batch(local_pod, kube_ns, links, abi.BATCH_ADD)
        veth = np.isin(res["err"], [abi.E_VETH_CIDR, abi.E_VETH_MAC])
        errs = np.where(veth, res["err"], q["err"])
        return self._outcome(res, errs, q)


def make_qdiscs(engine: Engine, props: list[LinkProperties]) -> np.ndarray:
    """common.MakeQdiscs for a batch of LinkProperties (common/qdisc.go:20-126)."""
    pd = Interner()
    prop = np.zeros((abi.NPROP, len(props)), np.uint32)
    gap = np.zeros(len(props), np.uint32)
    for i, p in enumerate(props):
        for k, f in enumerate(PROP_FIELDS):
            prop[k, i] = pd(getattr(p, f))
        gap[i] = p.gap
    return engine.make_qdiscs(pd.table(), prop, gap)
