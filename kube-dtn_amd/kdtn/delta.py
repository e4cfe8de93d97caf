"""Delta uploads against the engine's resident state (kdtn_epoch_upload_delta).

A controller that keeps the engine's link stores resident across reconciles sends, per
epoch, only the Topologies whose spec (or status.src_ip / status.net_ns) changed, each new
spec.links list as references into the previous desired store plus the records that are
new. `build_delta` derives that from two consecutive epochs' tables, the way the informer
cache would (the previous and the current object of every changed Topology): per Topology
positional record equality decides "changed"; inside a changed Topology each new record is
matched to an identical previous record by a 64-bit content hash, verified column by
column, else sent inline.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi
from .tables import EpochInput, Links, StrTab, Vnis

_M1, _M2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9)


def record_hash(L: Links) -> np.ndarray:
    """64-bit content hash of every record (7 keys, 12 props, gap, uid)."""
    h = np.full(L.n, 0x243F6A8885A308D3, np.uint64)
    with np.errstate(over="ignore"):
        cols = [L.key[k] for k in range(abi.NKEY)] + [L.prop[k] for k in range(abi.NPROP)] + [L.gap]
        for c in cols:
            h = (h ^ c.astype(np.uint64)) * _M1
            h ^= h >> np.uint64(29)
        u = L.uid.view(np.uint64)
        h = (h ^ u) * _M2
        h ^= h >> np.uint64(32)
    return h


def _seg(off: np.ndarray) -> np.ndarray:
    off = off.astype(np.int64)
    return np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))


def _same_records(a: Links, ia: np.ndarray, b: Links, ib: np.ndarray) -> np.ndarray:
    eq = a.uid[ia] == b.uid[ib]
    eq &= a.gap[ia] == b.gap[ib]
    eq &= (a.key[:, ia] == b.key[:, ib]).all(axis=0)
    eq &= (a.prop[:, ia] == b.prop[:, ib]).all(axis=0)
    return eq


@dataclass
class Delta:
    kdict: StrTab
    pdict: StrTab
    kdict_keep: int
    pdict_keep: int
    topo: np.ndarray        # u32 [n_changed] (indices of the new topology table)
    src_ip: np.ndarray      # u32
    net_ns: np.ndarray      # u32
    spec_nil: np.ndarray    # u8
    des_off: np.ndarray     # u32 [n_changed + 1]
    ref: np.ndarray         # u32
    records: Links
    vnis: Vnis
    prev: np.ndarray | None = None    # u32 [n_topos]: previous index | DELTA_NEW; None = same set
    ns: np.ndarray | None = None      # u32 [n_changed] metadata.namespace (created topologies)
    name: np.ndarray | None = None    # u32 [n_changed] metadata.name
    pod_slice: int = 0

    @property
    def n_changed(self) -> int:
        return int(self.topo.shape[0])

    @property
    def n_topos(self) -> int | None:
        return None if self.prev is None else int(self.prev.shape[0])

    def upload_bytes(self) -> int:
        """Host bytes this delta moves: arrays, inline records, dictionary suffixes."""
        kd = int(self.kdict.offs[-1]) - int(self.kdict.offs[self.kdict_keep]) + 4 * (self.kdict.n - self.kdict_keep + 1)
        pd = int(self.pdict.offs[-1]) - int(self.pdict.offs[self.pdict_keep]) + 4 * (self.pdict.n - self.pdict_keep + 1)
        remap = 0 if self.prev is None else 4 * len(self.prev) + 8 * self.n_changed
        return (13 * self.n_changed + 4 * (self.n_changed + 1) + 4 * len(self.ref) + 88 * self.records.n + kd + pd
                + 12 * self.vnis.n + remap)

    def to_c(self) -> abi.EpochDelta:
        d = abi.EpochDelta()
        d.kdict, d.pdict = self.kdict.to_c(), self.pdict.to_c()
        d.kdict_keep, d.pdict_keep = self.kdict_keep, self.pdict_keep
        d.n_changed = self.n_changed
        for f in ("topo", "src_ip", "net_ns", "des_off", "ref"):
            a = np.ascontiguousarray(getattr(self, f), np.uint32)
            setattr(self, f, a)
            setattr(d, f, abi.ptr(a if a.size else np.zeros(1, np.uint32), abi.u32p))
        self.spec_nil = np.ascontiguousarray(self.spec_nil, np.uint8)
        d.spec_nil = abi.ptr(self.spec_nil if self.spec_nil.size else np.zeros(1, np.uint8), abi.u8p)
        d.records = self.records.to_c()
        d.vnis = self.vnis.to_c()
        if self.prev is not None:
            for f in ("prev", "ns", "name"):
                a = np.ascontiguousarray(getattr(self, f), np.uint32)
                setattr(self, f, a)
                setattr(d, f, abi.ptr(a if a.size else np.zeros(1, np.uint32), abi.u32p))
            d.n_topos = len(self.prev)
            d.pod_slice = self.pod_slice
        self._keep = d
        return d


def topology_map(prev: EpochInput, new: EpochInput) -> np.ndarray | None:
    """Previous index of every topology of `new` matched by its informer key (namespace,
    name ids; the dictionaries are append-only so ids persist), -1 for a created one; None
    when both list the same Topologies in the same order."""
    P, N = prev.topos, new.topos
    if P.n == N.n and np.array_equal(P.ns, N.ns) and np.array_equal(P.name, N.name):
        return None
    kp = (P.ns.astype(np.uint64) << np.uint64(32)) | P.name.astype(np.uint64)
    kn = (N.ns.astype(np.uint64) << np.uint64(32)) | N.name.astype(np.uint64)
    order = np.argsort(kp, kind="stable")
    ks = kp[order]
    j = np.minimum(np.searchsorted(ks, kn), max(len(ks) - 1, 0))
    hit = (ks[j] == kn) if len(ks) else np.zeros(N.n, bool)
    pmap = np.where(hit, order[j] if len(ks) else 0, -1).astype(np.int64)
    kept = pmap[pmap >= 0]
    assert len(np.unique(kept)) == len(kept), "a Topology key listed twice"
    return pmap


def build_delta(prev: EpochInput, new: EpochInput, kdict_keep: int = 0, pdict_keep: int = 0,
                vnis: Vnis | None = None, pod_slice: int = 0) -> Delta:
    """The delta that turns the engine's state after `prev` (its desired store and topology
    rows) into `new`'s desired side. The dictionaries' kept prefixes are shared (ids of the
    previous epoch stay valid). Topologies are matched by (namespace, name): a Topology only
    in `new` is created (its spec inline, its status nil), one only in `prev` deleted.
    vnis: the VxlanManager snapshot the delta carries — by default `new`'s own snapshot, so
    the delta describes the same epoch a full upload of `new` would (Vnis.keep_resident()
    keeps the engine's map instead)."""
    P, N = prev.topos, new.topos
    pmap = topology_map(prev, new)
    T = N.n
    if pmap is None:
        pmap_ = np.arange(T, dtype=np.int64)
    else:
        pmap_ = pmap
    kept = pmap_ >= 0
    pk = np.where(kept, pmap_, 0)
    po, no = P.des_off.astype(np.int64), N.des_off.astype(np.int64)
    plen_all = np.diff(po)
    plen = np.where(kept, plen_all[pk] if P.n else 0, -1)
    nlen = np.diff(no)
    ph, nh = record_hash(prev.desired), record_hash(new.desired)
    tn = _seg(N.des_off)
    rel = np.arange(new.desired.n, dtype=np.int64) - no[tn]
    same_len = kept & (plen == nlen)
    pos_old = np.where(same_len[tn], po[pk[tn]] + rel, 0) if len(tn) else np.zeros(0, np.int64)
    if len(nh) and len(ph):
        pos_eq = same_len[tn] & (ph[pos_old] == nh)
    else:
        pos_eq = np.zeros(len(nh), bool)
    if pos_eq.any():                                              # hashes equal: verify exactly
        k = np.nonzero(pos_eq)[0]
        pos_eq[k] = _same_records(prev.desired, pos_old[k], new.desired, k)
    differs = np.bincount(tn[~pos_eq], minlength=T) > 0 if len(tn) else np.zeros(T, bool)
    nil_bit = (N.flags & abi.TOPO_SPEC_NIL) != 0
    p_src = np.where(kept, P.src_ip[pk] if P.n else 0, 0)
    p_net = np.where(kept, P.net_ns[pk] if P.n else 0, 0)
    p_nil = np.where(kept, (P.flags[pk] & abi.TOPO_SPEC_NIL) != 0 if P.n else False, False)
    changed = (~kept | ~same_len | differs | (p_src != N.src_ip) | (p_net != N.net_ns) | (p_nil != nil_bit))
    topo = np.nonzero(changed)[0]
    # records of the changed Topologies: a previous record with the same content (same
    # Topology first: the positional one, else any by hash), else inline
    sel = np.nonzero(changed[tn])[0] if len(tn) else np.zeros(0, np.int64)
    ref = np.full(len(sel), abi.DELTA_NEW, np.uint64)
    hit = pos_eq[sel]
    ref[hit] = pos_old[sel[hit]]
    miss = sel[~hit]
    if len(miss) and len(ph):
        oord = np.argsort(ph, kind="stable")
        osort = ph[oord]
        j = np.minimum(np.searchsorted(osort, nh[miss]), len(osort) - 1)
        cand = oord[j]
        ok = osort[j] == nh[miss]
        if ok.any():
            k = np.nonzero(ok)[0]
            ok[k] = _same_records(prev.desired, cand[k], new.desired, miss[k])
        r = np.where(~hit)[0]
        ref[r[ok]] = cand[ok]
    new_rec = sel[ref == abi.DELTA_NEW]
    ref[ref == abi.DELTA_NEW] = abi.DELTA_NEW | np.arange(len(new_rec), dtype=np.uint64)
    des_off = np.zeros(len(topo) + 1, np.uint32)
    np.cumsum(nlen[topo], out=des_off[1:]) if len(topo) else None
    d = Delta(new.kdict, new.pdict, kdict_keep, pdict_keep, topo.astype(np.uint32), N.src_ip[topo].astype(np.uint32),
              N.net_ns[topo].astype(np.uint32), nil_bit[topo].astype(np.uint8), des_off, ref.astype(np.uint32),
              new.desired.take(new_rec), vnis if vnis is not None else new.vnis)
    if pmap is not None:
        d.prev = np.where(pmap >= 0, pmap, abi.DELTA_NEW).astype(np.uint32)
        d.ns, d.name = N.ns[topo].astype(np.uint32), N.name[topo].astype(np.uint32)
        d.pod_slice = pod_slice
    return d
