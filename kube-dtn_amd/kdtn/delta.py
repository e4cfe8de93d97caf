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
    topo: np.ndarray        # u32 [n_changed]
    src_ip: np.ndarray      # u32
    net_ns: np.ndarray      # u32
    spec_nil: np.ndarray    # u8
    des_off: np.ndarray     # u32 [n_changed + 1]
    ref: np.ndarray         # u32
    records: Links
    vnis: Vnis

    @property
    def n_changed(self) -> int:
        return int(self.topo.shape[0])

    def upload_bytes(self) -> int:
        """Host bytes this delta moves: arrays, inline records, dictionary suffixes."""
        kd = int(self.kdict.offs[-1]) - int(self.kdict.offs[self.kdict_keep]) + 4 * (self.kdict.n - self.kdict_keep + 1)
        pd = int(self.pdict.offs[-1]) - int(self.pdict.offs[self.pdict_keep]) + 4 * (self.pdict.n - self.pdict_keep + 1)
        return (13 * self.n_changed + 4 * (self.n_changed + 1) + 4 * len(self.ref) + 88 * self.records.n + kd + pd
                + 12 * self.vnis.n)

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
        self._keep = d
        return d


def build_delta(prev: EpochInput, new: EpochInput, kdict_keep: int = 0, pdict_keep: int = 0,
                vnis: Vnis | None = None) -> Delta:
    """The delta that turns the engine's state after `prev` (its desired store and topology
    rows) into `new`'s desired side. Both epochs list the same Topologies in the same order
    and share the dictionaries' kept prefixes (ids of the previous epoch stay valid)."""
    P, N = prev.topos, new.topos
    assert P.n == N.n and np.array_equal(P.ns, N.ns) and np.array_equal(P.name, N.name), "same Topology set"
    T = N.n
    po, no = P.des_off.astype(np.int64), N.des_off.astype(np.int64)
    plen, nlen = np.diff(po), np.diff(no)
    ph, nh = record_hash(prev.desired), record_hash(new.desired)
    tn = _seg(N.des_off)
    rel = np.arange(new.desired.n, dtype=np.int64) - no[tn]
    same_len = plen == nlen
    pos_old = np.where(same_len[tn], po[tn] + rel, 0)
    pos_eq = same_len[tn] & (ph[pos_old] == nh) if len(nh) else np.zeros(0, bool)
    if pos_eq.any():                                              # hashes equal: verify exactly
        k = np.nonzero(pos_eq)[0]
        pos_eq[k] = _same_records(prev.desired, pos_old[k], new.desired, k)
    differs = np.bincount(tn[~pos_eq], minlength=T) > 0 if len(tn) else np.zeros(T, bool)
    nil_bit = (N.flags & abi.TOPO_SPEC_NIL) != 0
    changed = (~same_len | differs | (P.src_ip != N.src_ip) | (P.net_ns != N.net_ns)
               | (((P.flags ^ N.flags) & abi.TOPO_SPEC_NIL) != 0))
    topo = np.nonzero(changed)[0]
    # records of the changed Topologies: a previous record with the same content (same
    # Topology first: the positional one, else any by hash), else inline
    sel = np.nonzero(changed[tn])[0] if len(tn) else np.zeros(0, np.int64)
    ref = np.full(len(sel), abi.DELTA_NEW, np.uint64)
    hit = pos_eq[sel]
    ref[hit] = pos_old[sel[hit]]
    miss = sel[~hit]
    if len(miss):
        oord = np.argsort(ph, kind="stable")
        osort = ph[oord]
        j = np.searchsorted(osort, nh[miss])
        j = np.minimum(j, max(len(osort) - 1, 0))
        cand = oord[j] if len(oord) else np.zeros(len(miss), np.int64)
        ok = (osort[j] == nh[miss]) if len(oord) else np.zeros(len(miss), bool)
        if ok.any():
            k = np.nonzero(ok)[0]
            ok[k] = _same_records(prev.desired, cand[k], new.desired, miss[k])
        r = np.where(~hit)[0]
        ref[r[ok]] = cand[ok]
    new_rec = sel[ref == abi.DELTA_NEW]
    ref[ref == abi.DELTA_NEW] = abi.DELTA_NEW | np.arange(len(new_rec), dtype=np.uint64)
    des_off = np.zeros(len(topo) + 1, np.uint32)
    np.cumsum(nlen[topo], out=des_off[1:]) if len(topo) else None
    return Delta(new.kdict, new.pdict, kdict_keep, pdict_keep, topo.astype(np.uint32), N.src_ip[topo].astype(np.uint32),
                 N.net_ns[topo].astype(np.uint32), nil_bit[topo].astype(np.uint8), des_off, ref.astype(np.uint32),
                 new.desired.take(new_rec), vnis if vnis is not None else Vnis())
