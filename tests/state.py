"""Host restatement of the resident-state operations (test infrastructure): what
kdtn_epoch_commit and kdtn_epoch_upload_delta must leave in the engine.

commit: Reconcile's Status.Links = Spec.Links for CREATED Topologies and for DIFF Topologies
whose DelLinks / AddLinks / UpdateLinks RPCs all succeed (controllers/topology_controller.go:
81-85, 93-116, 125-138); a failing entry (delLink / addLink / UpdateLinks error, or the peer
rejecting a RemotePod) stops the Topology's RPC sequence and its status stays.
delta: the new desired store is the previous one with the changed Topologies' segments
replaced by their reference lists (previous record or inline record)."""
from __future__ import annotations

import numpy as np

from kdtn import abi
from kdtn.tables import EpochInput, Links, Topos


def _seg(off):
    off = np.asarray(off, np.int64)
    return np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))


def predicted_commit(inp: EpochInput, out) -> np.ndarray:
    """The engine's default commit decision per Topology (kdtn_epoch_commit mask = NULL)."""
    T = inp.topos.n
    fail = np.zeros(T, bool)
    if len(out.del_idx):
        fail |= np.bincount(_seg(out.del_off)[:len(out.del_idx)], weights=out.del_res["err"] != 0, minlength=T) > 0
    if len(out.add_idx):
        r, q = out.add_res, out.add_qdisc
        kinds = np.isin(r["kind"], (abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL))
        f = (r["err"] != 0) | (kinds & (q["err"] != 0)) | (r["remote_err"] != 0)
        fail |= np.bincount(_seg(out.add_off)[:len(out.add_idx)], weights=f, minlength=T) > 0
    if len(out.upd_idx):
        fail |= np.bincount(_seg(out.upd_off)[:len(out.upd_idx)], weights=out.upd_res["err"] != 0, minlength=T) > 0
    act = out.action
    return (act == abi.ACT_CREATED) | ((act == abi.ACT_DIFF) & ~fail)


def commit(inp: EpochInput, mask: np.ndarray) -> EpochInput:
    """The epoch tables after Status.Links = Spec.Links for the Topologies in mask."""
    T = inp.topos
    mask = np.asarray(mask, bool)
    ro, no = T.real_off.astype(np.int64), T.des_off.astype(np.int64)
    lens = np.where(mask, np.diff(no), np.diff(ro))
    off = np.zeros(T.n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    idx_side = []
    for t in range(T.n):
        idx_side.append((1, no[t], no[t + 1]) if mask[t] else (0, ro[t], ro[t + 1]))
    take_r = np.concatenate([np.arange(a, b) for s, a, b in idx_side if s == 0] or [np.zeros(0, np.int64)])
    take_d = np.concatenate([np.arange(a, b) for s, a, b in idx_side if s == 1] or [np.zeros(0, np.int64)])
    # interleave in topology order
    src = np.repeat(mask.astype(np.int8), lens)
    L = Links.empty(int(off[-1]))
    for side, take, sel in ((inp.realised, take_r, src == 0), (inp.desired, take_d, src == 1)):
        L.key[:, sel] = side.key[:, take]
        L.prop[:, sel] = side.prop[:, take]
        L.uid[sel] = side.uid[take]
        L.gap[sel] = side.gap[take]
    fl = T.flags.copy()
    spec_nil = (fl & abi.TOPO_SPEC_NIL) != 0
    fl[mask] = (fl[mask] & np.uint8(0xFF ^ abi.TOPO_STATUS_NIL)) | np.where(spec_nil[mask], abi.TOPO_STATUS_NIL, 0).astype(np.uint8)
    topos = Topos(T.ns, T.name, T.src_ip, T.net_ns, fl, off.astype(np.uint32), T.des_off)
    return EpochInput(inp.kdict, inp.pdict, topos, L, inp.desired, inp.vnis, pod_slice=inp.pod_slice)


def _gather(L: Links, idx: np.ndarray, out: Links, sel: np.ndarray) -> None:
    out.key[:, sel] = L.key[:, idx]
    out.prop[:, sel] = L.prop[:, idx]
    out.uid[sel] = L.uid[idx]
    out.gap[sel] = L.gap[idx]


def _segments(off: np.ndarray, which: np.ndarray) -> np.ndarray:
    """Concatenated record indices of the segments [off[t], off[t+1]) for t in `which`."""
    off = np.asarray(off, np.int64)
    lens = off[which + 1] - off[which]
    if not len(which) or lens.sum() == 0:
        return np.zeros(0, np.int64)
    start = np.repeat(off[which], lens)
    within = np.arange(int(lens.sum()), dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens)
    return start + within


def apply_delta(state: EpochInput, delta) -> EpochInput:
    """The epoch tables after kdtn_epoch_upload_delta(delta) on `state`: per new Topology its
    previous row (or, created, the delta's ns / name with a nil status and no realised
    records), the changed Topologies' spec from their reference lists, the rest unchanged."""
    T0 = state.topos
    if delta.prev is None:
        pmap = np.arange(T0.n, dtype=np.int64)
    else:
        pv = delta.prev.astype(np.int64)
        pmap = np.where(pv == abi.DELTA_NEW, -1, pv)
    Tn = len(pmap)
    kept = pmap >= 0
    pk = np.where(kept, pmap, 0)
    chg = np.full(Tn, -1, np.int64)
    chg[delta.topo.astype(np.int64)] = np.arange(delta.n_changed)
    ro, no = T0.real_off.astype(np.int64), T0.des_off.astype(np.int64)
    # topology rows
    ns = np.where(kept, T0.ns[pk] if T0.n else 0, 0).astype(np.uint32)
    name = np.where(kept, T0.name[pk] if T0.n else 0, 0).astype(np.uint32)
    src = np.where(kept, T0.src_ip[pk] if T0.n else 0, 0).astype(np.uint32)
    net = np.where(kept, T0.net_ns[pk] if T0.n else 0, 0).astype(np.uint32)
    fl = np.where(kept, T0.flags[pk] if T0.n else 0, abi.TOPO_STATUS_NIL).astype(np.uint8)
    c = chg >= 0
    k = chg[c]
    if delta.prev is not None:
        created = c & ~kept
        ns[created], name[created] = delta.ns[chg[created]], delta.name[chg[created]]
    src[c], net[c] = delta.src_ip[k], delta.net_ns[k]
    fl[c] = (fl[c] & np.uint8(0xFF ^ abi.TOPO_SPEC_NIL)) | np.where(delta.spec_nil[k] != 0, abi.TOPO_SPEC_NIL, 0).astype(np.uint8)
    # realised: kept Topologies' status segments in the new order
    rlen = np.where(kept, (ro[pk + 1] - ro[pk]) if T0.n else 0, 0)
    roff = np.zeros(Tn + 1, np.int64)
    np.cumsum(rlen, out=roff[1:])
    ridx = _segments(T0.real_off, pk[kept]) if kept.any() else np.zeros(0, np.int64)
    R = Links.empty(int(roff[-1]))
    _gather(state.realised, ridx, R, np.arange(len(ridx)))
    # desired: unchanged kept Topologies keep their segment, changed ones take their references
    dlen = np.where(kept, (no[pk + 1] - no[pk]) if T0.n else 0, 0)
    dlen[c] = delta.des_off[k + 1].astype(np.int64) - delta.des_off[k].astype(np.int64)
    doff = np.zeros(Tn + 1, np.int64)
    np.cumsum(dlen, out=doff[1:])
    L = Links.empty(int(doff[-1]))
    src_kind = np.zeros(L.n, np.int8)          # 0 previous desired record, 1 inline record
    src_idx = np.zeros(L.n, np.int64)
    keep_t = np.nonzero(~c & kept)[0]
    dst = _segments(doff, keep_t)
    src_idx[dst] = _segments(T0.des_off, pk[keep_t])
    chg_t = np.nonzero(c)[0]
    dst = _segments(doff, chg_t)
    refs = delta.ref[_segments(delta.des_off, chg[chg_t])].astype(np.int64)
    inl = (refs & abi.DELTA_NEW) != 0
    src_kind[dst] = inl
    src_idx[dst] = np.where(inl, refs & ~abi.DELTA_NEW, refs)
    _gather(state.desired, src_idx[src_kind == 0], L, src_kind == 0)
    _gather(delta.records, src_idx[src_kind == 1], L, src_kind == 1)
    topos = Topos(ns, name, src, net, fl, roff.astype(np.uint32), doff.astype(np.uint32))
    slice_ = state.pod_slice if delta.prev is None else (delta.pod_slice or 0)
    return EpochInput(delta.kdict, delta.pdict, topos, R, L, delta.vnis, pod_slice=slice_)


def same_tables(a: EpochInput, b: EpochInput) -> list[str]:
    """Names of the table columns that differ (empty = identical)."""
    bad = []
    for f in ("ns", "name", "src_ip", "net_ns", "flags", "real_off", "des_off"):
        if not np.array_equal(getattr(a.topos, f), getattr(b.topos, f)):
            bad.append(f)
    for side in ("realised", "desired"):
        x, y = getattr(a, side), getattr(b, side)
        for f in ("key", "prop", "uid", "gap"):
            if not np.array_equal(getattr(x, f), getattr(y, f)):
                bad.append(f"{side}.{f}")
    return bad
