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


def apply_delta(state: EpochInput, delta) -> EpochInput:
    """The epoch tables after kdtn_epoch_upload_delta(delta) on `state`."""
    T = state.topos
    no = T.des_off.astype(np.int64)
    pos = {int(t): k for k, t in enumerate(delta.topo)}
    parts = []
    lens = np.diff(no).copy()
    src, net, fl = T.src_ip.copy(), T.net_ns.copy(), T.flags.copy()
    for t in range(T.n):
        k = pos.get(t)
        if k is None:
            parts.append(("old", np.arange(no[t], no[t + 1])))
            continue
        r = delta.ref[delta.des_off[k]:delta.des_off[k + 1]].astype(np.int64)
        parts.append(("ref", r))
        lens[t] = len(r)
        src[t], net[t] = delta.src_ip[k], delta.net_ns[k]
        fl[t] = (int(fl[t]) & (0xFF ^ abi.TOPO_SPEC_NIL)) | (abi.TOPO_SPEC_NIL if delta.spec_nil[k] else 0)
    n = int(lens.sum())
    L = Links.empty(n)
    d = 0
    for kind, r in parts:
        for x in r.tolist():
            if kind == "ref" and x & abi.DELTA_NEW:
                s, j = delta.records, x & ~abi.DELTA_NEW
            else:
                s, j = state.desired, x
            L.key[:, d], L.prop[:, d], L.uid[d], L.gap[d] = s.key[:, j], s.prop[:, j], s.uid[j], s.gap[j]
            d += 1
    off = np.zeros(T.n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    topos = Topos(T.ns, T.name, src, net, fl, T.real_off, off.astype(np.uint32))
    return EpochInput(delta.kdict, delta.pdict, topos, state.realised, L, delta.vnis, pod_slice=state.pod_slice)


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
