"""getPod's API-server fallback (daemon/kubedtn/handler.go:27-41) across the C-ABI.

The informer store the engine resolves peers against may miss a Topology the API server has
(the GET at handler.go:38). Driver contract (include/kdtn.h, kdtn_epoch_late_pods): the
first run reports those peers as KDTN_E_PEER_LOOKUP; the driver lists the missed keys
(model.peer_misses), GETs them, grows the dictionary by an empty delta when the fetched
strings are new, passes the fetched pod rows to kdtn_epoch_late_pods and runs again. The
second run must equal the oracle over a table that holds the fetched Topologies (as rows
after the informer's, with no lists of their own) — i.e. what the reference computes once
its GET returned them.
"""
import random

import numpy as np
import pytest

import oracle as O
from helpers import random_epoch
from kdtn import abi, synth
from kdtn.delta import build_delta
from kdtn.model import Topology, TopologyReconciler, late_pod_rows, pack, peer_misses, unpack
from kdtn.tables import BatchesOut, EpochInput, Interner, Topos

pytestmark = pytest.mark.gpu
TICK = 15.625


def _trim(out: BatchesOut, T: int) -> BatchesOut:
    """The first T topologies' outputs (the rows after them have no entries)."""
    assert out.del_off[T] == out.del_off[-1] and out.add_off[T] == out.add_off[-1] and out.upd_off[T] == out.upd_off[-1]
    return BatchesOut(out.action[:T], out.del_off[:T + 1], out.add_off[:T + 1], out.upd_off[:T + 1],
                      out.del_idx, out.add_idx, out.upd_idx, out.del_res, out.add_res, out.upd_res,
                      out.add_qdisc, out.upd_qdisc)


def _with_rows(inp: EpochInput, kdict, rows: np.ndarray, spec_nil: np.ndarray) -> EpochInput:
    """inp's table plus one list-less Topology per late row (status = spec: no entries)."""
    T = inp.topos
    n = len(rows)
    nil = np.where(spec_nil, abi.TOPO_SPEC_NIL | abi.TOPO_STATUS_NIL, 0).astype(np.uint8)
    cat = lambda a, b: np.concatenate([a, b.astype(a.dtype)])
    topos = Topos(cat(T.ns, rows[:, 0]), cat(T.name, rows[:, 1]), cat(T.src_ip, rows[:, 2]),
                  cat(T.net_ns, rows[:, 3] & 0x7FFFFFFF), cat(T.flags, nil),
                  cat(T.real_off, np.full(n, T.real_off[-1])), cat(T.des_off, np.full(n, T.des_off[-1])))
    return EpochInput(kdict, inp.pdict, topos, inp.realised, inp.desired, inp.vnis)


def _assert_same(got, want, ctx):
    bad = got.mismatches(want)
    assert not bad, f"{ctx}: {bad}"


@pytest.mark.parametrize("seed", range(6))
def test_late_pods_random_epochs(engine, seed):
    """Random adversarial epochs with a fifth of the Topologies missing from the informer
    store; their strings partly new to the dictionary (the delta grows it first)."""
    rng = random.Random(seed)
    topos, vnis = random_epoch(seed, T=150, p_err=0.15)
    late_i = set(rng.sample(range(len(topos)), 30))
    kept = [t for i, t in enumerate(topos) if i not in late_i]
    # the API server's objects by key (a Topology always has a namespace there)
    store = {(t.namespace, t.name): t for i, t in enumerate(topos) if i in late_i and t.namespace}
    for t in store.values():                        # status strings the kept table never named
        if rng.random() < 0.5:
            t.src_ip = t.src_ip and f"10.9.{rng.randint(0, 255)}.{rng.randint(0, 255)}"
            t.net_ns = t.net_ns and f"/run/late/{t.name}"
    kd, pd = Interner(), Interner()
    inp = pack(kept, vnis, kd, pd)
    out0 = engine.reconcile(inp)
    _assert_same(out0, O.reconcile(inp, tick=TICK), f"seed {seed}: informer only")
    misses = peer_misses(inp, out0)
    fetched = [store[(ns.decode(), name.decode())] for ns, name in misses if (ns.decode(), name.decode()) in store]
    assert fetched, "the epoch should miss some of the late Topologies"
    D0 = inp.kdict.n
    rows = late_pod_rows(fetched, kd)
    grown = EpochInput(kd.table(), inp.pdict, inp.topos, inp.realised, inp.desired, inp.vnis)
    d = build_delta(inp, grown, D0, inp.pdict.n)
    assert d.n_changed == 0
    engine.upload_delta(d)
    engine.late_pods(rows)
    engine.run()
    engine.sync()
    out1 = engine.download()
    want = O.reconcile(_with_rows(grown, grown.kdict, rows, np.array([t.spec_links is None for t in fetched])),
                       tick=TICK)
    _assert_same(out1, _trim(want, len(kept)), f"seed {seed}: with late pods")
    # every fetched key resolves now; what remains missed is what the API server lacks too
    left = {(ns.decode(), name.decode()) for ns, name in peer_misses(grown, out1)}
    assert not left & set(store), left & set(store)
    # the rows are cleared by the next upload: the informer-only answer again
    engine.upload(inp)
    engine.run()
    engine.sync()
    _assert_same(engine.download(), out0, f"seed {seed}: late rows cleared")


def test_late_pods_mirror_reconciler(engine):
    """TopologyReconciler.reconcile_all(fetch=...) gives the batches of the whole store."""
    topos, vnis = random_epoch(11, T=120, p_err=0.1)
    late = {(t.namespace, t.name): t for t in topos[80:] if t.namespace}
    kept = topos[:80]
    order = []

    def fetch(ns, name):
        t = late.get((ns, name))
        if t is not None:
            order.append(t)
        return t
    got = TopologyReconciler(engine).reconcile_all(kept, vnis, fetch=fetch)
    assert order
    stubs = [Topology(t.name, t.namespace, None if t.spec_links is None else [],
                      None if t.spec_links is None else [], t.src_ip, t.net_ns) for t in order]
    full = pack(kept + stubs, vnis)
    want = unpack(kept, _trim(O.reconcile(full, tick=TICK), len(kept)))
    for a, b in zip(got, want):
        assert a.action == b.action and a.add == b.add and a.delete == b.delete
        assert a.properties_changed == b.properties_changed
        assert a.add_res.tobytes() == b.add_res.tobytes() and a.add_qdisc.tobytes() == b.add_qdisc.tobytes()


def test_late_pods_config2_tail():
    """Config-2 shape (20k pods): the last 5 % of the Topologies missing from the informer
    store, supplied late; every output field equals the oracle over the whole table."""
    from kdtn import Engine
    inp = synth.make(2, total_pods=20000)
    T = inp.topos
    K = T.n // 20
    Tk = T.n - K
    nk = int(T.des_off[Tk])
    rk = int(T.real_off[Tk])
    cut = EpochInput(inp.kdict, inp.pdict,
                     Topos(T.ns[:Tk], T.name[:Tk], T.src_ip[:Tk], T.net_ns[:Tk], T.flags[:Tk],
                           T.real_off[:Tk + 1], T.des_off[:Tk + 1]),
                     inp.realised.take(np.arange(rk)), inp.desired.take(np.arange(nk)), inp.vnis)
    spec_nil = (T.flags[Tk:] & abi.TOPO_SPEC_NIL) != 0
    rows = np.stack([T.ns[Tk:], T.name[Tk:], T.src_ip[Tk:],
                     T.net_ns[Tk:] | np.where(spec_nil, 0x80000000, 0).astype(np.uint32)]).T.astype(np.uint32)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        out0 = eng.reconcile(cut)
        assert (out0.add_res["err"] == abi.E_PEER_LOOKUP).sum() > 0
        eng.late_pods(rows)
        eng.run()
        eng.sync()
        out1 = eng.download()
    assert (out1.add_res["err"] == abi.E_PEER_LOOKUP).sum() == 0
    want = O.reconcile(_with_rows(cut, cut.kdict, rows, spec_nil), tick=TICK)
    _assert_same(out1, _trim(want, Tk), "config-2 tail")
