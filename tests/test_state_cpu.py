"""CPU: the resident-state host pieces — kdtn.delta.build_delta (the delta a controller sends
instead of the whole epoch) reproduces the next epoch exactly when applied to the previous
state (tests/state.py restatement of kdtn_epoch_upload_delta), moves little data for
churn-sized changes, and the commit restatement follows Reconcile's status write."""
import copy
import random

import numpy as np

import oracle as O
from helpers import random_epoch
from kdtn import abi, synth
from kdtn.delta import build_delta, record_hash
from kdtn.model import Link, LinkProperties, pack
from kdtn.tables import Interner
from state import apply_delta, commit, predicted_commit, same_tables


def mutate(topos, seed):
    """The next epoch of a Topology set: spec edits (deletes, property changes, new links,
    reorders, nil <-> list), status rows moving node, most Topologies untouched."""
    rng = random.Random(seed)
    out = copy.deepcopy(topos)
    for t in out:
        r = rng.random()
        if r < 0.5:
            continue
        if r < 0.55:
            t.spec_links = None
            continue
        if r < 0.6:
            t.src_ip = rng.choice(["10.0.0.1", "10.0.0.2", "10.0.0.9"])
        sp = list(t.spec_links or [])
        new = []
        for l in sp:
            x = rng.random()
            if x < 0.15:
                continue
            l = copy.deepcopy(l)
            if x < 0.3:
                l.properties = LinkProperties(latency=f"{rng.randint(1, 99)}ms", loss="0.5")
            new.append(l)
        for _ in range(rng.choice([0, 1, 2])):
            new.append(Link("eth9", "10.9.0.1/31", "", "eth8", "", "", rng.choice([x.name for x in out]),
                            rng.randint(1, 10**6), LinkProperties(rate="10Mbit")))
        if rng.random() < 0.2:
            rng.shuffle(new)
        t.spec_links = new
    return out


def test_delta_roundtrip_random_epochs():
    for seed in range(6):
        topos, _ = random_epoch(seed, T=120)
        kd, pd = Interner(), Interner()
        a = pack(topos, kdict=kd, pdict=pd)
        state = commit(a, np.ones(a.topos.n, bool))          # every Topology's status = spec
        b_topos = mutate(topos, seed + 100)
        ka, pa = a.kdict.n, a.pdict.n
        b = pack(b_topos, kdict=kd, pdict=pd)
        d = build_delta(a, b, ka, pa)
        got = apply_delta(state, d)
        assert not same_tables(got, type(b)(b.kdict, b.pdict, b.topos.__class__(
            b.topos.ns, b.topos.name, b.topos.src_ip, b.topos.net_ns,
            (state.topos.flags & abi.TOPO_STATUS_NIL) | (b.topos.flags & abi.TOPO_SPEC_NIL),
            state.topos.real_off, b.topos.des_off), state.realised, b.desired)), seed
        assert 0 < d.n_changed < a.topos.n
        assert (d.ref & abi.DELTA_NEW == 0).sum() > d.records.n      # most records referenced


def test_delta_is_small_for_churn():
    cs = synth.ChurnSequence(total_pods=5000)
    prev = cs.epoch_input(copy=True)
    cs.advance()
    new = cs.epoch_input(copy=True)
    d = build_delta(prev, new, prev.kdict.n, prev.pdict.n)
    full = 88 * new.desired.n + 25 * new.topos.n
    assert d.upload_bytes() < 0.1 * full, (d.upload_bytes(), full)
    state = commit(prev, np.ones(prev.topos.n, bool))
    got = apply_delta(state, d)
    assert np.array_equal(record_hash(got.desired), record_hash(new.desired))
    assert np.array_equal(got.topos.des_off, new.topos.des_off)


def test_predicted_commit_follows_reconcile():
    """CREATED and clean DIFF Topologies commit; a failing delLink / addLink (incl. a remote
    rejection) / UpdateLinks entry keeps the status (test_reach_cpu scenario)."""
    from test_reach_cpu import scenario
    inp = pack(scenario())
    out = O.reconcile(inp, tick=15.625)
    m = predicted_commit(inp, out)
    # a: remote rejection; b, c: SKIP (empty == empty); d: delLink fails; e: an UpdateLinks fails
    assert m.tolist() == [False, False, False, False, False]
    topos, _ = random_epoch(3, T=80)
    inp = pack(topos)
    out = O.reconcile(inp, tick=15.625)
    m = predicted_commit(inp, out)
    assert m[out.action == abi.ACT_CREATED].all() and not m[out.action == abi.ACT_SKIP].any()
    assert 0 < m.sum() < inp.topos.n
    st = commit(inp, m)
    nil = (st.topos.flags & abi.TOPO_STATUS_NIL) != 0
    assert np.array_equal(nil[m], (inp.topos.flags[m] & abi.TOPO_SPEC_NIL) != 0)


def _expected_after_delta(state, new, d):
    """What the state must be after the delta: new's rows, spec and desired side; each kept
    Topology's status carried over, a created one's nil and empty."""
    from kdtn.delta import topology_map
    from kdtn.tables import Links, Topos
    pmap = topology_map(state, new)
    pmap = np.arange(new.topos.n) if pmap is None else pmap
    kept = pmap >= 0
    ro = state.topos.real_off.astype(np.int64)
    rlen = np.where(kept, ro[np.maximum(pmap, 0) + 1] - ro[np.maximum(pmap, 0)], 0)
    roff = np.zeros(new.topos.n + 1, np.int64)
    np.cumsum(rlen, out=roff[1:])
    idx = np.concatenate([np.arange(ro[p], ro[p + 1]) for p in pmap[kept]] or [np.zeros(0, np.int64)])
    real = state.realised.take(idx) if len(idx) else Links.empty(0)
    st_nil = np.where(kept, state.topos.flags[np.maximum(pmap, 0)] & abi.TOPO_STATUS_NIL, abi.TOPO_STATUS_NIL)
    fl = (st_nil | (new.topos.flags & abi.TOPO_SPEC_NIL)).astype(np.uint8)
    T = new.topos
    return type(new)(new.kdict, new.pdict, Topos(T.ns, T.name, T.src_ip, T.net_ns, fl, roff.astype(np.uint32),
                                                 T.des_off), real, new.desired)


def _delete_and_create(topos, seed):
    """Some Topologies deleted, some new ones created (new names) linking to live pods."""
    rng = random.Random(seed)
    out = [t for t in copy.deepcopy(topos) if rng.random() > 0.1]
    names = [t.name for t in out]
    for k in range(rng.randint(1, 8)):
        t = copy.deepcopy(rng.choice(topos))
        t.name = f"created-{seed}-{k}"
        t.status_links = None
        t.spec_links = [Link("eth1", "10.7.0.1/31", "", "eth2", "10.7.0.2/31", "", rng.choice(names),
                             rng.randint(1, 10**6), LinkProperties(latency="3ms"))] if rng.random() < 0.8 else None
        out.insert(rng.randint(0, len(out)), t)
    return out


def test_delta_topology_set_changes():
    """Created and deleted Topologies (informer add / delete events) in one delta: the
    restatement of kdtn_epoch_upload_delta leaves exactly the next epoch's rows and spec, the
    kept Topologies' status moved with them and a nil status for the created ones."""
    for seed in range(6):
        topos, _ = random_epoch(seed, T=100)
        kd, pd = Interner(), Interner()
        a = pack(topos, kdict=kd, pdict=pd)
        mask = np.random.default_rng(seed).random(a.topos.n) < 0.7
        state = commit(a, mask)
        ka, pa = a.kdict.n, a.pdict.n
        b = pack(_delete_and_create(mutate(topos, seed + 50), seed), kdict=kd, pdict=pd)
        d = build_delta(state, b, ka, pa)
        assert d.prev is not None and (d.prev == abi.DELTA_NEW).any() and d.n_topos == b.topos.n
        created = d.prev[d.topo] == abi.DELTA_NEW
        assert (d.prev == abi.DELTA_NEW).sum() == created.sum()       # every created one has its spec
        got = apply_delta(state, d)
        assert not same_tables(got, _expected_after_delta(state, b, d)), seed


def test_delta_from_an_empty_desired_store():
    """The previous epoch had no spec records at all (every spec nil or empty): every record
    of the next one is inline."""
    topos, _ = random_epoch(2, T=30)
    kd, pd = Interner(), Interner()
    empty = copy.deepcopy(topos)
    for t in empty:
        t.spec_links = None
    a = pack(empty, kdict=kd, pdict=pd)
    assert a.desired.n == 0
    b = pack(topos, kdict=kd, pdict=pd)
    d = build_delta(a, b, a.kdict.n, a.pdict.n)
    assert d.records.n == b.desired.n and (d.ref & abi.DELTA_NEW != 0).all()
    state = commit(a, np.ones(a.topos.n, bool))
    assert not same_tables(apply_delta(state, d), _expected_after_delta(state, b, d))


def test_topology_set_churn_chain_roundtrip():
    """Three epochs of config-3 churn with 1 % of the Topologies deleted / re-created per epoch
    through build_delta + the restatement equal the generator's epochs."""
    tc = synth.TopologySetChurn(frac=0.02, total_pods=3000)
    prev = tc.epoch_input()
    state = commit(prev, np.ones(prev.topos.n, bool))
    for _ in range(3):
        tc.advance()
        new = tc.epoch_input()
        d = build_delta(state, new, state.kdict.n, state.pdict.n)
        assert d.prev is not None and (d.prev == abi.DELTA_NEW).sum() > 0
        assert new.topos.n - (d.prev != abi.DELTA_NEW).sum() == (d.prev == abi.DELTA_NEW).sum()
        got = apply_delta(state, d)
        assert not same_tables(got, _expected_after_delta(state, new, d))
        state = commit(got, np.ones(got.topos.n, bool))
