"""Sharded CR ingest (kdtn_json_ingest_shard): every rank decodes the whole TopologyList, so
dictionary ids and pod indices are the document's on every rank, and keeps only the
Topologies it owns (kdtn_topology_shard(namespace, name, G) == rank). Per rank: the kept
topologies are exactly the hash shard in document order, the shard's tables are the oracle's
full-document tables restricted to them, and its epoch equals the unsharded oracle epoch
topology for topology (peers are document indices on both sides, no mapping)."""
import numpy as np
import pytest

import oracle as O
from multishard import per_topology

pytestmark = pytest.mark.gpu
TICK = 15.625


def _kstr(tabs, i):
    o = tabs.kdict.offs
    return tabs.kdict.bytes_[o[i]:o[i + 1]].tobytes()


def _restrict(want, keep):
    """the oracle's full tables cut down to the topologies `keep` (document order)"""
    t = want.topos
    cols = {f: getattr(t, f)[keep] for f in ("ns", "name", "src_ip", "net_ns", "flags")}
    sides = {}
    for side, off in (("realised", t.real_off), ("desired", t.des_off)):
        L = getattr(want, side)
        rec = np.concatenate([np.arange(off[k], off[k + 1]) for k in keep]) if len(keep) else np.zeros(0, np.int64)
        cnt = np.array([off[k + 1] - off[k] for k in keep], np.int64)
        sides[side] = (L.key[:, rec], L.prop[:, rec], L.gap[rec], L.uid[rec],
                       np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32))
    return cols, sides


@pytest.mark.parametrize("config,nshards", [(1, 2), (3, 3), (4, 2), (4, 5)])
def test_sharded_ingest_equals_unsharded(config, nshards):
    from kdtn import Engine, synth, topology_shard
    kw = dict(pods_per_shard=3000) if config in (3, 4) else {}
    inp = synth.make(config, **kw)
    doc = synth.topology_list_json(inp)
    err, _, want = O.json_ingest(doc)
    assert err == 0
    ref = per_topology(want, O.reconcile(want, tick=TICK))
    T = want.topos.n
    owner = np.array([topology_shard(_kstr(want, int(want.topos.ns[t])), _kstr(want, int(want.topos.name[t])),
                                     nshards) for t in range(T)])
    eng = Engine(device=0, tick_in_usec=TICK, vxlan_base=5000)
    try:
        seen = np.zeros(T, np.int64)
        for r in range(nshards):
            keep = np.nonzero(owner == r)[0]
            info = eng.ingest(doc, shard=(nshards, r))
            assert (info.n_topos, info.n_kdict, info.n_pdict) == (len(keep), want.kdict.n, want.pdict.n)
            doc_idx = eng.ingest_doc_index()
            assert (doc_idx == keep).all(), f"shard {r}: kept topologies differ from the hash shard"
            got = eng.ingest_tables()
            cols, sides = _restrict(want, keep)
            for f, v in cols.items():
                assert (getattr(got.topos, f) == v).all(), f"shard {r}: topos.{f}"
            for side, (key, prop, gap, uid, off) in sides.items():
                L = getattr(got, side)
                assert (L.key == key).all() and (L.prop == prop).all(), f"shard {r}: {side} ids"
                assert (L.gap == gap).all() and (L.uid == uid).all(), f"shard {r}: {side} gap/uid"
                assert (getattr(got.topos, "real_off" if side == "realised" else "des_off") == off).all()
            eng.run()
            eng.sync()
            out = eng.download()
            mine = per_topology(got, out)            # peers: document indices already
            bad = np.nonzero((mine != ref[keep]).any(axis=1))[0]
            assert len(bad) == 0, f"shard {r}: {len(bad)} topologies differ, first doc index {keep[bad[0]]}"
            seen[keep] += 1
        assert (seen == 1).all()
    finally:
        eng.close()


def test_sharded_ingest_rank_setup_ends_with_next_ingest():
    """A sharded ingest leaves the context as rank r of G for its own epoch only: the next
    plain ingest (or upload) restores the single-shard setup, so it decodes the whole
    document and the VXLAN apply (single-shard contexts) works again."""
    from kdtn import Engine, synth
    inp = synth.make(1)
    doc = synth.topology_list_json(inp)
    eng = Engine(device=0, tick_in_usec=TICK)
    try:
        info = eng.ingest(doc, shard=(2, 1))
        assert info.n_topos < inp.topos.n
        info = eng.ingest(doc)
        assert info.n_topos == inp.topos.n
        assert (eng.ingest_doc_index() == np.arange(inp.topos.n)).all()
        eng.run()
        eng.sync()
        eng.vni_apply()
        eng.ingest(doc, shard=(2, 0))
        eng.upload(inp)                         # a plain upload after a sharded ingest
        eng.run()
        eng.sync()
        assert len(eng.download().upd_idx) == inp.desired.n
    finally:
        eng.close()
