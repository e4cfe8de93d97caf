"""Incremental CR ingest on the resident state (kdtn_json_ingest_delta): the informer's added /
updated Topology CRs as a TopologyList document plus the deleted rows, decoded on the GPU and
interned into the resident dictionaries (daemon/kubedtn/kubedtn.go:128-142 event stream;
controllers/topology_controller.go:81-85 for created CRs). A JSON-driven chain of config-3
churn epochs with Topologies created and deleted is compared, epoch by epoch, with the host
delta chain (kdtn_epoch_upload_delta over the generator's tables, tests/state.py restatement):
the same CRs with the same status and spec, id-free and order-free, and every epoch's
batches equal the oracle's on the engine's own tables."""
import copy
import json

import numpy as np
import pytest

import oracle as O
from kdtn import Engine, abi, synth
from kdtn.delta import build_delta
from kdtn.engine import KdtnError
from state import apply_delta, commit

pytestmark = pytest.mark.gpu
TICK = 15.625


def canon(inp):
    """The epoch as strings, Topologies sorted by (namespace, name): rows and both link
    segments — equal for two engines that hold the same CRs under different ids / orders."""
    K = np.empty(inp.kdict.n, dtype=object)
    K[:] = [inp.kdict.get(i) for i in range(inp.kdict.n)]
    P = np.empty(inp.pdict.n, dtype=object)
    P[:] = [inp.pdict.get(i) for i in range(inp.pdict.n)]
    T = inp.topos
    order = np.array(sorted(range(T.n), key=lambda t: (K[T.ns[t]], K[T.name[t]])), dtype=np.int64)

    def side(off, L):
        off = off.astype(np.int64)
        lens = off[order + 1] - off[order]
        idx = (np.repeat(off[order], lens) + np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens)
               if len(order) else np.zeros(0, np.int64))
        return [lens, K[L.key[:, idx]] if L.n else np.zeros(0), P[L.prop[:, idx]] if L.n else np.zeros(0),
                L.uid[idx], L.gap[idx]]

    rows = [K[T.ns[order]], K[T.name[order]], K[T.src_ip[order]], K[T.net_ns[order]], T.flags[order]]
    return rows + side(T.des_off, inp.desired) + side(T.real_off, inp.realised)


def same_canon(a, b):
    for i, (x, y) in enumerate(zip(canon(a), canon(b))):
        if x.shape != y.shape or not np.array_equal(x, y):
            return f"part {i} differs"
    return None


def key_rows(inp):
    kd = inp.kdict
    return {(kd.get(int(inp.topos.ns[t])), kd.get(int(inp.topos.name[t]))): t for t in range(inp.topos.n)}


def run_vs_oracle(eng, ctx):
    tables = eng.tables()
    eng.run()
    eng.sync()
    out = eng.download()
    bad = out.mismatches(O.reconcile(tables, tick=TICK))
    assert not bad, f"{ctx}: {bad}"
    return tables


def test_json_driven_resident_chain():
    tc = synth.TopologySetChurn(frac=0.01, total_pods=20000)
    prev = tc.epoch_input()
    with Engine(device=0, tick_in_usec=TICK) as ej, Engine(device=0, tick_in_usec=TICK) as eh:
        ej.ingest(synth.topology_list_json(prev))
        eh.upload(prev)
        tj = run_vs_oracle(ej, "JSON chain epoch 0")
        run_vs_oracle(eh, "host chain epoch 0")
        assert same_canon(tj, prev) is None
        state = prev
        for ep in range(1, 10):
            ej.commit(np.ones(ej.state_sizes().n_topos, np.uint8))
            eh.commit(np.ones(state.topos.n, np.uint8))
            state = commit(state, np.ones(state.topos.n, bool))
            tc.advance()
            new = tc.epoch_input()
            d = build_delta(state, new, state.kdict.n, state.pdict.n)
            eh.upload_delta(d)
            state = apply_delta(state, d)
            # the informer's events: the changed / created CRs, the rows of the deleted ones
            sel = np.zeros(new.topos.n, bool)
            sel[d.topo] = True
            doc = synth.topology_list_json(synth.select_topologies(new, sel))
            rows = key_rows(ej.tables())
            gone = set(rows) - set(key_rows(new))
            kd_before = ej.tables().kdict
            info = ej.ingest_delta(doc, deleted=np.array(sorted(rows[k] for k in gone), np.uint32))
            tj = ej.tables()
            assert info.n_topos == new.topos.n
            why = same_canon(tj, state)
            assert why is None, f"epoch {ep}: JSON chain and host chain differ ({why})"
            # resident ids stay: the dictionaries only grow
            n0 = kd_before.n
            assert np.array_equal(tj.kdict.offs[:n0 + 1], kd_before.offs)
            assert tj.kdict.bytes_[:len(kd_before.bytes_)].tobytes() == kd_before.bytes_.tobytes()
            run_vs_oracle(ej, f"JSON chain epoch {ep}")
            run_vs_oracle(eh, f"host chain epoch {ep}")


def test_ingest_delta_rejections_leave_the_state():
    """A TopologyList that lists a CR twice, a deleted row that is also listed or out of range,
    and a malformed document are refused; the resident state stays and a correct delta after
    them applies."""
    tc = synth.TopologySetChurn(frac=0.02, total_pods=3000)
    prev = tc.epoch_input()
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.ingest(synth.topology_list_json(prev))
        t0 = run_vs_oracle(eng, "epoch 0")
        one = np.zeros(prev.topos.n, bool)
        one[[3, 7]] = True
        part = synth.topology_list_json(synth.select_topologies(prev, one))
        dup_doc = synth.topology_list_json(synth.select_topologies(prev, np.array([3, 7, 3])))
        rows = key_rows(t0)
        k3 = (prev.kdict.get(int(prev.topos.ns[3])), prev.kdict.get(int(prev.topos.name[3])))
        # a CR the state does not hold yet (an informer add and update batched together)
        doc = json.loads(synth.topology_list_json(synth.select_topologies(prev, np.array([3]))))
        doc["items"][0]["metadata"]["name"] = "created-twice"
        doc["items"].append(copy.deepcopy(doc["items"][0]))
        new_dup_doc = json.dumps(doc).encode()
        cases = [("listed twice", dup_doc, [], abi.EINVAL),
                 ("created twice", new_dup_doc, [], abi.EINVAL),
                 ("deleted and listed", part, [rows[k3]], abi.EINVAL),
                 ("deleted out of range", part, [prev.topos.n + 5], abi.EINVAL),
                 ("malformed document", part[:-3], [], abi.EBADMSG)]
        for what, doc, dele, code in cases:
            with pytest.raises(KdtnError) as e:
                eng.ingest_delta(doc, deleted=np.array(dele, np.uint32))
            assert e.value.code == code, what
            assert same_canon(eng.tables(), t0) is None, what
            run_vs_oracle(eng, f"after a refused ingest ({what})")
        info = eng.ingest_delta(part, deleted=np.array([0], np.uint32))
        assert info.n_topos == prev.topos.n - 1
        run_vs_oracle(eng, "a correct incremental ingest after the refusals")
