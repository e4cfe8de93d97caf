"""Resident epoch state on the GPU: kdtn_epoch_commit (Status.Links = Spec.Links for the
committed Topologies, controllers/topology_controller.go:125-138) and kdtn_epoch_upload_delta
(only the changed Topologies' specs, as references into the previous desired store plus
inline records) against the host restatement (tests/state.py), and every epoch of a
resident chain bit-exact against the oracle on the tables the chain should hold."""
import copy

import numpy as np
import pytest

import oracle as O
from helpers import random_epoch
from kdtn import Engine, abi, synth
from kdtn.delta import build_delta
from kdtn.engine import pin_delta
from kdtn.model import pack
from kdtn.tables import EpochInput, Interner, Links, StrTab, Topos
from state import apply_delta, commit, predicted_commit, same_tables
from test_state_cpu import mutate

pytestmark = pytest.mark.gpu
TICK = 15.625


def _run_same(eng, expect, ctx):
    eng.run()
    eng.sync()
    out = eng.download()
    ora = O.reconcile(expect, tick=TICK)
    bad = out.mismatches(ora)
    assert not bad, f"{ctx}: {bad}"
    return ora


def _outputs_same(eng, expect, ctx):
    """The output stages on the resident state (the encoders' string tables built only for the
    strings the delta appended) equal the oracle's on the tables the state should hold."""
    out = eng.download()
    ora = O.reconcile(expect, tick=TICK)
    n = eng.encode()
    arena, off, err = eng.download_wire()
    want_a, want_off, want_err = O.encode_epoch(expect, out)
    assert n == len(want_a) and np.array_equal(off, want_off), ctx
    assert np.array_equal(err, want_err.astype(np.uint32)) and arena.tobytes() == want_a.tobytes(), ctx
    got = eng.remote_pods()
    want = O.remote_epoch(expect, ora)
    for name, g, w in zip(("arena", "off", "entry", "n_remote", "tc", "tc_off"), got, want):
        assert np.array_equal(np.asarray(g), np.asarray(w)), (ctx, name)
    ta, to = eng.tc_argv(len(out.add_idx), len(out.upd_idx))
    wa, wo = O.tc_epoch(expect, ora)
    assert np.array_equal(to, wo) and ta.tobytes() == wa.tobytes(), ctx


def test_commit_and_delta_random_epochs():
    """Adversarial epochs (failing links, nil lists, SKIP / CREATED / DIFF): the predicted
    commit and explicit masks, then a delta with spec edits, nil specs and node moves."""
    for seed in range(4):
        topos, vnis = random_epoch(seed, T=150, p_err=0.2)
        kd, pd = Interner(), Interner()
        a = pack(topos, vnis, kdict=kd, pdict=pd)
        with Engine(device=0, tick_in_usec=TICK) as eng:
            eng.upload(a)
            ora = _run_same(eng, a, f"seed {seed} epoch 0")
            if seed % 2 == 0:
                mask = predicted_commit(a, ora)
                n = eng.commit()
            else:
                mask = np.random.default_rng(seed).random(a.topos.n) < 0.6
                n = eng.commit(mask)
            assert n == int(mask.sum())
            state = commit(a, mask)
            assert not same_tables(eng.tables(), state), seed
            b = pack(mutate(topos, seed + 7), vnis, kdict=kd, pdict=pd)
            d = build_delta(a, b, a.kdict.n, a.pdict.n, vnis=b.vnis)
            eng.upload_delta(d)
            want = apply_delta(state, d)
            assert not same_tables(eng.tables(), want), seed
            eng.run()
            eng.sync()
            kt = eng.kernel_times()          # the pod tables were patched by the delta: no rebuild
            assert "full_prefix" in kt and "verify_prefix" not in kt, kt
            _run_same(eng, want, f"seed {seed} epoch 1")
            _outputs_same(eng, want, f"seed {seed} epoch 1")
            # a further delta on the patched tables (rows moving again)
            c = mutate(b_topos := mutate(topos, seed + 7), seed + 11)
            st2 = commit(want, predicted_commit(want, O.reconcile(want, tick=TICK)))
            eng.commit()
            c_in = pack(c, vnis, kdict=kd, pdict=pd)
            d2 = build_delta(b, c_in, b.kdict.n, b.pdict.n, vnis=c_in.vnis)
            eng.upload_delta(d2)
            w2 = apply_delta(st2, d2)
            _run_same(eng, w2, f"seed {seed} epoch 2")
            _outputs_same(eng, w2, f"seed {seed} epoch 2")


@pytest.mark.parametrize("pods", [20000])
def test_resident_churn_chain(pods):
    """Ten config-3 churn epochs through one context: after each epoch the status commit
    (alternately the engine's prediction and an all-succeeded mask) and a delta upload of the
    next epoch; the device tables equal the restatement's and every epoch's batches equal
    the oracle's on those tables."""
    cs = synth.ChurnSequence(total_pods=pods)
    prev = cs.epoch_input(copy=True)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(prev)
        ora = _run_same(eng, prev, "epoch 0")
        state = prev
        moved = 0
        for ep in range(1, 10):
            if ep % 2:
                mask = predicted_commit(state, ora)
                assert eng.commit() == int(mask.sum())
            else:
                mask = np.ones(state.topos.n, bool)
                eng.commit(mask)
            state = commit(state, mask)
            cs.advance()
            new = cs.epoch_input(copy=True)
            d = build_delta(state, new, state.kdict.n, state.pdict.n)
            moved += d.upload_bytes()
            eng.upload_delta(pin_delta(d) if ep % 2 else d)      # (one host block: merged copies)
            state = apply_delta(state, d)
            assert not same_tables(eng.tables(), state), ep
            ora = _run_same(eng, state, f"epoch {ep}")
            assert len(ora.del_idx) and len(ora.add_idx) and len(ora.upd_idx)
            if ep in (1, 2, 9):
                _outputs_same(eng, state, f"epoch {ep}")
        full = 9 * (88 * new.desired.n + 25 * new.topos.n)
        assert moved < 0.1 * full, (moved, full)


def test_all_committed_commit_keeps_every_view():
    """kdtn_epoch_commit with every Topology committed takes the fast path (the desired store
    becomes the realised one without reassembly): the tables, a re-run without a new upload,
    a delta upload, a partial commit after it and a full upload all stay exact."""
    topos, vnis = random_epoch(3, T=200, p_err=0.1)
    kd, pd = Interner(), Interner()
    a = pack(topos, vnis, kdict=kd, pdict=pd)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(a)
        _run_same(eng, a, "epoch 0")
        assert eng.commit(np.ones(a.topos.n, bool)) == a.topos.n
        state = commit(a, np.ones(a.topos.n, bool))
        assert not same_tables(eng.tables(), state)
        _run_same(eng, state, "re-run on the committed state")          # status == spec: no diff
        b = pack(mutate(topos, 5), vnis, kdict=kd, pdict=pd)
        d = build_delta(a, b, a.kdict.n, a.pdict.n, vnis=b.vnis)
        eng.upload_delta(d)
        want = apply_delta(state, d)
        assert not same_tables(eng.tables(), want)
        ora = _run_same(eng, want, "delta after the fast commit")
        mask = np.random.default_rng(1).random(want.topos.n) < 0.5
        assert eng.commit(mask) == int(mask.sum())
        st2 = commit(want, mask)
        assert not same_tables(eng.tables(), st2)
        _run_same(eng, st2, "partial commit after the fast one")
        eng.upload(b)
        _run_same(eng, b, "full upload after the commits")


def test_topology_set_churn_chain():
    """Ten config-3 churn epochs with 1 % of the Topologies deleted / re-created per epoch
    (informer delete / add events; CREATED path, controllers/topology_controller.go:81-85)
    through kdtn_epoch_upload_delta: the device tables equal the restatement's — the generator's
    epoch with the status the commits left — and every epoch's batches equal the oracle's on
    those tables; the last epoch also equals a second engine fed by a full upload."""
    from kdtn.delta import record_hash
    tc = synth.TopologySetChurn(frac=0.01, total_pods=20000)
    prev = tc.epoch_input()
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(prev)
        ora = _run_same(eng, prev, "epoch 0")
        state = prev
        for ep in range(1, 10):
            mask = predicted_commit(state, ora) if ep % 2 else np.ones(state.topos.n, bool)
            assert eng.commit(mask if ep % 2 == 0 else None) == int(mask.sum())
            state = commit(state, mask)
            tc.advance()
            new = tc.epoch_input()
            d = build_delta(state, new, state.kdict.n, state.pdict.n)
            assert d.prev is not None and (d.prev == abi.DELTA_NEW).any()
            eng.upload_delta(d)
            state = apply_delta(state, d)
            assert np.array_equal(record_hash(state.desired), record_hash(new.desired))
            assert np.array_equal(state.topos.name, new.topos.name)
            assert not same_tables(eng.tables(), state), ep
            ora = _run_same(eng, state, f"epoch {ep}")
            created = d.prev[d.topo] == abi.DELTA_NEW
            assert (ora.action[d.topo[created]] == abi.ACT_CREATED).all()
    with Engine(device=0, tick_in_usec=TICK) as full:
        full.upload(state)
        _run_same(full, state, "full upload of the last epoch")


def test_delta_rejections_leave_the_state():
    """A delta the engine refuses (kept dictionary not the resident one, references / inline
    ids / topology map out of range, a created Topology without a spec) returns KDTN_EINVAL
    and leaves the resident state: the tables, a run on them, and the corrected delta after."""
    import dataclasses
    from kdtn.engine import KdtnError
    topos, vnis = random_epoch(5, T=120, p_err=0.1)
    kd, pd = Interner(), Interner()
    a = pack(topos, vnis, kdict=kd, pdict=pd)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(a)
        _run_same(eng, a, "epoch 0")
        eng.commit(np.ones(a.topos.n, bool))
        state = commit(a, np.ones(a.topos.n, bool))
        b = pack(mutate(topos, 9), vnis, kdict=kd, pdict=pd)
        good = build_delta(a, b, a.kdict.n, a.pdict.n, vnis=b.vnis)
        assert good.n_changed > 2 and good.records.n > 0 and len(good.ref) > 0
        R = dataclasses.replace
        kb, ko = good.kdict.bytes_, good.kdict.offs
        strs = [bytes(kb[ko[i]:ko[i + 1]]) for i in range(good.kdict.n)]
        strs[1] += b"-longer"                 # same string count, the kept prefix ends elsewhere
        bads = {"shrunk kept dictionary": R(good, kdict_keep=a.kdict.n - 1),
                "kept prefix at another offset": R(good, kdict=StrTab.from_list(strs)),
                "ref out of range": R(good, ref=np.where(np.arange(len(good.ref)) == len(good.ref) - 1,
                                                        np.uint32(a.desired.n + 7), good.ref).astype(np.uint32)),
                # far outside any allocation: the GPU checks must stop every later kernel
                "ref far out of range": R(good, ref=np.full(len(good.ref), 0x7FFFFFF0, np.uint32)),
                "inline ref far out of range": R(good, ref=np.full(len(good.ref), abi.DELTA_NEW | 0x7FFFFFF,
                                                                   np.uint32)),
                "topo far out of range": R(good, topo=np.full(good.n_changed, 0x7FFFFFF0, np.uint32)),
                "topo not ascending": R(good, topo=good.topo[::-1].copy()),
                "inline id out of range": R(good, records=dataclasses.replace(
                    good.records, key=np.where(np.arange(good.records.n) == 0, np.uint32(b.kdict.n + 3),
                                               good.records.key).astype(np.uint32))),
                "prev named twice": R(good, prev=np.r_[0, np.arange(a.topos.n - 1)].astype(np.uint32),
                                      ns=b.topos.ns[good.topo], name=b.topos.name[good.topo]),
                "created without spec": R(good, prev=np.r_[np.arange(a.topos.n), abi.DELTA_NEW].astype(np.uint32),
                                          ns=b.topos.ns[good.topo], name=b.topos.name[good.topo])}
        for what, d in bads.items():
            with pytest.raises(KdtnError) as e:
                eng.upload_delta(d)
            assert e.value.code == abi.EINVAL, what
            assert not same_tables(eng.tables(), state), what
            _run_same(eng, state, f"after a rejected delta ({what})")
        eng.upload_delta(good)
        _run_same(eng, apply_delta(state, good), "the corrected delta")


def test_delta_inline_record_referenced_twice():
    """An inline record referenced by several entries (allowed by the ABI: references are
    free-form) is placed at every position (the general placement path), and a record no
    entry references is ignored."""
    import dataclasses
    topos, vnis = random_epoch(8, T=150, p_err=0.1)
    kd, pd = Interner(), Interner()
    a = pack(topos, vnis, kdict=kd, pdict=pd)
    b = pack(mutate(topos, 21), vnis, kdict=kd, pdict=pd)
    good = build_delta(a, b, a.kdict.n, a.pdict.n, vnis=b.vnis)
    new_at = np.nonzero(good.ref & abi.DELTA_NEW)[0]
    assert len(new_at) >= 3
    ref = good.ref.copy()
    ref[new_at[1]] = ref[new_at[0]]           # record of new_at[1] now unreferenced, new_at[0]'s twice
    ref[new_at[2]] = ref[new_at[0]]
    d = dataclasses.replace(good, ref=ref)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(a)
        _run_same(eng, a, "epoch 0")
        eng.commit(np.ones(a.topos.n, bool))
        state = commit(a, np.ones(a.topos.n, bool))
        eng.upload_delta(d)
        want = apply_delta(state, d)
        assert not same_tables(eng.tables(), want)
        _run_same(eng, want, "inline record referenced three times")


def test_async_download_pipelined_chain():
    """kdtn_epoch_download_async overlapping the next delta upload: every epoch's outputs, read
    after download_wait, equal the oracle's, while the next epoch's upload and run go on."""
    from kdtn.tables import BatchesOut
    cs = synth.ChurnSequence(total_pods=5000)
    prev = cs.epoch_input(copy=True)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(prev)
        eng.run()
        eng.sync()
        T = prev.topos.n
        bufs = [BatchesOut.alloc(T, prev.desired.n, prev.desired.n, prev.desired.n, pinned=True) for _ in range(2)]
        pend = (eng.download_async(bufs[0]), O.reconcile(prev, tick=TICK))
        eng.commit(np.ones(T, np.uint8))
        state = commit(prev, np.ones(T, bool))
        for ep in range(1, 6):
            cs.advance()
            new = cs.epoch_input(copy=True)
            d = build_delta(state, new, state.kdict.n, state.pdict.n)
            eng.upload_delta(d)                   # beside the previous epoch's copies
            state = apply_delta(state, d)
            eng.run()
            eng.sync()
            eng.download_wait()
            got, want = pend
            assert not got.mismatches(want), f"epoch {ep - 1}: {got.mismatches(want)}"
            pend = (eng.download_async(bufs[ep % 2]), O.reconcile(state, tick=TICK))
            eng.commit(np.ones(T, np.uint8))
            state = commit(state, np.ones(T, bool))
        eng.download_wait()
        got, want = pend
        assert not got.mismatches(want)


class _ScatteredLinks(Links):
    """The same records with no two columns adjacent in host memory (each id column, the gap
    and the uid in one buffer, in reverse column order with a gap between them), so a delta
    upload copies every column on its own and places each as it arrives."""

    def to_c(self) -> abi.LinkTable:
        n = self.n
        w = n + 16
        buf = np.zeros((abi.NKEY + abi.NPROP + 1) * w, np.uint32)
        cols = [self.key[k] for k in range(abi.NKEY)] + [self.prop[k] for k in range(abi.NPROP)] + [self.gap]
        views = []
        for c, a in enumerate(cols):
            at = (len(cols) - 1 - c) * w
            buf[at:at + n] = a
            views.append(buf[at:at + n])
        self._buf, self._uid = buf, np.array(self.uid, np.int64)
        t = abi.LinkTable()
        t.n = n
        for k in range(abi.NKEY):
            t.key[k] = abi.ptr(views[k], abi.u32p)
        for k in range(abi.NPROP):
            t.prop[k] = abi.ptr(views[abi.NKEY + k], abi.u32p)
        t.gap = abi.ptr(views[-1], abi.u32p)
        t.uid = abi.ptr(self._uid, abi.i64p)
        return t


def test_delta_records_in_separate_columns():
    """Churn epochs whose inline records come as 20 separate column arrays (plus the uid): every
    column is its own copy and its own placement launch; tables and batches stay exact."""
    cs = synth.ChurnSequence(total_pods=20000)
    prev = cs.epoch_input(copy=True)
    with Engine(device=0, tick_in_usec=TICK) as eng:
        eng.upload(prev)
        _run_same(eng, prev, "epoch 0")
        state = prev
        for ep in range(1, 5):
            eng.commit(np.ones(state.topos.n, bool))
            state = commit(state, np.ones(state.topos.n, bool))
            cs.advance()
            new = cs.epoch_input(copy=True)
            d = build_delta(state, new, state.kdict.n, state.pdict.n)
            r = d.records
            if ep % 2:
                d = copy.copy(d)
                d.records = _ScatteredLinks(r.key, r.uid, r.prop, r.gap)
            eng.upload_delta(d)
            state = apply_delta(state, d)
            assert not same_tables(eng.tables(), state), ep
            _run_same(eng, state, f"epoch {ep} ({'separate' if ep % 2 else 'adjacent'} columns)")
