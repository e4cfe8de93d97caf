"""kdtn_epoch_vni_apply on the GPU against the oracle (or_vni_apply, pinned by
tests/test_vni_state_cpu.py): the VxlanManager maps after each epoch's reached entries,
bit-exact including order, and the resident map carried into the next epoch
(KDTN_VNI_RESIDENT) giving the same batches as the oracle fed the applied map."""
import numpy as np
import pytest

from helpers import random_epoch_input
from kdtn import Engine, synth
from kdtn.engine import KdtnError
from kdtn.tables import Vnis

import oracle as O

pytestmark = pytest.mark.gpu


def same(a, b):
    return all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(a, b)) and len(a[0]) == len(b[0])


@pytest.mark.parametrize("seed", range(8))
def test_vni_apply_random_epochs(seed):
    _, inp = random_epoch_input(seed, T=96)
    want_out = O.reconcile(inp, tick=15.625)
    want = O.vni_apply(inp, want_out)
    with Engine(device=0, tick_in_usec=15.625) as eng:
        got_out = eng.reconcile(inp)
        assert not got_out.mismatches(want_out)
        got = eng.vni_apply()
        assert same((got.node, got.vni, got.net_ns), want)
        assert np.array_equal(eng.vni_download().node, want[0])
        # the keys whose result depends on the reference's goroutine order (kdtn_vni_contested)
        assert same(eng.vni_contested(), O.vni_contested(inp, want_out))


@pytest.mark.parametrize("config", [3, 4])
def test_vni_resident_chain(config):
    """Three epochs; each uploads KDTN_VNI_RESIDENT after the first, so the engine decides
    vni_hit against the map its own apply left. Config 3: churn epochs (deletes hit the map
    the adds of earlier epochs wrote); config 4: the WAN twin re-reconciled on its applied map."""
    with Engine(device=0, tick_in_usec=15.625) as eng:
        cs = synth.ChurnSequence(total_pods=4000) if config == 3 else None
        inp = cs.epoch_input() if cs else synth.make(4, total_pods=3000)
        vn = None
        hits = 0
        for ep in range(3):
            oin = inp
            if vn is not None:
                oin.vnis = vn                                     # the oracle's own chain
            want_out = O.reconcile(oin, tick=15.625)
            if ep == 0:
                eng.upload(inp)
            else:
                keep = inp.vnis
                inp.vnis = Vnis.keep_resident()
                eng.upload(inp, kd_keep)                       # the map's ids: a kept prefix
                inp.vnis = keep
            kd_keep = inp.kdict.n
            eng.run()
            eng.sync()
            got_out = eng.download()
            bad = got_out.mismatches(want_out)
            assert not bad, f"epoch {ep}: {bad}"
            hits += int(want_out.del_res["vni_hit"].sum()) + int(want_out.add_res["vni_hit"].sum())
            want = O.vni_apply(oin, want_out)
            got = eng.vni_apply()
            assert same((got.node, got.vni, got.net_ns), want), f"epoch {ep}: map differs"
            assert same(eng.vni_contested(), O.vni_contested(oin, want_out)), f"epoch {ep}: contested keys differ"
            vn = Vnis(*[np.array(a, copy=True) for a in want])
            if cs:
                cs.advance()
                inp = cs.epoch_input()
        assert hits > 0


def test_rerun_after_apply_keeps_epoch_start_snapshot():
    """run → vni_apply → run on one upload: the second run decides vni_hit against the same
    epoch-start snapshot (identical outputs), a second apply gives the same map, and the
    next upload with KDTN_VNI_RESIDENT starts from the applied map."""
    inp = synth.make(4, total_pods=3000)
    want_out = O.reconcile(inp, tick=15.625)
    want = O.vni_apply(inp, want_out)
    with Engine(device=0, tick_in_usec=15.625) as eng:
        eng.upload(inp)
        eng.run()
        eng.sync()
        first = eng.download()
        assert not first.mismatches(want_out)
        got = eng.vni_apply()
        assert same((got.node, got.vni, got.net_ns), want)
        eng.run()
        eng.sync()
        assert not eng.download().mismatches(want_out), "re-run saw the applied map"
        got2 = eng.vni_apply()
        assert same((got2.node, got2.vni, got2.net_ns), want)
        keep = inp.vnis
        inp.vnis = Vnis.keep_resident()
        eng.upload(inp, inp.kdict.n)
        inp.vnis = Vnis(*[np.array(a, copy=True) for a in want])
        next_want = O.reconcile(inp, tick=15.625)
        inp.vnis = keep
        eng.run()
        eng.sync()
        assert not eng.download().mismatches(next_want)


def test_resident_map_needs_kept_dictionary():
    """KDTN_VNI_RESIDENT is refused when the upload does not keep the dictionary the map's ids
    were made for, and always for a JSON ingest (its dictionary is the engine's own)."""
    from kdtn import KdtnError, abi
    inp = synth.make(4, total_pods=2000)
    with Engine(device=0, tick_in_usec=15.625) as eng:
        eng.reconcile(inp)
        eng.vni_apply()
        keep = inp.vnis
        inp.vnis = Vnis.keep_resident()
        try:
            with pytest.raises(KdtnError) as e:
                eng.upload(inp)                                # kdict_keep = 0
            assert e.value.code == abi.EINVAL
            with pytest.raises(KdtnError) as e:
                eng.ingest(synth.topology_list_json(synth.make(1)), vnis=Vnis.keep_resident())
            assert e.value.code == abi.EINVAL
        finally:
            inp.vnis = keep


def test_vni_contested_counts_random_epochs():
    """kdtn_vni_contested over adversarial epochs (VNI collisions, deletes of stored keys) equals
    the oracle, and the epochs do produce contested keys; KDTN_EINVAL before an apply."""
    total = 0
    with Engine(device=0, tick_in_usec=15.625) as eng:
        for seed in range(16):
            _, inp = random_epoch_input(seed, T=80)
            want_out = O.reconcile(inp, tick=15.625)
            got_out = eng.reconcile(inp)
            assert not got_out.mismatches(want_out)
            with pytest.raises(KdtnError):
                eng.vni_contested()                      # no apply since this run
            eng.vni_apply()
            want = O.vni_contested(inp, want_out)
            assert same(eng.vni_contested(), want), seed
            total += len(want[0])
    assert total > 0
