"""VxlanManager state after an epoch (kdtn_epoch_vni_apply's oracle, or_vni_apply) pinned by
an independent dict-based restatement of the daemons' map mutations:
delLink → Delete(vni) when Get(vni) == local netns (daemon/kubedtn/handler.go:480-487),
cross-node addLink → Store(vni, local netns) (:440) and the peer's Update → Store(vni, peer
netns) (:192; common/utils.go:39-48), physical peer → local Update Store (:348-371); reached
entries only (handler.go:601-607, 622-628; topology_controller.go:93-116). Order: deletes,
then adds, first add of a key wins."""
import numpy as np
import pytest

from helpers import random_epoch_input
from kdtn import abi, synth

import oracle as O


def dict_apply(inp, out):
    T = inp.topos.n
    src, netns = inp.topos.src_ip, inp.topos.net_ns
    snap = {}
    for n, v, s in zip(inp.vnis.node.tolist(), inp.vnis.vni.tolist(), inp.vnis.net_ns.tolist()):
        snap.setdefault((n, v), s)                                  # first entry of a key
    dele, adds = set(), {}

    def fails(r, q):
        if r["err"]:
            return True
        return r["kind"] in (abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL) and q["err"] != 0

    for t in range(T):
        ok = True
        for e in range(out.del_off[t], out.del_off[t + 1]):
            r = out.del_res[e]
            if r["err"]:
                ok = False
                break
            if r["vni_hit"]:
                dele.add((int(src[t]), int(r["vni"])))
        if not ok:
            continue
        for e in range(out.add_off[t], out.add_off[t + 1]):
            r = out.add_res[e]
            if fails(r, out.add_qdisc[e]):
                break
            k = int(r["kind"])
            if k in (abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL):
                adds.setdefault((int(src[t]), int(r["vni"])), int(netns[t]))
            if k == abi.KIND_CROSS_NODE:
                if r["remote_err"]:
                    break
                adds.setdefault((int(r["vtep"]), int(r["vni"])), int(netns[int(r["peer_topo"])]))
    rows = [(n, v, s) for (n, v), s in adds.items()]                 # insertion order
    rows += [(n, v, s) for (n, v), s in snap.items() if (n, v) not in dele and (n, v) not in adds]
    return rows


def as_rows(arrs):
    return list(zip(*(a.tolist() for a in arrs)))


@pytest.mark.parametrize("seed", range(12))
def test_oracle_vni_apply_random_epochs(seed):
    _, inp = random_epoch_input(seed, T=80)
    out = O.reconcile(inp, tick=15.625)
    assert as_rows(O.vni_apply(inp, out)) == dict_apply(inp, out)


def test_oracle_vni_apply_churn_chain():
    """Config-3 churn epochs with the map carried across epochs: deletes start to hit."""
    cs = synth.ChurnSequence(total_pods=3000)
    vn = None
    hits = 0
    for ep in range(3):
        inp = cs.epoch_input()
        if vn is not None:
            inp.vnis = vn
        out = O.reconcile(inp, tick=15.625)
        hits += int(out.del_res["vni_hit"].sum())
        got = O.vni_apply(inp, out)
        assert as_rows(got) == dict_apply(inp, out)
        from kdtn.tables import Vnis
        vn = Vnis(*[np.array(a, copy=True) for a in got])
        cs.advance()
    assert hits > 0


def dict_contested(inp, out):
    """Keys whose result depends on the goroutine order: two Stores of different netns, or a
    Store of the netns a reached delLink of the key compares Get(vni) against."""
    T = inp.topos.n
    src, netns = inp.topos.src_ip, inp.topos.net_ns
    dels, stores = set(), []

    def fails(r, q):
        if r["err"]:
            return True
        return r["kind"] in (abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL) and q["err"] != 0

    for t in range(T):
        ok = True
        for e in range(out.del_off[t], out.del_off[t + 1]):
            r = out.del_res[e]
            if r["err"]:
                ok = False
                break
            dels.add((int(src[t]), int(r["vni"]), int(netns[t])))
        if not ok:
            continue
        for e in range(out.add_off[t], out.add_off[t + 1]):
            r = out.add_res[e]
            if fails(r, out.add_qdisc[e]):
                break
            k = int(r["kind"])
            if k in (abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL):
                stores.append(((int(src[t]), int(r["vni"])), int(netns[t])))
            if k == abi.KIND_CROSS_NODE:
                if r["remote_err"]:
                    break
                stores.append(((int(r["vtep"]), int(r["vni"])), int(netns[int(r["peer_topo"])])))
    first = {}
    for key, ns in stores:
        first.setdefault(key, ns)
    hot = set()
    for key, ns in stores:
        if ns != first[key] or (key[0], key[1], ns) in dels:
            hot.add(key)
    return [k for k in first if k in hot]                 # order of the winning store


def test_oracle_vni_contested_random_epochs():
    total = 0
    for seed in range(16):
        _, inp = random_epoch_input(seed, T=80)
        out = O.reconcile(inp, tick=15.625)
        node, vni = O.vni_contested(inp, out)
        got = list(zip(node.tolist(), vni.tolist()))
        assert got == dict_contested(inp, out), seed
        total += len(got)
    assert total > 0                                      # the adversarial epochs do collide


def test_oracle_vni_contested_churn_chain():
    cs = synth.ChurnSequence(total_pods=3000)
    vn = None
    for ep in range(3):
        inp = cs.epoch_input()
        if vn is not None:
            inp.vnis = vn
        out = O.reconcile(inp, tick=15.625)
        node, vni = O.vni_contested(inp, out)
        assert list(zip(node.tolist(), vni.tolist())) == dict_contested(inp, out)
        from kdtn.tables import Vnis
        vn = Vnis(*[np.array(a, copy=True) for a in O.vni_apply(inp, out)])
        cs.advance()
