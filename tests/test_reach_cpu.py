"""CPU (oracle): which batch entries the daemons reach, and what that means for the
RemotePod fan-out and the `tc` argv (include/kdtn.h "which batch entries the daemons reach").

Reconcile sends DelLinks, AddLinks, UpdateLinks and stops at the first failed RPC
(controllers/topology_controller.go:93-116); each daemon handler stops at its first failing
link (daemon/kubedtn/handler.go:601-607, 622-628, 644-662). A cross-node link whose
RemotePod the peer rejects (link.PeerIp set but not a CIDR: vxlan.go:80-83 on the peer)
fails after its own local steps (handler.go:448-451). A same-node veth pair gets its
qdiscs on both ends (common/veth.go:53-60)."""
import numpy as np

import oracle as O
from kdtn import abi
from kdtn.model import Link, LinkProperties, Topology, pack

TBF = LinkProperties(rate="1Gbit")


def scenario():
    a_links = [Link("eth0", "10.1.0.1/31", "", "eth9", "10.1.0.0/31", "", "b", 1, TBF),   # same node
               Link("eth1", "10.1.0.3/31", "", "eth8", "10.0.0.9", "", "c", 2, TBF),      # remote rejects
               Link("eth2", "10.1.0.5/31", "", "eth7", "10.1.0.4/31", "", "c", 3, TBF)]   # never reached
    d_old = [Link("eth0", "bad-ip", "", "eth0", "", "", "c", 10)]                           # delLink fails
    d_new = [Link("eth1", "10.2.0.1/31", "", "eth1", "10.2.0.0/31", "", "c", 11, TBF)]
    e_old = [Link(f"eth{u}", "10.3.0.1/31" if u != 21 else "nope", "", "eth0", "", "", "c", u)
             for u in (20, 21, 22)]
    e_new = [Link(**{**l.__dict__, "properties": TBF}) for l in e_old]
    return [Topology("a", "default", a_links, [], "10.0.0.1", "/ns/a"),
            Topology("b", "default", [], [], "10.0.0.1", "/ns/b"),
            Topology("c", "default", [], [], "10.0.0.2", "/ns/c"),
            Topology("d", "default", d_new, d_old, "10.0.0.1", "/ns/d"),
            Topology("e", "default", e_new, e_old, "10.0.0.1", "/ns/e")]


def test_reach_rule_fanout_and_tc():
    topos = scenario()
    inp = pack(topos)
    out = O.reconcile(inp, tick=15.625)
    a0 = out.add_off[0]
    assert list(out.add_res["kind"][a0:a0 + 3]) == [abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_CROSS_NODE]
    assert list(out.add_res["remote_err"][a0:a0 + 3]) == [0, abi.E_REMOTE_CIDR, 0]
    assert out.del_res["err"][out.del_off[3]] == abi.E_VETH_CIDR
    # fan-out: a's second link sends its RemotePod (then the batch aborts); d's add is never sent
    node, off, idx = O.fanout(out, inp.topos.n)
    assert len(node) == 1 and list(idx) == [a0 + 1]
    # tc: a.0 on both veth ends, a.1 locally, e's first update only
    arena, off = O.tc_epoch(inp, out)
    na = len(out.add_idx)
    cmds = {g: arena[int(off[g]):int(off[g + 1])].tobytes().split(b"\0")[3]
            for g in range(len(off) - 1) if off[g + 1] > off[g]}
    u0 = 2 * na + out.upd_off[4]
    assert cmds == {2 * a0: b"eth0", 2 * a0 + 1: b"eth9", 2 * a0 + 2: b"eth1", u0: b"eth20"}, cmds


def test_kubedtn_add_links_stops_at_remote_rejection():
    """model.KubeDTN.add_links' outcome counts the peer's rejection as the link's error."""
    res = np.zeros(3, abi.RESOLVED_DTYPE)
    res["kind"] = abi.KIND_CROSS_NODE
    res["remote_err"][1] = abi.E_REMOTE_CIDR
    q = np.zeros(3, abi.QDISC_DTYPE)
    from kdtn.model import KubeDTN
    errs = np.where(res["err"] != 0, res["err"], q["err"])
    errs = np.where(errs != 0, errs, res["remote_err"])
    out = KubeDTN._outcome(res, errs, q)
    assert not out.response and out.first_failed == 1 and out.err == abi.E_REMOTE_CIDR


def test_oracle_adversarial_epochs_run_clean():
    """The oracle over adversarial random epochs (duplicates, nil vs empty, invalid strings,
    >CAP hubs): reconcile, fan-out, tc argv and wire encoding complete with consistent sizes
    (this file also runs under ASan/UBSan, tests/test_oracle_sanitizers.py)."""
    from helpers import random_epoch_input, wire_epoch_input
    for seed in range(4):
        _, inp = random_epoch_input(seed, T=60, big=1 if seed == 3 else 0, p_err=0.3)
        out = O.reconcile(inp, tick=15.625)
        assert out.add_off[-1] == len(out.add_idx) and out.del_off[-1] == len(out.del_idx)
        node, off, idx = O.fanout(out, inp.topos.n)
        assert off[-1] == len(idx)
        arena, toff = O.tc_epoch(inp, out)
        assert toff[-1] == len(arena) and len(toff) == 2 * len(out.add_idx) + len(out.upd_idx) + 1
        _, winp = wire_epoch_input(seed, T=40)
        wout = O.reconcile(winp)
        a, woff, err = O.encode_epoch(winp, wout)
        assert int(woff[-1]) == len(a)
