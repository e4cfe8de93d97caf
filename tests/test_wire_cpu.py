"""CPU: the wire-encoding oracle (oracle/kdtn_oracle_wire.c, proto.Marshal of the
LinksBatchQuery requests Reconcile sends) against the Python protobuf runtime and the
committed golden fixtures (tests/golden/wire.json, tests/golden/make_wire_golden.py)."""
import json
import os

import numpy as np
import pytest

import oracle as O
import wire_pb
from helpers import golden_epoch, random_epoch_input, wire_epoch_input
from kdtn import abi
from kdtn.model import pack

HERE = os.path.dirname(os.path.abspath(__file__))


def _check_epoch(inp, out):
    arena, off, err = O.encode_epoch(inp, out)
    T = inp.topos.n
    want = wire_pb.epoch_bytes(inp, out)
    n_err = n_msg = 0
    for (lst, t), w in want.items():
        a, b = int(off[lst * T + t]), int(off[lst * T + t + 1])
        if w is None:
            assert err[t] >> lst & 1 and a == b, (lst, t)
            n_err += 1
        else:
            assert not err[t] >> lst & 1, (lst, t)
            assert arena[a:b].tobytes() == w, (lst, t)
            n_msg += bool(w)
    return n_msg, n_err


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_protobuf_runtime(seed):
    topos, inp = wire_epoch_input(seed)
    n_msg, n_err = _check_epoch(inp, O.reconcile(inp))
    assert n_msg > 20 and n_err > 0


def test_golden_wire_fixture(golden):
    with open(os.path.join(HERE, "golden", "wire.json")) as f:
        fx = json.load(f)
    for tr in golden["transitions"]:
        inp = pack(golden_epoch(golden, tr))
        out = O.reconcile(inp)
        arena, off, err = O.encode_epoch(inp, out)
        T = inp.topos.n
        got = [arena[int(off[i]):int(off[i + 1])].tobytes().hex() for i in range(3 * T)]
        assert got == fx[tr["name"]]["batches"], tr["name"]
        assert err.tolist() == fx[tr["name"]]["err"]


def test_utf8_validity_edges():
    ok = ["", "a", "µ", "日本", "🙂", b"\xf4\x8f\xbf\xbf", b"\xef\xbf\xbf"]
    bad = [b"\x80", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80",
           b"\xf5\x80\x80\x80", b"\xe2\x82", b"a\xff"]
    assert all(O.utf8_valid(s) for s in ok)
    assert not any(O.utf8_valid(s) for s in bad)


def test_tc_argv_known_answer(golden):
    """SetVethQdiscs' TBF command (common/qdisc.go:252-266) for the bandwidth sample
    (config/samples/tc/bandwidth.yaml: rate "1Gbit" → Rate 1e9, getTbfBurst 4e6)."""
    tr = next(t for t in golden["transitions"] if t["name"] == "S1->S2")
    topos = golden_epoch(golden, tr)
    inp = pack(topos)
    out = O.reconcile(inp)
    arena, off = O.tc_epoch(inp, out)
    cmds = [arena[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
    cmds = [c.split(b"\0")[:-1] for c in cmds if c]
    assert cmds, "the bandwidth transition updates links with a TBF"
    by_rate = {c[10]: c for c in cmds}
    want = [b"qdisc", b"add", b"dev", cmds[0][3], b"parent", b"1:1", b"handle", b"10:0", b"tbf", b"rate",
            b"1000000000", b"burst", b"4000000", b"latency", b"50ms", b"minburst", b"1500"]
    assert by_rate[b"1000000000"][:3] == want[:3] and by_rate[b"1000000000"][4:] == want[4:]
    assert all(len(c) == 17 for c in cmds)


def _check_remote(inp, out):
    """or_remote_epoch against the Python protobuf runtime, message by message; the message
    list = the fan-out's senders, then every reached PHYSICAL add whose MakeVeth passed."""
    arena, off, entry, nr, tc, tc_off = O.remote_epoch(inp, out)
    node, foff, fidx = O.fanout(out, inp.topos.n)
    assert nr == len(fidx) and list(entry[:nr]) == list(fidx)
    T = inp.topos.n
    t_of = np.searchsorted(out.add_off[:T + 1], np.arange(len(out.add_idx)), side="right") - 1
    # reached: no earlier failing entry of the topology's Del → Add sequence (or_reach)
    ok = np.ones(T, bool)
    reached = np.zeros(len(out.add_idx), bool)
    for t in range(T):
        if (out.del_res["err"][out.del_off[t]:out.del_off[t + 1]] != 0).any():
            ok[t] = False
        for e in range(out.add_off[t], out.add_off[t + 1]):
            if not ok[t]:
                break
            reached[e] = True
            r, q = out.add_res[e], out.add_qdisc[e]
            if r["err"] or (r["kind"] in (abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE, abi.KIND_PHYSICAL) and q["err"]) \
                    or r["remote_err"]:
                ok[t] = False
    phys = [e for e in range(len(out.add_idx))
            if reached[e] and out.add_res["kind"][e] == abi.KIND_PHYSICAL and out.add_res["err"][e] == 0]
    assert list(entry[nr:]) == phys
    n_err = 0
    for m, e in enumerate(entry):
        want = wire_pb.remote_pod_bytes(inp, out, int(e), int(t_of[e]), m >= nr, inp.topos.net_ns)
        got = arena[int(off[m]):int(off[m + 1])].tobytes()
        if want is None:
            n_err += 1
            assert got == b"", m
        else:
            assert got == want, m
        cmd = tc[int(tc_off[m]):int(tc_off[m + 1])].tobytes()
        q, r = out.add_qdisc[e], out.add_res[e]
        if m < nr and q["has_tbf"] and not r["remote_err"]:
            j = int(out.add_idx[e])
            args = cmd.split(b"\0")[:-1]
            assert args[:3] == [b"qdisc", b"add", b"dev"] and len(args) == 17
            assert args[3] == inp.kdict.get(int(inp.desired.key[abi.KEY_COLS.index("peer_intf"), j]))
            assert args[10] == str(int(q["tbf_rate"])).encode()
        else:
            assert cmd == b""
    return nr, len(entry) - nr, n_err


def test_remote_pods_match_protobuf_runtime():
    tot = np.zeros(3, int)
    for seed in range(6):
        _, inp = wire_epoch_input(seed)
        tot += _check_remote(inp, O.reconcile(inp))
    for seed in range(4):
        _, inp = random_epoch_input(seed, T=100, p_err=0.05)
        tot += _check_remote(inp, O.reconcile(inp))
    assert tot[0] > 20 and tot[1] > 0, tot


def test_remote_pod_known_answer():
    """A cross-node add from pod a (node 10.0.0.1) to pod b (10.0.0.2), uid 7 → VNI 5007,
    latency 10ms + rate 1Gbit: the RemotePod b's daemon receives, byte for byte."""
    from kdtn.model import Link, LinkProperties, Topology
    props = LinkProperties(latency="10ms", rate="1Gbit")
    a = Topology("a", "ns1", [Link("eth1", "10.9.0.1/31", "", "eth2", "10.9.0.0/31", "", "b", 7, props)], [],
                 "10.0.0.1", "/run/ns/a")
    b = Topology("b", "ns1", [], [], "10.0.0.2", "/run/ns/b")
    inp = pack([a, b])
    out = O.reconcile(inp)
    arena, off, entry, nr, tc, tc_off = O.remote_epoch(inp, out)
    assert nr == 1 and len(entry) == 1
    props_b = b"\x0a\x0410ms" + b"\x32\x051Gbit"
    body = (b"\x0a\x09/run/ns/b" + b"\x12\x04eth2" + b"\x1a\x0b10.9.0.0/31" + b"\x22\x0810.0.0.1" +
            b"\x2a\x03ns1" + b"\x30" + bytes([0x8f, 0x27]) + b"\x3a" + bytes([len(props_b)]) + props_b + b"\x42\x01b")
    assert arena.tobytes() == bytes([len(body)]) + body
    assert tc.tobytes().split(b"\0")[:-1] == [b"qdisc", b"add", b"dev", b"eth2", b"parent", b"1:1", b"handle",
                                               b"10:0", b"tbf", b"rate", b"1000000000", b"burst", b"4000000",
                                               b"latency", b"50ms", b"minburst", b"1500"]


def test_remote_pod_marshal_error_is_empty():
    """A RemotePod with a string that is not valid UTF-8 (here the peer's status.net_ns)
    cannot be marshalled: its message is empty, the others are unaffected."""
    from kdtn.model import Link, LinkProperties, Topology
    a = Topology("a", "ns1", [Link("eth1", "", "", "eth2", "", "", "b", 7, LinkProperties()),
                             Link("eth3", "", "", "eth4", "", "", "c", 8, LinkProperties())], [],
                 "10.0.0.1", "/run/ns/a")
    b = Topology("b", "ns1", [], [], "10.0.0.2", b"/run/\xff")
    c = Topology("c", "ns1", [], [], "10.0.0.3", "/run/ns/c")
    inp = pack([a, b, c])
    out = O.reconcile(inp)
    arena, off, entry, nr, tc, tc_off = O.remote_epoch(inp, out)
    assert nr == 2 and off[1] == off[0] and off[2] > off[1]
    assert _check_remote(inp, out) == (2, 0, 1)
