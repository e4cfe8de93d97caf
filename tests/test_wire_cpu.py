"""CPU: the wire-encoding oracle (oracle/kdtn_oracle_wire.c, proto.Marshal of the
LinksBatchQuery requests Reconcile sends) against the Python protobuf runtime and the
committed golden fixtures (tests/golden/wire.json, tests/golden/make_wire_golden.py)."""
import json
import os

import numpy as np
import pytest

import oracle as O
import wire_pb
from helpers import golden_epoch, wire_epoch_input
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
