"""CPU: pin the oracle (the CPU restatement of the reference path) to the golden vectors.

The reference is Go and cannot be built here; its own tests hold no vectors for this path
(SURVEY §8c). These known answers are hand-derived from the reference sources and its
sample CRs (tests/golden/make_golden.py), plus exact-arithmetic checks of the float32
parse that do not depend on glibc.
"""
import random
from fractions import Fraction

import numpy as np
import pytest

import oracle as O
from helpers import ACTIONS, golden_epoch, midpoint_strings, random_float_strings, uids_by_topology
from kdtn import abi
from kdtn.model import pack


def test_p2u_known_answers(golden):
    for s, want in golden["p2u"].items():
        ok, v = O.parse_pct(s)
        assert ok, s
        assert O.p2u(v) == want, s


def test_vni_and_time2tick_known_answers(golden):
    for uid, want in golden["vni"].items():
        assert O.vni_from_uid(int(uid)) == want
    for t, want in golden["time2tick"].items():
        assert O.time2tick(int(t), golden["tick_in_usec"]) == want


def test_qdisc_known_answers(golden):
    names = [n for n, _ in abi.Qdisc._fields_]
    for case in golden["qdisc"]:
        q = O.make_qdisc(case["props"], golden["tick_in_usec"])
        if "err" in case:
            assert abi.ERR_NAMES[q["err"]] == case["err"], case
            assert q["has_netem"] == 0
            continue
        assert q["err"] == 0, case
        if case.get("has_netem") == 0:
            assert q["has_netem"] == 0 and q["has_tbf"] == 0, case
            continue
        assert q["has_netem"] == 1
        for f in names[:13]:
            assert q[f] == case["netem"].get(f, 0), (case, f)
        if "tbf" in case:
            assert q["has_tbf"] == 1
            assert [q["tbf_rate"], q["tbf_buffer"], q["tbf_minburst"]] == case["tbf"]
        else:
            assert q["has_tbf"] == 0


@pytest.mark.parametrize("idx", range(5))
def test_sample_transitions(golden, idx):
    tr = golden["transitions"][idx]
    topos = golden_epoch(golden, tr)
    out = O.reconcile(pack(topos), tick=golden["tick_in_usec"])
    got = uids_by_topology(topos, out)
    for name, exp in tr["expect"].items():
        assert got[name]["action"] == ACTIONS[exp["action"]], (tr["name"], name)
        for k in ("del", "add", "upd"):
            assert got[name][k] == exp[k], (tr["name"], name, k)


def test_sample_resolve(golden):
    tr = next(t for t in golden["transitions"] if t["name"] == "S0->S0p")
    topos = golden_epoch(golden, tr)
    inp = pack(topos)
    out = O.reconcile(inp, tick=golden["tick_in_usec"])
    add, dl = golden["resolve"]
    r = out.add_res[0]
    assert abi.KIND_CROSS_NODE == r["kind"] and r["vni"] == add["vni"] and r["err"] == 0
    assert inp.kdict.get(int(r["vtep"])).decode() == add["vtep"]
    assert r["peer_topo"] == 2   # r3
    assert out.del_res[0]["vni"] == dl["vni"] and out.del_res[0]["err"] == 0


def test_calc_diff_first_match_and_duplicates():
    """CalcDiff (topology_controller.go:288-318) edge semantics on the oracle."""
    from kdtn.model import Link, LinkProperties, Topology
    a = Link("eth1", "1.1.1.1/24", "", "eth1", "", "", "p", 1)
    a2 = Link("eth1", "1.1.1.1/24", "", "eth1", "", "", "p", 1, LinkProperties(latency="5ms"))
    b = Link("eth2", "", "", "eth2", "", "", "p", 2)
    # old has a duplicate key: both old records match new[0] (first match) → upd twice
    t1 = Topology("x", spec_links=[a2, a], status_links=[a, a])
    # new has duplicate keys; old lacks them → both added
    t2 = Topology("y", spec_links=[b, b], status_links=[a])
    # same records, different order → positional DeepEqual fails, CalcDiff finds nothing
    t3 = Topology("z", spec_links=[b, a], status_links=[a, b])
    # nil vs empty
    t4 = Topology("w", spec_links=[], status_links=None)
    t5 = Topology("v", spec_links=[], status_links=[])
    t6 = Topology("u", spec_links=None, status_links=[a])
    topos = [t1, t2, t3, t4, t5, t6]
    got = uids_by_topology(topos, O.reconcile(pack(topos)))
    assert got["x"] == {"action": abi.ACT_DIFF, "del": [], "add": [], "upd": [1, 1]}
    assert got["y"] == {"action": abi.ACT_DIFF, "del": [1], "add": [2, 2], "upd": []}
    assert got["z"] == {"action": abi.ACT_DIFF, "del": [], "add": [], "upd": []}
    assert got["w"]["action"] == abi.ACT_CREATED
    assert got["v"]["action"] == abi.ACT_SKIP
    assert got["u"] == {"action": abi.ACT_DIFF, "del": [1], "add": [], "upd": []}


def _f32_round(fr: Fraction):
    """Correctly rounded float32 of a rational (exact, ties to even); None on overflow."""
    if fr == 0:
        return 0.0
    neg = fr < 0
    fr = abs(fr)
    x = np.float32(float(fr))   # within 1 ulp
    cands = set()
    for c in (x, np.nextafter(x, np.float32(0)), np.nextafter(x, np.float32(np.inf))):
        cands.add(float(c))
        cands.add(float(np.nextafter(c, np.float32(0))))
        cands.add(float(np.nextafter(c, np.float32(np.inf))))
    cands = sorted(c for c in cands if np.isfinite(c))
    best = min(cands, key=lambda c: (abs(Fraction(c) - fr),
                                     int(np.float32(c).view(np.uint32)) & 1))
    if best > 3.4028234663852886e38:
        return None
    return -best if neg else best


def test_float32_parse_exact_rounding():
    rng = random.Random(7)
    strs = midpoint_strings(rng, 150) + [s for s in random_float_strings(rng, 400)
                                         if "x" not in s.lower() and "_" not in s]
    checked = 0
    for s in strs:
        try:
            fr = Fraction(s)
        except (ValueError, ZeroDivisionError):
            continue
        if abs(fr) > Fraction(10) ** 39 or s.strip() != s:
            continue
        ok, v = O.parse_float32(s)
        want = _f32_round(fr)
        if want is None:
            assert not ok, s
            continue
        assert ok, s
        assert np.float32(v).view(np.uint32) == np.float32(want).view(np.uint32) or (v == 0 and want == 0), (s, v, want)
        checked += 1
    assert checked > 300


def test_parser_grammar_edges():
    # ParseFloat grammar (special, underscores, hex), ParseDuration units, ParseRate unicode
    assert O.parse_pct("1_0") == (True, 10.0)
    assert not O.parse_pct("_10")[0] and not O.parse_pct("1__0")[0] and not O.parse_pct("1_.5")[0]
    assert O.parse_pct("0x1p-2") == (True, 0.25) and not O.parse_pct("0x1")[0]
    assert not O.parse_pct("+nan")[0] and not O.parse_pct("infinity")[0] and not O.parse_pct("1e")[0]
    assert O.parse_pct("-0")[0] and O.parse_pct("-1e-50")[0] and not O.parse_pct("-1e-45")[0]
    assert O.parse_duration("1.5µs") == (True, 1) and O.parse_duration("2μs") == (True, 2)
    assert not O.parse_duration("10")[0] and not O.parse_duration("-5ms")[0]
    assert O.parse_duration("-0") == (True, 0) and O.parse_duration("1h30m") == (True, 5400000000 % 2**32)
    assert O.parse_rate(" 1gbit ") == (True, 10**9) and O.parse_rate("1İbit") == (True, 1)
    assert O.parse_rate("1Kbit") == (True, 1000)       # KELVIN SIGN lower-cases to 'k'
    assert O.parse_rate(" 1Mbit　") == (True, 10**6)
    assert not O.parse_rate("1 Mbit")[0] and not O.parse_rate("bit")[0]
    assert O.parse_rate("   ") == (True, 0)
    assert O.parse_rate("18446744073709551615bps") == (True, (2**64 - 1) * 8 % 2**64)
