"""GPU parity: libkdtn.so (HIP, gfx950) vs the CPU oracle, bit for bit, through the C-ABI.

Every output field of the epoch (actions, batch offsets and lists, resolve records,
qdisc structs) is compared byte-for-byte. Sizes are small enough for the oracle to finish
in seconds, except the full-size config-2 test which checks size-independent properties
plus an oracle-checked window of topologies.
"""
import random

import numpy as np
import pytest

import oracle as O
from helpers import (ACTIONS, golden_epoch, midpoint_strings, random_epoch_input,
                     random_float_strings, uids_by_topology, DURS, PCTS, RATES, IPS, MACS)
from kdtn import abi, synth
from kdtn.model import Link, LinkProperties, Topology, TopologyReconciler, make_qdiscs, pack
from kdtn.tables import Interner

pytestmark = pytest.mark.gpu
TICK = 15.625


def assert_same(eng_out, ora_out, ctx=""):
    bad = eng_out.mismatches(ora_out)
    if bad:
        f = bad[0]
        a, b = getattr(eng_out, f), getattr(ora_out, f)
        n = min(len(a), len(b))
        diff = [i for i in range(n) if a[i].tobytes() != b[i].tobytes()][:5]
        raise AssertionError(f"{ctx}: fields {bad} differ; {f} len {len(a)} vs {len(b)}; "
                             f"first idx {diff}: {[a[i] for i in diff]} vs {[b[i] for i in diff]}")


@pytest.mark.parametrize("idx", range(5))
def test_golden_transitions(engine, golden, idx):
    tr = golden["transitions"][idx]
    topos = golden_epoch(golden, tr)
    inp = pack(topos)
    out = engine.reconcile(inp)
    got = uids_by_topology(topos, out)
    for name, exp in tr["expect"].items():
        assert got[name]["action"] == ACTIONS[exp["action"]], (tr["name"], name)
        for k in ("del", "add", "upd"):
            assert got[name][k] == exp[k], (tr["name"], name, k)
    assert_same(out, O.reconcile(inp, tick=TICK), tr["name"])


def test_golden_qdisc_known_answers(engine, golden):
    props = [LinkProperties.from_dict(dict(c["props"])) for c in golden["qdisc"]]
    got = make_qdiscs(engine, props)
    for i, c in enumerate(golden["qdisc"]):
        want = O.make_qdisc(c["props"], TICK)
        assert got[i].tobytes() == want.tobytes(), c


@pytest.mark.parametrize("seed", range(24))
def test_random_epochs(engine, seed):
    topos, inp = random_epoch_input(seed, T=150)
    assert_same(engine.reconcile(inp), O.reconcile(inp, tick=TICK), f"seed {seed}")


def test_topologies_larger_than_lds_window(engine):
    # two hubs with > CAP (2048, kdtn_kernels.h) records on both sides → the global-scratch
    # path of k_reconcile's CalcDiff window,
    # plus a workgroup whose sum exceeds CAP through several mid-size topologies
    topos, inp = random_epoch_input(1234, T=140, big=2, p_err=0.05)
    assert max(inp.topos.real_off[1:] - inp.topos.real_off[:-1]) > 2000
    assert_same(engine.reconcile(inp), O.reconcile(inp, tick=TICK), "hubs")


def _props_batch(strings, field):
    pd = Interner()
    n = len(strings)
    prop = np.zeros((abi.NPROP, n), np.uint32)
    k = abi.PROP_COLS.index(field)
    for i, s in enumerate(strings):
        prop[k, i] = pd(s)
    return pd.table(), prop, np.zeros(n, np.uint32)


def test_hex_percentages_vs_oracle(engine):
    """Hexadecimal percentages around the float32 subnormal range (a negative value that rounds
    to -0 is accepted, one that rounds to a nonzero subnormal is an error), around 100 and with
    more than 16 digits (the sticky bit): GPU MakeQdiscs equals the oracle's, whose hexadecimal
    rounding is pinned by Go's atof32 table and exact rationals (tests/test_oracle_go_stdlib.py)."""
    rng = random.Random(23)
    strs = []
    for _ in range(3000):
        nd = rng.randint(1, 22)
        digs = "".join(rng.choice("0123456789abcdef") for _ in range(nd))
        if rng.random() < 0.3:
            digs = "1" + "0" * rng.randint(0, 20) + rng.choice(["", "1", "8", "80000000000000001"])
        cut = rng.randint(0, len(digs))
        mant = digs[:cut] + ("." if rng.random() < 0.6 else "") + digs[cut:]
        e = rng.choice([rng.randint(-200, -120), rng.randint(-4 * len(digs) - 160, -4 * len(digs) - 140),
                        rng.randint(-4 * len(digs) + 2, -4 * len(digs) + 12)])
        strs.append(f"{rng.choice(['', '-', '+'])}0x{mant}p{e}")
    pd, prop, gap = _props_batch(strs, "loss")
    got = engine.make_qdiscs(pd, prop, gap)
    for i, s in enumerate(strs):
        want = O.make_qdisc({"loss": s}, TICK)
        assert got[i].tobytes() == want.tobytes(), (s, got[i], want)


@pytest.mark.parametrize("field,pool", [("loss", "pct"), ("jitter", "dur"), ("rate", "rate"),
                                        ("latency", "dur"), ("reorder_prob", "pct")])
def test_parser_fuzz_vs_oracle(engine, field, pool):
    rng = random.Random(hash((field, pool)) & 0xFFFF)
    if pool == "pct":
        strs = PCTS + midpoint_strings(rng, 300) + random_float_strings(rng, 3000)
    elif pool == "dur":
        strs = DURS + [f"{rng.randint(0, 10**rng.randint(1, 19))}.{rng.randint(0, 10**rng.randint(1, 22))}"
                       f"{rng.choice(['ns', 'us', 'µs', 'ms', 's', 'm', 'h'])}" for _ in range(2000)]
        strs += ["".join(rng.choice("0123456789.nsuµmh+-") for _ in range(rng.randint(1, 10)))
                 for _ in range(2000)]
    else:
        strs = RATES + [f"{rng.choice([' ', '', chr(0xa0)])}{rng.randint(0, 10**rng.randint(1, 21))}"
                        f"{rng.choice(['', 'k', 'K', 'm', 'G', 't', 'T'])}{rng.choice(['', 'i', 'I'])}"
                        f"{rng.choice(['', 'bit', 'bps', 'BIT', 'Bps', 'b'])}{rng.choice(['', ' ', chr(0x3000)])}"
                        for _ in range(3000)]
    strs = list(dict.fromkeys(strs))
    pd, prop, gap = _props_batch(strs, field)
    got = engine.make_qdiscs(pd, prop, gap)
    for i, s in enumerate(strs):
        want = O.make_qdisc({field: s}, TICK)
        assert got[i].tobytes() == want.tobytes(), (field, s, got[i], want)


def test_cidr_mac_via_epoch(engine):
    rng = random.Random(5)
    ips = IPS + ["1.2.3.4/32", "255.255.255.255/0", "::/0", "::ffff:1.2.3.4/96", "1::2::3/64",
                 "1:2:3:4:5:6:7:8/128", "1:2:3:4:5:6:7:8:9/128", "::1.2.3.4/128", "1.2.3/24",
                 "01.2.3.4/8", "0.0.0.0/00", "1.2.3.4/", "/24", "1.2.3.4/3x"]
    macs = MACS + ["00:00:5e:00:53:01:02:03:04:05:06:07:08:09:0a:0b:0c:0d:0e:0f", "0000.5e00.5301.0203",
                   "00:00:5E:00:53:0G", "00:00:5e:00:53:01:", "000.05e00.5301"]
    links = []
    uid = 1
    for ip in ips:
        for mac in macs:
            links.append(Link("eth0", ip, mac, "eth1", rng.choice(ips), rng.choice(macs), "b", uid))
            uid += 1
    topos = [Topology("a", "default", links, [], "10.0.0.1", "/ns/a"),
             Topology("b", "default", [], [], "10.0.0.1", "/ns/b")]
    inp = pack(topos)
    out = engine.reconcile(inp)
    assert_same(out, O.reconcile(inp, tick=TICK), "cidr/mac")
    errs = set(out.add_res["err"].tolist())
    assert {0, abi.E_VETH_CIDR, abi.E_VETH_MAC, abi.E_PEER_VETH_CIDR} <= errs


def _mutate(rng: random.Random, s: str, alphabet: str) -> str:
    s = list(s)
    for _ in range(rng.randint(0, 3)):
        op = rng.randint(0, 2)
        k = rng.randint(0, len(s))
        if op == 0:
            s.insert(k, rng.choice(alphabet))
        elif op == 1 and s:
            del s[min(k, len(s) - 1)]
        elif s:
            s[min(k, len(s) - 1)] = rng.choice(alphabet)
    return "".join(s)


def test_key_predicates_fuzz(engine):
    """net.ParseCIDR / net.ParseMAC / localhost / physical/ predicates of key strings (the
    register fast path of k_kdict_flags and its generic fallback) against the oracle; long
    strings take the generic parsers."""
    rng = random.Random(11)
    ipa, maca = "0123456789./:", "0123456789abcdefABCDEFG:-."
    ips = [f"{rng.randint(0, 300)}.{rng.randint(0, 300)}.{rng.randint(0, 300)}.{rng.randint(0, 300)}"
           f"/{rng.choice(['', '0', '00', '032', '33', str(rng.randint(0, 40))])}" for _ in range(800)]
    ips += [_mutate(rng, rng.choice(ips), ipa) for _ in range(1500)]
    ips += ["".join(rng.choice(ipa) for _ in range(rng.randint(0, 30))) for _ in range(700)]
    ips += ["0" * 30 + "1.2.3.4/8", "1.2.3.4/" + "0" * 25 + "8", "255.255.255.255/32", "1.2.3.4/32x"]
    ips += ["1" * k + ".2.3.4/8" for k in (1500, 1800, 2100, 2400, 2700, 3000, 3300, 3600)]
    ips += ["localhost", "default", "physical/1.2.3.4"] + [f"10.{k}.0.1/24" for k in range(40)]
    # the byte-range classifier: bytes next to '.'..'9' (',' '-' ':' ';'), non-ASCII bytes whose
    # low 7 bits are '.' / '/' / digits (U+00AE, U+00AF, U+00B1), lengths around 18 / 19 / 24
    near = "0123456789./:-,;\u00ae\u00af\u00b1"
    ips += ["".join(rng.choice(near) for _ in range(rng.randint(1, 24))) for _ in range(600)]
    ips += [_mutate(rng, f"{rng.randint(0, 255)}.{rng.randint(0, 255)}.{rng.randint(0, 255)}."
                         f"{rng.randint(0, 255)}/{rng.randint(0, 32)}", near) for _ in range(600)]
    ips += ["::1/128", "1::/64", "fe80::1/64", "::ffff:1.2.3.4/96", "1.2.3.4/00000000032", "10.10.10.10/000032",
            "255.255.255.255/032", "255.255.255.255/3", "255.255.255.25/32", "1.2.3.4/\u00b2", "1.2.3.4\u00ae5/8",
            "1.2.3.4/8/", "1.2.3.4//8", "1..3.4/8", ".1.2.3/8", "1.2.3.4./8", "01.2.3.4/8", "1.2.3.04/8",
            "0.0.0.0/0", "1.2.3.256/8", "1.2.3.4/33", "1.2.3.4/-1", "123.123.123.123/12", "123.123.123.123/1"]
    macs = [":".join(f"{rng.randint(0, 255):02x}" for _ in range(rng.choice([6, 8, 20])))
            for _ in range(300)]
    macs += [_mutate(rng, rng.choice(macs), maca) for _ in range(700)]
    macs += ["".join(rng.choice(maca) for _ in range(rng.randint(10, 26))) for _ in range(300)]
    # the register (SWAR) form decides 17- and 23-byte ':' / '-' layouts: both separators,
    # mixed separators, upper case, non-hex and non-ASCII bytes in any position
    macs += [rng.choice(":-").join(f"{rng.randint(0, 255):02X}" for _ in range(rng.choice([6, 8])))
             for _ in range(200)]
    macs += [_mutate(rng, rng.choice(macs[-200:]), maca + "gG@`/\u00e9") for _ in range(400)]
    macs += ["aa:bb:cc:dd:ee:f\u00e9", "aa-bb-cc-dd-ee-ff", "aa-bb:cc-dd-ee-ff", "AA:BB:CC:DD:EE:FF:00:11",
             "aa:bb:cc:dd:ee:ff:00:1g", "0a:1b:2c:3d:4e:5f"]
    peers = ["b", "localhost", "localhos", "localhostx", "physical/10.0.0.9", "physical/", "physical",
             "Physical/1"]
    links = []
    uid = 1
    for ip in ips:
        links.append(Link("eth0", ip, "", "eth1", "", "", rng.choice(peers), uid))
        uid += 1
    for mac in macs:
        links.append(Link("eth0", "10.0.0.1/24", mac, "eth1", "", "", rng.choice(peers), uid))
        uid += 1
    topos = [Topology("a", "default", links, [], "10.0.0.1", "/ns/a"),
             Topology("b", "default", [], [], "10.0.0.2", "/ns/b")]
    inp = pack(topos)
    out = engine.reconcile(inp)
    assert_same(out, O.reconcile(inp, tick=TICK), "key predicates")
    errs = out.add_res["err"]
    assert (errs == abi.E_VETH_CIDR).sum() > 100 and (errs == abi.E_VETH_MAC).sum() > 100
    assert (errs == 0).sum() > 100


@pytest.mark.parametrize("cfg,pods", [(1, 0), (2, 20000), (3, 20000), (4, 5000)])
def test_synthetic_configs_small(engine, cfg, pods):
    inp = synth.make(cfg, pods_per_shard=pods) if pods else synth.make(cfg)
    out = engine.reconcile(inp)
    assert_same(out, O.reconcile(inp, tick=TICK), f"config {cfg}")
    if cfg == 1:
        assert len(out.upd_idx) == 100_000 and len(out.add_idx) == 0
    if cfg in (2, 4):
        assert len(out.add_idx) == inp.desired.n


def test_repeat_runs_are_identical(engine):
    inp = synth.make(3, pods_per_shard=20000)
    engine.upload(inp)
    engine.run()
    engine.sync()
    a = engine.download()
    engine.run()
    engine.sync()
    b = engine.download()
    assert not a.mismatches(b)


def test_reconciler_mirror_calc_diff(engine):
    a = Link("eth1", "1.1.1.1/24", "", "eth1", "", "", "p", 1)
    a2 = Link("eth1", "1.1.1.1/24", "", "eth1", "", "", "p", 1, LinkProperties(latency="5ms"))
    b = Link("eth2", "", "", "eth2", "", "", "p", 2)
    rec = TopologyReconciler(engine)
    add, dele, chg = rec.calc_diff([a, a], [a2, a])
    assert (add, dele, [l.uid for l in chg]) == ([], [], [1, 1])
    add, dele, chg = rec.calc_diff([a], [b, b])
    assert ([l.uid for l in add], [l.uid for l in dele], chg) == ([2, 2], [1], [])


def test_config2_full_size_properties(engine):
    """BASELINE config 2 at full size (1M pods, 10M links): size-independent properties
    plus a bit-exact check of every output field of every topology against the oracle
    (oracle.reconcile_parallel: disjoint topology ranges on the host's cores)."""
    inp = synth.make(2, pods_per_shard=1_000_000)
    out = engine.reconcile(inp)
    N, T = inp.desired.n, inp.topos.n
    assert N == 10_000_000 and T == 1_000_000
    assert len(out.add_idx) == N and len(out.del_idx) == 0 and len(out.upd_idx) == 0
    assert np.array_equal(out.add_idx, np.arange(N, dtype=np.uint32))      # spec order kept
    assert np.array_equal(out.add_off, inp.topos.des_off)
    assert (out.action == abi.ACT_DIFF).all()
    kinds = np.bincount(out.add_res["kind"], minlength=6)
    assert kinds[abi.KIND_CROSS_NODE] > 0.9 * N and kinds[abi.KIND_SAME_NODE] > 0
    assert (out.add_res["vni"] == (5000 + inp.desired.uid).astype(np.int32)).all()
    rate_err = (out.add_qdisc["err"] == abi.E_RATE).mean()
    assert 0.0002 < rate_err < 0.001
    ora = O.reconcile_parallel(inp, tick=TICK)
    bad = out.mismatches(ora)
    assert not bad, bad


def test_full_prefix_shortcut_boundaries(engine):
    """k_full_prefix: chunks before the first partial topology take their batch bases from
    the record offsets, later ones run the look-back. A CREATED topology (and one needing
    comparisons) in the middle of an all-AddLinks epoch moves that boundary."""
    inp = synth.make(2, pods_per_shard=20000)
    inp.topos.flags = inp.topos.flags.copy()
    inp.topos.flags[7001] |= abi.TOPO_STATUS_NIL            # CREATED: no entries
    inp.topos.flags[13000] |= abi.TOPO_SPEC_NIL if inp.topos.des_off[13001] == inp.topos.des_off[13000] else 0
    assert_same(engine.reconcile(inp), O.reconcile(inp, tick=TICK), "boundary")
    inp3 = synth.make(3, pods_per_shard=20000)               # churn: comparisons everywhere
    assert_same(engine.reconcile(inp3), O.reconcile(inp3, tick=TICK), "churn")


def _wire_same(engine, inp, ctx):
    engine.upload(inp)
    engine.run()
    engine.sync()
    out = engine.download()
    n = engine.encode()
    arena, off, err = engine.download_wire()
    # the oracle encodes the engine's own batches: this checks the encoding, the batches
    # themselves are checked against the oracle epoch by the other tests
    want_a, want_off, want_err = O.encode_epoch(inp, out)
    assert n == len(want_a), (ctx, n, len(want_a))
    assert np.array_equal(off, want_off), ctx
    assert np.array_equal(err, want_err.astype(np.uint32)), ctx
    assert arena.tobytes() == want_a.tobytes(), ctx
    return n


@pytest.mark.parametrize("seed", range(6))
def test_wire_encoding_random_epochs(engine, seed):
    """GPU proto.Marshal of every LinksBatchQuery (multi-byte and invalid UTF-8, 2-byte
    length varints, negative uids, large gaps) equals the oracle, which tests/test_wire_cpu.py
    pins to the Python protobuf runtime."""
    from helpers import wire_epoch_input
    topos, inp = wire_epoch_input(seed)
    assert _wire_same(engine, inp, f"seed {seed}") > 0


def test_wire_encoding_golden_and_synthetic(engine, golden):
    for tr in golden["transitions"]:
        _wire_same(engine, pack(golden_epoch(golden, tr)), tr["name"])
    for cfg, pods in ((1, 0), (2, 20000), (3, 20000), (4, 5000)):
        inp = synth.make(cfg, pods_per_shard=pods) if pods else synth.make(cfg)
        _wire_same(engine, inp, f"config {cfg}")


def test_diff_only_entry_point(engine):
    """kdtn_diff (gate + CalcDiff, no resolve/qdisc) gives the oracle's actions and lists."""
    topos, inp = random_epoch_input(21, T=150)
    got, want = engine.diff(inp), O.reconcile(inp, tick=TICK)
    for f in ("action", "del_off", "add_off", "upd_off", "del_idx", "add_idx", "upd_idx"):
        assert getattr(got, f).tobytes() == getattr(want, f).tobytes(), f


@pytest.mark.parametrize("seed", [4, 9])
def test_daemon_resolve_matches_epoch(engine, seed):
    """kdtn_resolve (one LinksBatchQuery against the informer's pods) plans every link as
    the full epoch does for a topology whose whole spec is added (status empty) or whose
    whole status is deleted (spec nil)."""
    from helpers import random_epoch
    from kdtn.model import pack as pack_topos
    topos, vnis = random_epoch(seed, T=120)
    for i in range(0, len(topos), 5):                       # fresh pods: status [] → all adds
        if topos[i].spec_links:
            topos[i].status_links = []
    for i in range(2, len(topos), 11):                      # deleted specs: all deletes
        if topos[i].status_links:
            topos[i].spec_links = None
    inp = pack_topos(topos, vnis)
    ref = O.reconcile(inp, tick=TICK)
    T = inp.topos
    checked = 0
    for t in range(T.n):
        if ref.action[t] != abi.ACT_DIFF:
            continue
        nr, nd = T.real_off[t + 1] - T.real_off[t], T.des_off[t + 1] - T.des_off[t]
        if nr == 0 and nd > 0:
            links = inp.desired.take(np.arange(T.des_off[t], T.des_off[t + 1]))
            res, q = engine.resolve(inp.kdict, inp.pdict, T, t, links, abi.BATCH_ADD, inp.vnis)
            a0, a1 = ref.add_off[t], ref.add_off[t + 1]
            assert res.tobytes() == ref.add_res[a0:a1].tobytes(), t
            assert q.tobytes() == ref.add_qdisc[a0:a1].tobytes(), t
            checked += 1
        elif nd == 0 and nr > 0 and T.flags[t] & abi.TOPO_SPEC_NIL:
            links = inp.realised.take(np.arange(T.real_off[t], T.real_off[t + 1]))
            res, _ = engine.resolve(inp.kdict, inp.pdict, T, t, links, abi.BATCH_DEL, inp.vnis)
            d0, d1 = ref.del_off[t], ref.del_off[t + 1]
            assert res.tobytes() == ref.del_res[d0:d1].tobytes(), t
            checked += 1
    assert checked >= 10


def test_kubedtn_batch_handlers(engine, golden):
    """KubeDTN.add_links / del_links / update_links on the sample triangle: kinds, VNIs and
    the first-error abort of the daemon handlers (handler.go:592-671)."""
    from kdtn.model import KubeDTN
    tr = golden["transitions"][1]
    topos = golden_epoch(golden, tr)
    d = KubeDTN(engine, topos, vxlan=[(topos[0].src_ip, 5001, "/other/ns")])
    r1 = topos[0]
    ok = d.add_links(r1.name, r1.namespace, r1.spec_links)
    assert ok.response and ok.first_failed == -1
    assert set(ok.plans["kind"].tolist()) <= {abi.KIND_SAME_NODE, abi.KIND_CROSS_NODE}
    assert (ok.plans["vni"] == [5000 + l.uid for l in r1.spec_links]).all()
    bad = [Link(**{**r1.spec_links[0].__dict__})] + [Link("eth9", "1.2.3.4", "", "eth9", "", "", "r2", 77)]
    res = d.add_links(r1.name, r1.namespace, bad)
    assert not res.response and res.first_failed == 1 and res.err == abi.E_VETH_CIDR
    ghost = [Link("eth8", "", "", "eth8", "", "", "nobody", 78)]
    assert d.add_links(r1.name, r1.namespace, ghost).err == abi.E_PEER_LOOKUP
    upd = d.update_links(r1.name, r1.namespace, [Link("eth1", "", "", "eth1", "", "", "r2", 1,
                                                       LinkProperties(rate="1.5Gbit"))])
    assert not upd.response and upd.err == abi.E_RATE
    dl = d.del_links(r1.name, r1.namespace, r1.spec_links)
    assert dl.response and dl.plans["vni_hit"].sum() == 0


def test_pod_names_shared_across_namespaces(engine):
    """getPod keys are (namespace, name) (handler.go:27-41): a name used in several
    namespaces, and a duplicate key (the informer's first object wins), go through the
    engine's overflow table; lookups from every namespace match the oracle."""
    rng = random.Random(8)
    nss = ["ns1", "ns2", "ns3", "default"]
    topos = []
    names = ["a", "b", "c"]
    for i in range(40):
        ns = nss[i % 4]
        name = names[i % 3] if i < 30 else f"u{i}"
        links = [Link(f"eth{k}", "", "", f"eth{k}", "", "", rng.choice(names + ["u31", "zz"]), 1000 * i + k,
                      LinkProperties(latency="1ms"))
                 for k in range(rng.randint(1, 4))]
        topos.append(Topology(name, ns, links, [], rng.choice(["10.0.0.1", "10.0.0.2", ""]),
                              rng.choice(["/run/ns/x", ""]) if i % 5 else "/run/ns/y"))
    topos.append(Topology("a", "", [Link("eth0", "", "", "eth0", "", "", "a", 99)], [], "10.0.0.1", "/n"))
    inp = pack(topos)
    out = engine.reconcile(inp)
    assert_same(out, O.reconcile(inp, tick=TICK), "shared names")
    kinds = set(out.add_res["kind"].tolist())
    assert abi.KIND_CROSS_NODE in kinds and (out.add_res["err"] == abi.E_PEER_LOOKUP).any()
    # repeated epochs on the same context (stamped table, no clearing) stay exact
    inp2 = pack(topos[5:])
    assert_same(engine.reconcile(inp2), O.reconcile(inp2, tick=TICK), "second epoch")
    assert_same(engine.reconcile(inp), O.reconcile(inp, tick=TICK), "third epoch")


def _fanout_same(engine, inp, ctx):
    out = engine.reconcile(inp)
    node, off, idx = engine.fanout()
    wn, wo, wi = O.fanout(O.reconcile(inp, tick=TICK), inp.topos.n)
    assert np.array_equal(node, wn) and np.array_equal(off, wo) and np.array_equal(idx, wi), ctx
    # every grouped entry is a CROSS_NODE add whose daemon is its peer's src_ip
    for k in range(len(node)):
        sel = idx[off[k]:off[k + 1]]
        assert (out.add_res["vtep"][sel] == node[k]).all()
        assert (out.add_res["kind"][sel] == abi.KIND_CROSS_NODE).all()
    return len(idx)


def test_remote_fanout_grouping(engine):
    """RemotePod RPCs grouped per destination daemon (with the batch-abort rule) equal the
    oracle's grouping on random epochs and the synthetic configs."""
    for seed in (1, 2, 3):
        topos, inp = random_epoch_input(seed, T=150, p_err=0.2)
        _fanout_same(engine, inp, f"seed {seed}")
    assert _fanout_same(engine, synth.make(2, pods_per_shard=20000), "config 2") > 100000
    assert _fanout_same(engine, synth.make(4, pods_per_shard=5000), "config 4") > 1000


def _remote_same(engine, inp, ctx, encode_first=False):
    out = engine.reconcile(inp)
    if encode_first:            # the run's wire encoding supplies the properties fields
        engine.encode()
    got = engine.remote_pods()
    want = O.remote_epoch(inp, O.reconcile(inp, tick=TICK))
    names = ("arena", "off", "entry", "n_remote", "tc", "tc_off")
    for name, g, w in zip(names, got, want):
        if name == "n_remote":
            assert g == w, (ctx, name)
        else:
            assert np.array_equal(np.asarray(g), np.asarray(w)), (ctx, name)
    return got[3], len(got[2]) - got[3]


def test_remote_pod_messages(engine):
    """RemotePod request bodies (UpdateRemote payloads in fan-out order, then the physical
    peers' local Updates) and the receiving daemons' tc argv, bit-exact against the oracle
    (pinned to the Python protobuf runtime, tests/test_wire_cpu.py) on adversarial random
    epochs (invalid UTF-8, negative uids / VNIs, 2-byte length varints) and configs 2 and 4."""
    from helpers import wire_epoch_input
    for seed in range(4):
        _remote_same(engine, wire_epoch_input(seed, T=120)[1], f"wire seed {seed}")
        _remote_same(engine, random_epoch_input(seed + 40, T=150, p_err=0.1)[1], f"seed {seed}")
    nr, _ = _remote_same(engine, synth.make(2, pods_per_shard=20000), "config 2")
    assert nr > 100000
    nr, nph = _remote_same(engine, synth.make(4, pods_per_shard=5000), "config 4")
    assert nr > 1000 and nph > 0


def test_remote_pod_messages_after_wire_encoding(engine):
    """The same with the run's wire encoding done first: each message's properties field is
    copied from its AddLinks entry's Link bytes, except in batches that failed to marshal
    (invalid UTF-8: those messages take their strings), bit-exact against the oracle."""
    from helpers import wire_epoch_input
    for seed in range(4):
        _remote_same(engine, wire_epoch_input(seed, T=120)[1], f"wire seed {seed}", encode_first=True)
        _remote_same(engine, random_epoch_input(seed + 40, T=150, p_err=0.1)[1], f"seed {seed}", encode_first=True)
    nr, _ = _remote_same(engine, synth.make(2, pods_per_shard=20000), "config 2", encode_first=True)
    assert nr > 100000
    nr, nph = _remote_same(engine, synth.make(4, pods_per_shard=5000), "config 4", encode_first=True)
    assert nr > 1000 and nph > 0


def test_tc_argv_synthesis(engine):
    """`tc qdisc add ... tbf` argv per AddLinks / UpdateLinks entry (common/qdisc.go:252-266)
    equals the oracle's on random epochs and the synthetic configs."""
    cases = [random_epoch_input(s, T=150)[1] for s in (5, 6)]
    cases += [synth.make(1), synth.make(2, pods_per_shard=20000), synth.make(3, pods_per_shard=20000)]
    for k, inp in enumerate(cases):
        out = engine.reconcile(inp)
        arena, off = engine.tc_argv(len(out.add_idx), len(out.upd_idx))
        wa, wo = O.tc_epoch(inp, O.reconcile(inp, tick=TICK))
        assert np.array_equal(off, wo), k
        assert arena.tobytes() == wa.tobytes(), k


def test_reach_rule_scenario_and_error_heavy_epochs(engine):
    """Batch-abort rule across the DelLinks → AddLinks → UpdateLinks RPC sequence, remote
    rejection of a RemotePod (peer_ip without a mask) and both veth ends of a same-node pair:
    fan-out and tc argv equal the oracle on a hand-built scenario and on error-heavy random
    epochs; resolve records carry remote_err exactly as the oracle."""
    from test_reach_cpu import scenario
    cases = [pack(scenario())] + [random_epoch_input(s, T=150, p_err=0.4)[1] for s in (31, 32, 33)]
    for k, inp in enumerate(cases):
        ora = O.reconcile(inp, tick=TICK)
        out = engine.reconcile(inp)
        assert_same(out, ora, f"case {k}")
        node, off, idx = engine.fanout()
        wn, wo, wi = O.fanout(ora, inp.topos.n)
        assert np.array_equal(node, wn) and np.array_equal(off, wo) and np.array_equal(idx, wi), k
        arena, toff = engine.tc_argv(len(out.add_idx), len(out.upd_idx))
        wa, wto = O.tc_epoch(inp, ora)
        assert np.array_equal(toff, wto) and arena.tobytes() == wa.tobytes(), k
    assert (ora.add_res["remote_err"] == abi.E_REMOTE_CIDR).any()


def test_append_only_dictionaries_keep_parsed_tables(engine):
    """kdtn_epoch_in.kdict_keep / pdict_keep: consecutive epochs whose interners only grow
    upload and parse only the new strings; the outputs equal a fresh full upload's and the
    oracle's. A later upload that keeps a shorter prefix (strings after it replaced,
    "localhost" / "default" moved) recomputes them; keeping more than was parsed fails."""
    from kdtn.abi import EINVAL
    from kdtn.engine import KdtnError
    kd, pd = Interner(), Interner()
    prev = None
    for seed in (41, 42, 43):
        topos, vnis = __import__("helpers").random_epoch(seed, T=120)
        inp = pack(topos, vnis, kdict=kd, pdict=pd)
        keep = (prev.kdict.n, prev.pdict.n) if prev is not None else (0, 0)
        engine.upload(inp, *keep)
        engine.run()
        engine.sync()
        got = engine.download()
        assert_same(got, O.reconcile(inp, tick=TICK), f"keep seed {seed}")
        prev = inp
    with pytest.raises(KdtnError) as e:                      # more than the parsed prefix
        engine.upload(prev, prev.kdict.n + 1, 0)
    assert e.value.code == EINVAL
    # a shorter kept prefix, then strings that differ from the previous suffix
    topos, vnis = __import__("helpers").random_epoch(44, T=80)
    kd2, pd2 = Interner(), Interner()
    for i in range(min(40, len(kd) - 1)):
        kd2(prev.kdict.get(i + 1))
    for i in range(min(10, len(pd) - 1)):
        pd2(prev.pdict.get(i + 1))
    kd2("zz-new"), kd2("localhost"), kd2("default")
    inp = pack(topos, vnis, kdict=kd2, pdict=pd2)
    engine.upload(inp, 41, 11)
    engine.run()
    engine.sync()
    assert_same(engine.download(), O.reconcile(inp, tick=TICK), "shorter prefix")


def test_timer_totals_sum_the_synced_epochs(engine):
    """kdtn_timer_totals: the HIP-event marks of every synced epoch since the last reset, per
    stage (bench.py reads them once per timed loop); equal to the per-epoch marks summed."""
    _, inp = random_epoch_input(5, T=400)
    engine.upload(inp)
    engine.set_timing(1)
    try:
        engine.timer_totals(reset=True)
        per = []
        for _ in range(3):
            engine.run()
            engine.sync()
            per.append(engine.kernel_times())
        tot = engine.timer_totals(reset=True)
        assert set(tot) == set(per[0]) and "reconcile" in tot, (tot, per[0])
        for k, (ms, n) in tot.items():
            assert n == 3, (k, n)
            assert abs(ms - sum(p[k] for p in per)) <= 1e-3 * max(ms, 1e-3), (k, ms, per)
        assert engine.timer_totals() == {}                # reset cleared them
    finally:
        engine.set_timing(2)                              # the context's default


def test_download_into_page_locked_buffers(engine):
    """kdtn_epoch_download / _async into page-locked buffers (the SDMA engine copies them)
    equal the copies into pageable memory, every field; a second epoch reuses the buffers."""
    from kdtn.tables import BatchesOut
    for seed in (3, 4):
        topos, inp = random_epoch_input(seed, T=150)
        engine.upload(inp)
        engine.run()
        engine.sync()
        plain = engine.download()
        cap = max(inp.realised.n, inp.desired.n, 1)
        pinned = BatchesOut.alloc(inp.topos.n, cap, cap, cap, pinned=True)
        assert_same(engine.download(into=pinned), plain, f"seed {seed}: sync download")
        again = BatchesOut.alloc(inp.topos.n, cap, cap, cap, pinned=True)
        view = engine.download_async(again)
        engine.download_wait()
        assert_same(view, plain, f"seed {seed}: async download")
        assert_same(plain, O.reconcile(inp, tick=TICK), f"seed {seed}")


def _loaded_hip_runtime():
    """The HIP runtime this process already loaded (torch's or ROCm's), for hipHostRegister."""
    import ctypes
    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
    assert paths, "no HIP runtime mapped"
    return ctypes.CDLL(sorted(paths)[0])


def test_download_into_registered_host_memory(engine):
    """destinations registered with hipHostRegister (LOCKED pointers) reach the SDMA
    engine through their agent address; every field equals the pageable download."""
    import ctypes
    import mmap
    from kdtn.tables import BatchesOut
    hip = _loaded_hip_runtime()
    topos, inp = random_epoch_input(7, T=150)
    engine.upload(inp)
    engine.run()
    engine.sync()
    plain = engine.download()
    cap = max(inp.realised.n, inp.desired.n, 1)
    shapes = BatchesOut.alloc(inp.topos.n, cap, cap, cap)
    maps, regs, arrays = [], [], []
    try:
        for a in vars(shapes).values():
            n = max(a.nbytes, 1)
            m = mmap.mmap(-1, (n + 4095) // 4096 * 4096)
            maps.append(m)
            arr = np.frombuffer(m, dtype=np.uint8, count=a.nbytes).view(a.dtype).reshape(a.shape)
            addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
            assert hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(len(m)), 0) == 0
            regs.append(addr)
            arrays.append(arr)
        into = BatchesOut(*arrays)
        assert_same(engine.download(into=into), plain, "registered: sync download")
        for a in arrays:
            a[...] = 0
        view = engine.download_async(into)
        engine.download_wait()
        assert_same(view, plain, "registered: async download")
    finally:
        for addr in regs:
            hip.hipHostUnregister(ctypes.c_void_p(addr))
        del arrays


def test_output_stages_without_sync_use_this_runs_counts(engine):
    """an output stage called after kdtn_epoch_run without kdtn_epoch_sync reads this
    run's list totals (counts_fresh), not the previous epoch's: a large epoch is synced, then a
    small one is only run, and its download and wire encoding equal the small epoch's."""
    _, big = random_epoch_input(11, T=400)
    _, small = random_epoch_input(12, T=60)
    engine.upload(small)
    engine.run()
    engine.sync()
    want = engine.download()
    n_want = engine.encode()
    wire_want = engine.download_wire()
    engine.upload(big)
    engine.run()
    engine.sync()
    engine.upload(small)
    engine.run()                                          # no sync before the stages
    assert engine.encode() == n_want
    for a, b in zip(engine.download_wire(), wire_want):
        np.testing.assert_array_equal(a, b)
    engine.upload(big)
    engine.run()
    engine.sync()
    engine.upload(small)
    engine.run()
    assert_same(engine.download(), want, "download without sync")


def test_go_stdlib_vectors_on_the_gpu(engine):
    """Go's published known answers (tests/test_oracle_go_stdlib.py: time parseDurationTests,
    strconv atof32tests / atoftests / parseUint64Tests, net parseCIDRTests / parseIPTests /
    parseMACTests)
    through the GPU parsers: a duration as a link's latency (MakeQdiscs, E_LATENCY iff Go rejects
    it or it is negative), a float as its loss (E_LOSS iff ParseFloatPercentage rejects it), an
    integer as its rate (E_RATE iff ParseUint rejects it), a CIDR as local_ip (MakeVeth,
    E_VETH_CIDR iff invalid and non-empty), a MAC as local_mac (E_VETH_MAC iff invalid); every
    output also equals the oracle's."""
    from test_oracle_go_stdlib import (GO_CIDRS, GO_DURATION_ERRORS, GO_DURATIONS, GO_MACS, GO_PARSE_IP_CIDRS,
                                       GO_PARSE_UINT64, GO_PCT_INPUTS, GO_TRIMSPACE_RATES, _latin1_or_utf8,
                                       go_percentage)
    strs = [s for s, _ in GO_DURATIONS] + GO_DURATION_ERRORS
    pd, prop, gap = _props_batch(strs, "latency")
    got = engine.make_qdiscs(pd, prop, gap)
    for i, s in enumerate(strs):
        want = O.make_qdisc({"latency": s}, TICK)
        assert got[i].tobytes() == want.tobytes(), (s, got[i], want)
        ok = i < len(GO_DURATIONS) and GO_DURATIONS[i][1] >= 0
        assert (got[i]["err"] == 0) == ok and (ok or got[i]["err"] == abi.E_LATENCY), (s, got[i]["err"])
    pd, prop, gap = _props_batch(GO_PCT_INPUTS, "loss")
    got = engine.make_qdiscs(pd, prop, gap)
    for i, s in enumerate(GO_PCT_INPUTS):
        want = O.make_qdisc({"loss": s}, TICK)
        assert got[i].tobytes() == want.tobytes(), (s[:40], got[i], want)
        ok = go_percentage(s) is not None
        assert (got[i]["err"] == 0) == ok and (ok or got[i]["err"] == abi.E_LOSS), (s[:40], got[i]["err"])
    rates = GO_PARSE_UINT64 + [(_latin1_or_utf8(s), v) for s, v in GO_TRIMSPACE_RATES]
    strs = [s for s, _ in rates]
    pd, prop, gap = _props_batch(strs, "rate")
    got = engine.make_qdiscs(pd, prop, gap)
    for i, (s, v) in enumerate(rates):
        want = O.make_qdisc({"rate": s}, TICK)
        assert got[i].tobytes() == want.tobytes(), (s, got[i], want)
        assert (got[i]["err"] == 0) == (v is not None) and (v is not None or got[i]["err"] == abi.E_RATE), s
    links, want_err = [], []
    uid = 1
    for ip, valid in GO_CIDRS + GO_PARSE_IP_CIDRS:      # MakeVeth parses a non-empty IP only (veth.go:21)
        links.append(Link("eth0", ip, "00:00:5e:00:53:01", "eth1", "", "", "b", uid))
        want_err.append(0 if valid or ip == "" else abi.E_VETH_CIDR)
        uid += 1
    for mac, valid in GO_MACS:
        links.append(Link("eth0", "10.0.0.1/24", mac, "eth1", "", "", "b", uid))
        want_err.append(0 if valid else abi.E_VETH_MAC)
        uid += 1
    topos = [Topology("a", "default", links, [], "10.0.0.1", "/ns/a"),
             Topology("b", "default", [], [], "10.0.0.2", "/ns/b")]
    inp = pack(topos)
    out = engine.reconcile(inp)
    assert_same(out, O.reconcile(inp, tick=TICK), "Go stdlib vectors")
    errs = out.add_res["err"][np.argsort(out.add_idx)]
    assert errs.tolist() == want_err
